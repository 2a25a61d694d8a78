/* oracle.h — CPU restatement of the step (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product (sph-test_amd/libsphhip.so) never links or calls it.
 *
 * Model R follows /root/reference/Assets/Compute/SimulateParticles.compute:102-408
 * line by line (Jacobi semantics, gather-form reaction torque: SPEC_SPH.md §1).
 * Model S follows SPEC_SPH.md §2 (no reference source exists for it: SURVEY.md §0).
 *
 * PARITY UNPINNED by reference fixtures: the reference has no tests, golden vectors or
 * CPU path, and its HLSL cannot be compiled or run here (no dxc/fxc/Unity/dotnet;
 * SURVEY.md §4, §8c). The restatement is pinned instead by hand-derived known-answer
 * cases (tests/test_oracle_kat.py) and by committed fixtures (tests/golden/).
 */
#ifndef SPH_ORACLE_H
#define SPH_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- common grid (SPEC_SPH.md §0) ---- */
typedef struct {
    float origin[3];
    float inv_cell;     /* x, y */
    float inv_cell_z;   /* z sub-cells: cell / zsub */
    int32_t G[3];       /* G[2] counts z sub-cells */
    int32_t zwin;       /* neighbour z window in sub-cells (zsub + 1) */
    int32_t xsub;       /* x sub-columns per column: keys count sub-columns (SPEC_SPH.md §0) */
    float inv_cxs;      /* xsub / cell (exact) */
} or_grid;

uint32_t or_cell_key(const or_grid* g, float x, float y, float z);
void or_keys(const or_grid* g, int n, const float* pos3, uint32_t* keys);
/* stable counting sort by key; perm[i] = source slot of sorted slot i */
void or_stable_sort(int n, const uint32_t* keys, uint32_t nkeys, uint32_t* perm);
/* cell_start[k] = first sorted index with key >= k, k = 0..nkeys */
void or_cell_start(int n, const uint32_t* sorted_keys, uint32_t nkeys, uint32_t* cell_start);

/* ---- Model S (SPEC_SPH.md §2) ---- */
typedef struct {
    int32_t dim;
    float dx, h, rho0, c0, alpha, eps_xsph;
    float g[3];
    float L[3];
    float wall_e;
    float f_amp, f_freq;
    /* derived by or_sph_derive */
    float mass, B, sigma, inv_h, four_h2;
    or_grid grid;
} or_sph_params;

void or_sph_derive(or_sph_params* p);
/* One step. Arrays are permuted in place into this step's sorted order.
 * rho/prho (optional) receive pass-1 results in that order; cell_start (optional, C+1). */
int or_sph_step(const or_sph_params* p, int n, float* pos3, float* vel3, int32_t* id,
                float dt, float t, float* rho, float* prho, uint32_t* cell_start,
                int nthreads);
/* or_sph_step plus diagnostics in the sorted order (each optional): acc3 = the pair sum
 * a_i = -Σ m(Pρ_i + Pρ_j + Π_ij)F(r)x_ij (no gravity / forcing); mag5 = the error scales the GPU parity
 * tests normalise by: Σ m|F|r(|Pρ_i| + |Pρ_j| + |Π_ij|) (the acceleration terms before they cancel),
 * Σ|pair XSPH term|, and Σ m|F|r(E_i + E_j) with E = (B/ρ²)(5(ρ/ρ0)^7 + 2) (the acceleration's change
 * per unit relative error of the densities: the stiff Tait EOS amplifies pass-1 rounding); then the two support-edge
 * conditioning terms OR_DIAG_DQ bounds: Σ_{q>=1} 2·m|F|r(|Pρ_i| + |Pρ_j| + |Π_ij|)·δq/(2 − q) and
 * Σ_{q>=1} 3|pair XSPH term|·δq/(2 − q). For q >= 1 a pair's F·r is ∝ (2 − q)² and its W ∝ (2 − q)³, so two
 * evaluations whose q differ by δq (r² by an fma chain or by plain products, r by rsq or sqrt: a few ulp of q) differ
 * in the term by 2δq/(2 − q), 3δq/(2 − q) of it, which grows without bound at the support edge.
 * mag5 holds five floats per particle. */
#define OR_DIAG_DQ (1.0 / 2097152.0) /* δq = 2^-21: four ulp of q in [1, 2) */
int or_sph_step_diag(const or_sph_params* p, int n, float* pos3, float* vel3, int32_t* id, float dt, float t,
                     float* rho, float* prho, uint32_t* cell_start, float* acc3, float* mag5, int nthreads);
/* Phases of or_sph_step over sorted arrays (sk = sorted keys, cs = cell start), used by the
 * slab-decomposition tests: targets [i0, i1); neighbours may be any sorted slot (ghosts). */
void or_sph_density_range(const or_sph_params* p, const float* pos3, const uint32_t* sk, const uint32_t* cs,
                          int i0, int i1, float* rho, float* prho, int nthreads);
void or_sph_force_range(const or_sph_params* p, const float* pos3, const float* vel3, const float* rho,
                        const float* prho, const uint32_t* sk, const uint32_t* cs, int i0, int i1, float dt,
                        float t, float* pos_out, float* vel_out, int nthreads);
/* or_sph_force_range with the diagnostics of or_sph_step_diag (acc3, mag5 at the target's slot) */
void or_sph_force_range_diag(const or_sph_params* p, const float* pos3, const float* vel3, const float* rho,
                             const float* prho, const uint32_t* sk, const uint32_t* cs, int i0, int i1, float dt,
                             float t, float* pos_out, float* vel_out, float* acc3, float* mag5, int nthreads);
/* Dam-break lattice init (SPEC_SPH.md; the same integer hash as the device init). */
void or_sph_lattice(int dim, int nx, int ny, int nz, float dx, float x0, float y0, float z0,
                    uint32_t seed, float jitter, float* pos3);

/* ---- Model R (SPEC_SPH.md §1) ---- */
typedef struct {
    float position[3]; float radius;
    float velocity[3]; float mass;
    float angularVelocity[3]; float momentOfInertia;
    float drag; float repulsionStrength; float padding1; float padding2;
    float rotation[4];
    int32_t modeIndex;
} or_particle84;   /* SimulateParticles.compute:23-40, 84 bytes */

typedef struct {
    float dt, spawn_radius, global_drag, torque_factor, torque_damping, boundary_friction,
          roll_mult, repulsion_strength;
    int32_t drag_id;            /* DragInput.selectedID (compute:70-74), -1 = none */
    float drag_target[3];
    float drag_strength;
} or_contact_params;

/* One step on n active particles (AoS, in/out). torque_int (optional, n*3) receives the
 * per-particle int torque sums that UpdateRotation consumed. */
int or_contact_step(const or_contact_params* p, int n, or_particle84* parts, int32_t* torque_int,
                    int nthreads);

/* AdhesionConnection (compute:43-55; CellAdhesionManager.cs:511-524), 84 bytes */
typedef struct {
    int32_t particleA, particleB;
    float restLength, springStiffness, springDamping;
    float connectionColor[4];
    float initialRelOrientation[4];
    float anchorLocalPosA[3];
    float anchorLocalPosB[3];
    float anchorConstraintStiffness;
    int32_t enableAnchorConstraint;
} or_adhesion84;

/* The same step with nconn adhesion bonds applied between ApplySPHForces and the drag
 * (controller:284-310; compute:424-607). terms (optional, 16*nconn int32) receives what each
 * bond's thread adds: Δv_A(x,y,z,0), Δv_B(x,y,z,0), Δq_A(xyzw), Δq_B(xyzw), fixed point ×1e6. */
int or_contact_step_bonds(const or_contact_params* p, int n, or_particle84* parts, int32_t* torque_int,
                          const or_adhesion84* conns, int nconn, int32_t* terms, int nthreads);

/* InitParticles (compute:118-194): n records, the first `active` initialised, the rest zero */
void or_init_particles(int n, int active, float spawn_radius, float min_radius, float max_radius, float density,
                       int genome_modes, int default_mode, or_particle84* out);

/* CellSplitData (ParticleSystemController.cs:136-147), 92 bytes */
typedef struct {
    int32_t parent;
    float posA[3], posB[3], velA[3], velB[3], rotA[4], rotB[4];
    int32_t modeA, modeB;
} or_split92;
/* ProcessPendingSplits' buffer edit (:832-959): returns the new active count */
int or_split_particles(or_particle84* parts, int active, const or_split92* splits, int count);

#ifdef __cplusplus
}
#endif
#endif
