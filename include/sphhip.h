/* sphhip.h — C ABI of libsphhip.so, the MI355X (gfx950) particle step.
 *
 * This is the drop-in boundary for the reference's per-frame GPU path. The reference
 * drives its HLSL kernels through Unity's engine API from ParticleSystemController
 * (/root/reference/Assets/Scripts/ParticleSystemController.cs); each entry point below
 * names the reference call site(s) it replaces. Conventions:
 *   - extern "C", cdecl, blittable structs (every field 4 bytes: C# Pack=4 works as is);
 *   - return 0 (SPH_OK) or a negative sph_status; no exception crosses the ABI;
 *     sph_last_error() holds the message of the last failure on that context;
 *   - the library owns device memory, the caller owns every host array;
 *   - one context per thread, not thread-safe (the reference is single-threaded:
 *     Unity main thread);
 *   - particle arrays passed in or out are in PARTICLE INDEX order (the index the
 *     reference uses for particleBuffer[i]); the device keeps them cell-sorted internally.
 */
#ifndef SPHHIP_H
#define SPHHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPH_ABI_VERSION 2

typedef struct sph_ctx sph_ctx;

typedef enum sph_status {
    SPH_OK = 0,
    SPH_ERR_INVALID = -1,   /* bad argument / out-of-range count */
    SPH_ERR_HIP = -2,       /* HIP runtime failure (no device, launch error, …) */
    SPH_ERR_CAPACITY = -3,  /* count > capacity; resize first */
    SPH_ERR_STATE = -4,     /* call not valid for this model / not initialised */
    SPH_ERR_NOMEM = -5
} sph_status;

typedef enum sph_model {
    SPH_MODEL_CONTACT = 0,  /* Model R: SimulateParticles.compute:211-408 (SPEC_SPH.md §1) */
    SPH_MODEL_WCSPH = 1     /* Model S: weakly-compressible SPH (SPEC_SPH.md §2) */
} sph_model;

#define SPH_FLAG_PROFILE 1  /* time every kernel launch with HIP events (sph_get_kernel_stat) */
#define SPH_FLAG_VALIDATE 2 /* multi-GPU step: wait after every step and check every slab's device sizes */

/* replaces: new ComputeBuffer(particleCount, 84) … (ParticleSystemController.cs:373-388) */
typedef struct sph_config {
    int32_t model;          /* sph_model */
    int32_t dim;            /* 2 or 3 (Model R: 3) */
    int32_t capacity;       /* particleCount (ParticleSystemController.cs:12); ndev > 1: per-GPU minimum */
    int32_t flags;          /* SPH_FLAG_* */
    int32_t ndev;           /* GPUs this context drives (0 or 1: one). ndev > 1 (Model S): the domain is
                               cut into x-slabs over devices device, device+1, ... (modulo the visible
                               count), one slab context per GPU, halos moved by device-to-device copies
                               over xGMI; sph_init_scenario / sph_step / sph_read_* work as for one GPU */
} sph_config;

/* replaces: computeShader.SetFloat/SetInt uniforms (ParticleSystemController.cs:255-263,
 * 496-508; SimulateParticles.compute:89-100) plus the Model S constants of SPEC_SPH.md §2. */
typedef struct sph_params {
    /* --- Model R uniforms (reference names) --- */
    float spawn_radius;                       /* spawnRadius */
    float min_radius, max_radius;             /* minRadius, maxRadius */
    float global_drag_multiplier;             /* globalDragMultiplier */
    float torque_factor;                      /* torqueFactor */
    float torque_damping;                     /* torqueDamping */
    float boundary_friction;                  /* boundaryFriction */
    float rolling_contact_radius_multiplier;  /* rollingContactRadiusMultiplier */
    float density;                            /* density */
    float repulsion_strength;                 /* repulsionStrength */
    int32_t active_particle_count;            /* activeParticleCount */
    /* --- Model S --- */
    float dx, h, rho0, c0, alpha, xsph_eps;
    float gravity[3];
    float box[3];                              /* tank extent; walls at 0 and box[a] */
    float wall_restitution;
    float forcing_amp, forcing_freq;           /* f_ext = (amp·sin(2π f t), 0, 0) */
} sph_params;

typedef enum sph_scenario_kind {
    SPH_SCENARIO_DAMBREAK = 0,  /* fluid column at the tank's low-x corner */
    SPH_SCENARIO_SLOSHING = 1,  /* fluid layer filling the tank floor + lateral forcing */
    SPH_SCENARIO_SPHERE = 2     /* Model R: sph_init_scenario with nx = count initialises all nx
                                   particles as InitParticles does (= sph_init_particles(nx, nx, 0, 0)) */
} sph_scenario_kind;

typedef struct sph_scenario {
    int32_t kind;               /* sph_scenario_kind */
    int32_t dim;
    int32_t nx, ny, nz;         /* fluid lattice (particles per axis) */
    int32_t tx, ty, tz;         /* tank extent in units of dx */
    float dx;
    uint32_t seed;
    float jitter;               /* lattice jitter amplitude in units of dx (0.01) */
} sph_scenario;

/* replaces: DragInput (ParticleSystemController.cs:149-154; compute:70-74), 20 bytes */
typedef struct sph_drag_input {
    int32_t selected_id;
    float target[3];
    float strength;
} sph_drag_input;

typedef struct sph_stats {
    int64_t steps;              /* steps taken since create / last upload */
    double sim_time;            /* Σ dt */
    int32_t active;             /* active particle count */
    int32_t capacity;
    int32_t grid[3];            /* cells per axis */
    int32_t key_bits;           /* radix-sort key width */
    int64_t device_bytes;       /* device memory held by the context */
} sph_stats;

typedef struct sph_kernel_stat {
    char name[32];
    int64_t launches;
    double total_ms;            /* Σ HIP-event durations (SPH_FLAG_PROFILE only) */
    double bytes_per_launch;    /* algorithmic HBM bytes of the last launch */
    int64_t timed;              /* launches that carried events: total_ms / timed is the mean duration */
} sph_kernel_stat;

/* ---- lifetime: replaces InitializeBuffers / ReleaseBuffers (controller:373-482) ---- */
int sph_create(const sph_config* cfg, int32_t device, sph_ctx** out);
void sph_destroy(sph_ctx* ctx);
/* replaces ResizeParticleBuffers (controller:1162-1222): keeps the active particles */
int sph_resize(sph_ctx* ctx, int32_t capacity);
const char* sph_last_error(const sph_ctx* ctx);
int32_t sph_abi_version(void);

/* Run the step on a caller-provided HIP stream (hipStream_t as void*; NULL = own stream). */
int sph_set_stream(sph_ctx* ctx, void* hip_stream);
int sph_get_stream(sph_ctx* ctx, void** hip_stream);

/* ---- configuration: replaces SetFloat/SetInt (controller:255-263, 496-508) ---- */
int sph_set_params(sph_ctx* ctx, const sph_params* params);
int sph_get_params(const sph_ctx* ctx, sph_params* params);
/* Derive the SPEC_SPH.md §2 constants (h, c0, box, forcing …) for a scenario. Pure; no ctx. */
int sph_scenario_params(const sph_scenario* sc, sph_params* out, float* dt_out);

/* ---- particle data: replaces particleBuffer.SetData/GetData (controller:519-522,794,959)
 *      and InitParticles (compute:118-194, controller:484-552) ---- */
int sph_upload_particles_aos84(sph_ctx* ctx, const void* src, int32_t count);
int sph_download_particles_aos84(sph_ctx* ctx, void* dst, int32_t count);
int sph_upload_state(sph_ctx* ctx, const float* pos_xyz, const float* vel_xyz, int32_t count);
int sph_init_scenario(sph_ctx* ctx, const sph_scenario* sc);

/* ---- Model R particle lifecycle ---- */
/* replaces: InitParticles (compute:118-194) dispatched by InitializeParticles
 * (controller:484-512). `count` particles (the buffer length, <= capacity); the first `active`
 * are initialised by the reference's hash RNG from the current params (spawnRadius, min/maxRadius,
 * density), the rest are zero as a fresh ComputeBuffer. genome_modes / default_mode are the
 * reference's genomeModesCount / defaultGenomeMode (compute:64-68; 0 = no genome, modeIndex -1).
 * Sets active_particle_count = active. */
int sph_init_particles(sph_ctx* ctx, int32_t count, int32_t active, int32_t genome_modes,
                       int32_t default_mode);

/* CellSplitData (controller:136-147), 92 bytes */
typedef struct sph_split {
    int32_t parent_index;
    float position_a[3], position_b[3];
    float velocity_a[3], velocity_b[3];
    float rotation_a[4], rotation_b[4];   /* x, y, z, w */
    int32_t child_a_mode, child_b_mode;
} sph_split;

/* replaces: the buffer half of ProcessPendingSplits (controller:780-959): per split, child A
 * overwrites the parent's position/velocity/rotation/modeIndex, child B is a copy of child A at
 * index active+k with its own position/velocity/rotation/modeIndex; then active += count.
 * Grows the capacity on the device when needed to max(active+count, 2·capacity) (:788-792) and the
 * particle count to at least active+count. Parents must be distinct and < active.
 * *active_out (optional) receives the new activeParticleCount. No host round trip of the
 * particle buffer (the reference reads and rewrites all of it, :793-794, :959). */
int sph_split_particles(sph_ctx* ctx, const sph_split* splits, int32_t count, int32_t* active_out);

/* replaces: particleBuffer.GetData / SetData (array, 0, first, count) on a particle index range
 * (controller:519-522, 535, 691, 736). 84-byte records, Model R only. */
int sph_get_particles_aos84(sph_ctx* ctx, int32_t first, int32_t count, void* dst);
int sph_set_particles_aos84(sph_ctx* ctx, int32_t first, int32_t count, const void* src);

/* ---- the per-frame step: replaces the Dispatch sequence of Update()
 *      (controller:265-331: torque clear, ClearGrid, BuildHashGrid, ApplySPHForces,
 *       ApplyDragForce, UpdateMotion, UpdateRotation) ---- */
int sph_step(sph_ctx* ctx, float dt, int32_t nsteps);
/* the simulated time t (Σ dt; Time.time in the reference's frame loop) the next step starts at: the
 * sloshing forcing f_ext(t) reads it. Uploads and scenario inits reset it to 0; this sets it after an
 * upload, e.g. to resume a saved state. Not for ndev > 1 groups. */
int sph_set_sim_time(sph_ctx* ctx, double t);
/* replaces HandleMouseDrag → dragInputBuffer.SetData (controller:975-1034) */
int sph_set_drag(sph_ctx* ctx, const sph_drag_input* drag);
/* replaces: adhesionConnectionBuffer.SetData + the ApplyAdhesionConstraints /
 * ApplyAdhesionDeltas dispatches (controller:285-310; compute:424-607). `conn84` holds `count`
 * 84-byte AdhesionConnection records (compute:43-55, CellAdhesionManager.cs:511-524) whose
 * particleA/B are particle indices. The bonds persist: every later sph_step applies them
 * (Model R only) until the next call; count 0 removes them. The caller applies its own cap
 * (the reference's maxAdhesionConnections, controller:129,287). */
int sph_set_adhesion(sph_ctx* ctx, const void* conn84, int32_t count);
/* the last step's per-bond fixed-point terms (×1e6), 16 int32 per bond:
 * Δv_A(x,y,z,0), Δv_B(x,y,z,0), Δq_A(x,y,z,w), Δq_B(x,y,z,w) — what each bond's thread adds
 * with InterlockedAdd in the reference (compute:451-456, 509-512, 536-539, 568-581). */
int sph_read_adhesion_terms(sph_ctx* ctx, int32_t* terms16, int32_t count);

/* ---- readback: replaces Copy*ToReadbackBuffer + GetData (compute:410-422,
 *      controller:327-333) and AsyncGPUReadback (controller:1115-1159) ---- */
int sph_read_positions(sph_ctx* ctx, float* xyz, int32_t count);
int sph_read_rotations(sph_ctx* ctx, float* xyzw, int32_t count);
int sph_read_velocities(sph_ctx* ctx, float* xyz, int32_t count);
int sph_read_angular_velocities(sph_ctx* ctx, float* xyz, int32_t count);
int sph_read_density(sph_ctx* ctx, float* rho, int32_t count);   /* Model S, pass-1 ρ */
int sph_read_pressure_term(sph_ctx* ctx, float* prho, int32_t count);   /* Model S, pass-1 P/ρ² */
int sph_synchronize(sph_ctx* ctx);

/* replaces: AsyncGPUReadback.Request(buffer, callback) + r.GetData<T>() (controller:1115-1159).
 * request: the chosen fields of the CURRENT state (particle index order) are copied on the device
 * and sent to pinned host memory on a side stream; the caller keeps stepping meanwhile. One
 * request is outstanding per context: a new one replaces an unread one. status: SPH_OK when the
 * data is on the host, SPH_READBACK_PENDING while in flight (the callback's "done" test).
 * get: waits if needed, then copies `field` (one flag) into dst (count >= sph_readback_count). */
#define SPH_READBACK_POSITIONS 1    /* float xyz  (positionReadbackBuffer, compute:410-415) */
#define SPH_READBACK_ROTATIONS 2    /* float xyzw (rotationReadbackBuffer, compute:417-422), Model R */
#define SPH_READBACK_PARTICLES 4    /* 84-byte Particle (particleBuffer), Model R */
#define SPH_READBACK_PENDING 1
int sph_request_readback(sph_ctx* ctx, int32_t fields);
int sph_readback_status(sph_ctx* ctx);
int sph_readback_get(sph_ctx* ctx, int32_t field, void* dst, int32_t count);
int sph_readback_count(sph_ctx* ctx, int32_t* count);

/* ---- render interop: replaces sphereMaterial.SetBuffer("particleBuffer") + the indirect-args
 * update (controller:335-347; InstancedParticles.shader:27-47 reads the 84-byte records) ----
 * export: the particles as 84-byte records in index order into a caller DEVICE buffer (e.g. the
 * renderer's structured buffer), enqueued on the context stream (sph_get_stream), no host copy.
 * draw args: args[1] (instanceCount of a 5-uint DrawMeshInstancedIndirect buffer in device memory)
 * = activeParticleCount, enqueued on the context stream. */
int sph_export_aos84_device(sph_ctx* ctx, void* dev_dst, int32_t count);
int sph_write_draw_args(sph_ctx* ctx, void* dev_args);

/* ---- introspection (tests / bench) ---- */
int sph_get_stats(sph_ctx* ctx, sph_stats* out);
int sph_get_kernel_stat(sph_ctx* ctx, int32_t index, sph_kernel_stat* out);
int sph_reset_kernel_stats(sph_ctx* ctx);
/* SPH_FLAG_PROFILE: time the launches of one step in `every` (default 1; the events cost the step
 * ~15 us at C3, so a bench samples); the other steps launch without events */
int sph_set_profile_every(sph_ctx* ctx, int32_t every);
/* sorted-slot views of the last step (slot order = cell order) */
int sph_read_sorted_ids(sph_ctx* ctx, int32_t* ids, int32_t count);
int sph_read_cell_start(sph_ctx* ctx, uint32_t* cell_start, int32_t count);
int sph_read_torque_int(sph_ctx* ctx, int32_t* xyz, int32_t count);  /* Model R, index order */
/* Model S neighbour passes: how often a workgroup left the LDS-staged fast path since the last
 * reset (sparse or splashing regions): [0] density planes processed row by row in chunks, [1] density
 * rows gathered straight from global memory, [2] / [3] the same for the force pass. reset != 0
 * zeroes them after the read. The passes count only after the first call of this function or of
 * sph_read_hit_mask_counts on the context (counting costs atomics on one address). */
int sph_read_path_counts(sph_ctx* ctx, uint32_t counts[4], int32_t reset);
/* Model S pass 2 takes its hits from pass 1's hit mask (8 words = 256 candidates per target):
 * [0] wave-planes (one wave, one dx plane) that scanned by distance instead, because a lane's
 * candidates passed the mask, or no valid mask exists (a force pass without a density pass since the
 * last change of the slot order), [1] waves run (3 planes each).
 * reset != 0 zeroes them after the read. */
int sph_read_hit_mask_counts(sph_ctx* ctx, uint32_t counts[2], int32_t reset);
/* The incremental re-sort's path counters since the last reset (both models; always counted, no cost on the
 * fast path): [0] key/slot ranges that counted against the whole mover list (slow: O(slots x movers); 0 in
 * every measured scene), [1] lanes whose insertion slot lay below the staged slot window (a whole-list count
 * each), [2] ranges whose dest entries overflowed LDS and ran in passes over key sub-intervals (a dam-break
 * front entering empty columns), [3] their passes, [4] the largest dest-entry count of one range (recorded
 * above a quarter of the LDS capacity; maximum, not sum, over a group), [5] cell shares whose mover keys
 * overflowed LDS (one stream of the mover list per pass instead of one in all), [6..7] 0. reset != 0 zeroes them
 * after the read. Replaces no Unity call (the reference rebuilds its grid every frame, compute:196-209). */
int sph_read_resort_counts(sph_ctx* ctx, uint32_t counts[8], int32_t reset);
/* Model S: particles whose cell key changed in the last step (the movers the next incremental re-sort
 * places; 0 with SPH_RESORT=0). Waits for the context's stream. */
int sph_read_mover_count(sph_ctx* ctx, uint32_t* movers);
/* stable LSD radix sort of (key, index) on the device: the sort of the step, exposed for
 * bit-exact parity tests. perm[i] = source index of sorted slot i. */
int sph_debug_radix_sort(sph_ctx* ctx, const uint32_t* keys, int32_t count, int32_t key_bits,
                         uint32_t* perm_out, uint32_t* sorted_keys_out);
/* Test hook, Model S: add dv to the velocity of particle `id` between steps, in every context of a
 * group that holds it (tests/test_gpu_multi.py: a particle made to cross several slab columns in one
 * step, the decomposition's column-jump fallback and its window-exit stop). Not a Unity call.
 * On an RCCL rank every rank calls it between the same two steps (the next step then re-packs its
 * halo messages instead of using the ones sent during the last step, on every rank alike). */
int sph_debug_kick(sph_ctx* ctx, int32_t id, const float dv[3]);

/* ---- slab decomposition (multi-GPU; SPEC_SPH.md §3). New capability: the reference is one
 *      GPU. One context per rank owns global cell columns [cx_lo, cx_hi)
 *      plus one halo column per side. The HOST moves the packed device buffers between ranks
 *      (RCCL over xGMI: sph_test_amd.slab / bench.py). Per step:
 *        count_sends(_async) → pack_send(0/1) → [exchange] → assemble → density → ranges →
 *        pack_rho(0/1) → [exchange] → force(interior) ∥ [rho in flight] → unpack_rho → force(boundary)
 *        → finish_step.
 *      Particle records are 32 bytes: (x, y, z, id-bits, u, v, w, old-key-bits): the particle's
 *      sorted key before this step as a global cell key (0xffffffff: none), which lets the
 *      receiver re-sort incrementally. assemble reads the received records in place on the
 *      context stream: keep dev_left / dev_right intact until that stream has passed it. ---- */
typedef struct sph_slab {
    int32_t cx_lo, cx_hi;       /* owned columns of the global grid; neighbours exist iff
                                   cx_lo > 0 / cx_hi < columns */
} sph_slab;
#define SPH_SLAB_RECORD_BYTES 32
/* ranges[]: ghost-left [0,1), owned [2,3), ghost-right [4,5), boundary column cx_lo [6,7),
 * boundary column cx_hi-1 [8,9), all as sorted-slot index ranges [begin, end). */
int sph_slab_set(sph_ctx* ctx, const sph_slab* slab);
/* re-balancing (between steps): the owned particles per GLOBAL column (zero outside the owned
 * columns; ncols >= the grid's columns), and a new owned range that keeps the particles: the next
 * step's exchange sends the columns that changed owner (move each cut by at most one column). */
int sph_slab_column_counts(sph_ctx* ctx, int64_t* counts, int32_t ncols);
int sph_slab_recut(sph_ctx* ctx, const sph_slab* slab);
int sph_slab_init_scenario(sph_ctx* ctx, const sph_scenario* sc);
int sph_slab_count_sends(sph_ctx* ctx, int32_t counts[2]);
/* the same counts written to DEVICE memory (int64[2]: left, right) without a host sync; the
 * host sends them to the neighbours as they are. pack_send then needs capacity >= the owned
 * count (sph_slab_send_capacity) instead of the exact count. */
int sph_slab_count_sends_async(sph_ctx* ctx, int64_t* dev_counts);
int sph_slab_send_capacity(sph_ctx* ctx, int32_t* capacity);
int sph_slab_pack_send(sph_ctx* ctx, int32_t side, void* dev_records, int32_t capacity);
int sph_slab_assemble(sph_ctx* ctx, const void* dev_left, int32_t n_left, const void* dev_right,
                      int32_t n_right);
/* assemble reads the ranges back asynchronously; sph_slab_ranges waits for that copy (and so
 * does every call below that needs them, except density, which reads them on the device).
 * Calling density before ranges keeps the GPU busy while the host waits. */
int sph_slab_ranges(sph_ctx* ctx, int32_t ranges[10]);
int sph_slab_density(sph_ctx* ctx);
int sph_slab_pack_rho(sph_ctx* ctx, int32_t side, void* dev_rho_prho, int32_t capacity);
int sph_slab_unpack_rho(sph_ctx* ctx, int32_t side, const void* dev_rho_prho, int32_t count);
int sph_slab_force(sph_ctx* ctx, float dt, int32_t part);   /* 0 all, 1 interior, 2 boundary */
int sph_slab_finish_step(sph_ctx* ctx, float dt);
/* owned particles as 8-float records (x, y, z, u, v, w, id-bits, ρ); count >= owned */
int sph_slab_read_owned(sph_ctx* ctx, float* records, int32_t count, int32_t* n_owned);

/* ---- the multi-GPU step inside the library (SPEC_SPH.md §3). A multi-GPU
 *      context (sph_config.ndev > 1, or one context per process joined by sph_comm_init) runs the
 *      whole decomposed step in sph_step: migration + x,v halo, incremental re-sort across the halo,
 *      density, ρ halo overlapped with the interior force pass, boundary force pass, and the
 *      re-balancing of the cuts every sph_set_rebalance steps. Every per-step size stays on the device
 *      (message headers; no host read per step): halo messages have capacities both neighbours derive
 *      from the counts of two steps before; an overflow is detected on the device and reported by a
 *      later sph_step as SPH_ERR_CAPACITY. ---- */
typedef struct sph_comm_id {
    char internal[128];         /* an RCCL unique id (ncclUniqueId) */
} sph_comm_id;
/* rank 0 creates the id; the host hands the 128 bytes to every rank (any channel) */
int sph_comm_unique_id(sph_comm_id* out);
/* one process per GPU: this context is rank `rank` of `nranks`, exchanging over RCCL (xGMI). Model S,
 * before sph_init_scenario, which then keeps this rank's slab of the scenario (equal-count cuts). */
int sph_comm_init(sph_ctx* ctx, const sph_comm_id* id, int32_t nranks, int32_t rank);
/* re-balancing interval of the multi-GPU step in steps (default 50; 0: off) */
int sph_set_rebalance(sph_ctx* ctx, int32_t every);
/* the decomposition: this process's rank and the world size, its (first local) slab, the particles
 * it owns (ndev > 1: all of them), and the global particle count */
typedef struct sph_decomp {
    int32_t rank, world, local_ranks;
    sph_slab cut;
    int64_t owned, total;
    int32_t rebalances;
} sph_decomp;
int sph_get_decomposition(sph_ctx* ctx, sph_decomp* out);

#ifdef __cplusplus
}
#endif
#endif /* SPHHIP_H */
