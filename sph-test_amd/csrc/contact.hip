// contact.hip — Model R: the reference's soft-sphere contact step (SPEC_SPH.md §1), gfx950.
//
// One fused kernel replaces five of the reference's dispatches per frame:
//   ApplySPHForces (SimulateParticles.compute:211-309), ApplyDragForce (:311-324),
//   UpdateMotion (:326-357), UpdateRotation (:379-408) and the torqueAccumBuffer clear
//   (ParticleSystemController.cs:265).
// With adhesion bonds the reference runs its two bond kernels between ApplySPHForces and the
// drag (controller:284-310), so the frame splits in three: k_contact_forces, the bond pass
// (adhesion.hip), k_contact_finish.
// Jacobi semantics: all reads come from the start-of-step arrays, all writes go to the
// *_o arrays. The reaction torque the reference scatters with three InterlockedAdds per
// contact (compute:291-294) is gathered instead: particle a sums the truncated int3 terms b's
// thread would scatter into it. int32 addition is associative, so the sum is bit-identical to the
// atomic one, with no atomics and no ordering dependence. b's term needs no second evaluation of the
// pair body from b's side: that evaluation's torqueB equals a's own torqueA bit for bit up to the
// sign of zero components (below, reaction_equals_own), which the truncation to int removes.
// Every rounding is the one written (no fused multiply-adds), as in the oracle: with the double-evaluated
// intrinsics (vec3.h) the Model R step is bit-identical to oracle/contact_oracle.c.
#pragma clang fp contract(off)
#ifdef SPH_CONTACT_PROBE
namespace sph { extern __device__ uint64_t g_ct_probe[]; }
#define FZ_PROBE(slot) \
    do { if (threadIdx.x == 0 && blockIdx.x < 256) sph::g_ct_probe[blockIdx.x * 32 + (slot)] = wall_clock64(); } while (0)
#endif
#include "bonds.h"
#include "common.h"
#include "fused_perm.h"
#include "vec3.h"

namespace sph {

constexpr int CT_BLK = 256;
constexpr float TORQUE_SCALE = 10000.0f;   // compute:19

struct Body { f3 pos, vel, omg; float r; };

// ApplySPHForces' pair body (compute:248-295) from `self`'s thread.
// hit: 0 none, 1 repulsion only, 2 repulsion + rolling friction.
__device__ __forceinline__ int contact_pair(const ContactConst& c, const Body& A, const Body& B,
                                            f3& force, f3& torqueA, f3& torqueB) {
    const float effectiveRadiusA = A.r * 0.5f;
    const float effectiveRadiusB = B.r * 0.5f;
    const f3 delta = A.pos - B.pos;
    const float dist = len(delta);
    const float overlap = (effectiveRadiusA + effectiveRadiusB) - dist;
    if (!(overlap > 0.001f)) return 0;
    const f3 dir = delta / dist;
    const float overlapFalloff = saturate(overlap / (effectiveRadiusA + effectiveRadiusB));
    const float falloff = saturate(1.0f - dist / (effectiveRadiusA + effectiveRadiusB));
    force = dir * falloff * c.repulsion_strength * overlapFalloff;
    const f3 contactPointA = A.pos - dir * effectiveRadiusA;
    const f3 contactPointB = B.pos + dir * effectiveRadiusB;
    const f3 surfaceVelA = A.vel + cross(A.omg, contactPointA - A.pos);
    const f3 surfaceVelB = B.vel + cross(B.omg, contactPointB - B.pos);
    const f3 relSurfaceVel = surfaceVelA - surfaceVelB;
    const f3 tangentVel = relSurfaceVel - dir * dot(relSurfaceVel, dir);
    const float slipSpeed = len(tangentVel);
    if (!(slipSpeed > 1e-4f)) return 1;
    const f3 frictionDir = tangentVel / slipSpeed;
    const float torqueInput = fabsf(slipSpeed * c.torque_factor);
    float frictionMag = pow125_r(torqueInput);   // pow(x, 1.25) :279
    frictionMag = fminf(frictionMag, 10.0f);
    const float torqueRadiusScale = overlapFalloff * overlapFalloff;   // pow(x, 2.0) :282
    const float effectiveRadiusTorqueA = torqueRadiusScale * effectiveRadiusA * c.roll_mult;
    const float effectiveRadiusTorqueB = torqueRadiusScale * effectiveRadiusB * c.roll_mult;
    torqueA = cross(-dir * effectiveRadiusTorqueA, -frictionDir * frictionMag);
    torqueB = cross(dir * effectiveRadiusTorqueB, frictionDir * frictionMag);
    return 2;
}
// reaction_equals_own: b's thread evaluates contact_pair(c, B, A) and scatters its torqueB into a (compute:291-294).
// Every quantity of that evaluation is the one of contact_pair(c, A, B), exactly or negated exactly, because IEEE
// subtraction, multiplication, division and sqrt are sign-symmetric and + is commutative, with no contraction
// (fp contract off): delta' = -delta, dist' = dist, the same overlap, falloffs and contact points, dir' = -dir,
// relSurfaceVel' = -relSurfaceVel, dot(rel', dir') = dot(rel, dir), tangentVel' = -tangentVel, the same slipSpeed
// (so the same hit code), frictionDir' = -frictionDir, the same frictionMag, and effectiveRadiusTorqueB' is the
// expression of effectiveRadiusTorqueA. So torqueB' = cross(-dir * eRTA, -frictionDir * frictionMag) = torqueA, with
// at most the sign of a zero component differing (b - a = +0 where -(a - b) = -0), and ftoi(+-0) = 0. The oracle
// evaluates both sides; the Model R bit-exact tests compare the int torque sums.

// Cell skipping (r6). The reference scans the 27 cells of 4.0 around a target (compute:228-233), and a contact needs
// dist < (rA + rB)/2 − 0.001 (:251-253). With every radius at most rmax (ContactConst::rmax), a cell whose nearest
// point lies farther than rA/2 + rmax/2 holds no contact: the pass drops such rows ((x, y) cells) and each row's end z
// cells. The candidates that remain keep their order (rows in order, slots increasing), so every sum equals the
// oracle's bit for bit (the oracle scans all 27). Per axis, in cell units from the coordinate cell_coord rounds
// (g = (x − o)/cell, cell c): a lower neighbour cell lies more than f = g − c below the target, an upper one more than
// 1 − f above (f is only larger, or 1 − f only larger, for a target clamped into an edge cell). The bound keeps a
// margin (1.001·reach + 0.001) far above the rounding of g. An rmax not yet known (+inf), negative or NaN radii, or a
// NaN coordinate skip nothing. At the rate table's sphere (radii 1.5-2, rmax 2) a target keeps ~8 of its 27 cells.
struct CellReach {
    float fx, fy, fz, r2;   // r2: the squared bound in cell units (+inf: no skipping)
};
// ContactConst::rmv from the device word (a contact kernel's first statement, so the load joins its first round trip)
__device__ __forceinline__ void rmax_load(ContactConst& c) {
    c.rmv = c.rmax ? __uint_as_float(ld_vec(c.rmax)) : __builtin_inff();
}
__device__ __forceinline__ CellReach cell_reach(const GridDesc& g, const ContactConst& c, float4 pa, int32_t cx, int32_t cy,
                                                int32_t cz) {
    CellReach q;
    q.fx = (pa.x - g.ox) * g.inv_cell - (float)cx;
    q.fy = (pa.y - g.oy) * g.inv_cell - (float)cy;
    q.fz = (pa.z - g.oz) * g.inv_cz - (float)cz;
    const float reach = 0.5f * pa.w + 0.5f * c.rmv;
    const float b = (reach * 1.001f + 0.001f) * g.inv_cell;
    q.r2 = (reach >= 0.0f && reach < 1e30f && g.inv_cell == g.inv_cz) ? b * b : __builtin_inff();
    return q;
}
// Row (dx, dy): false when its (x, y) cells lie beyond reach, else its z cells [z0, z1] (of [cz − 1, cz + 1]) in reach
__device__ __forceinline__ bool reach_row(const CellReach& q, int dx, int dy, int32_t cz, int32_t gz, int32_t& z0,
                                          int32_t& z1) {
    const float lx = dx < 0 ? q.fx : (dx > 0 ? 1.0f - q.fx : 0.0f);
    const float ly = dy < 0 ? q.fy : (dy > 0 ? 1.0f - q.fy : 0.0f);
    const float l2 = lx * lx + ly * ly, ua = q.fz, ub = 1.0f - q.fz;
    if (l2 > q.r2) return false;
    z0 = cz > 0 && !(l2 + ua * ua > q.r2) ? cz - 1 : cz;
    z1 = cz < gz - 1 && !(l2 + ub * ub > q.r2) ? cz + 1 : cz;
    return true;
}

// ApplySPHForces' neighbour loop (compute:228-300) for slot a, then its integration
// (:302-306): v1 = v + F/m·dt, w1 = ω + T/I·dt, and the int reaction torque sums.
__device__ __forceinline__ void contact_accumulate(const float4* __restrict__ pos, const float4* __restrict__ vel,
                                                   const float4* __restrict__ omg, const uint32_t* __restrict__ cs,
                                                   const GridDesc& g, const ContactConst& c, int32_t a, float4 pa,
                                                   float4 va, float4 wa, f3& v, f3& w, uint32_t tq[3]) {
    const Body A{xyz(pa), xyz(va), xyz(wa), pa.w};
    const float dt = c.dt;
    f3 totalForce = mk(0, 0, 0), totalTorque = mk(0, 0, 0);
    tq[0] = tq[1] = tq[2] = 0u;   // wrapping int32 sums (InterlockedAdd)
    const int32_t cx = cell_cx(g, pa.x);
    const int32_t cy = cell_coord(pa.y, g.oy, g.inv_cell, g.gy);
    const int32_t cz = cell_coord(pa.z, g.oz, g.inv_cz, g.gz);
    const CellReach cr = cell_reach(g, c, pa, cx, cy, cz);
#pragma unroll 1
    for (int k = 0; k < 9; ++k) {
        const int32_t xx = cx + k / 3 - 1, yy = cy + k % 3 - 1;
        int32_t z0, z1;
        if (xx < 0 || xx >= g.gx || yy < 0 || yy >= g.gy || !reach_row(cr, k / 3 - 1, k % 3 - 1, cz, g.gz, z0, z1))
            continue;
        const uint32_t rowk = ((uint32_t)xx * (uint32_t)g.gy + (uint32_t)yy) * (uint32_t)g.gz;
        const uint32_t j0 = cs[rowk + (uint32_t)z0], j1 = cs[rowk + (uint32_t)z1 + 1u];
#pragma unroll 1
        for (uint32_t j = j0; j < j1; ++j) {
            if ((int32_t)j == a) continue;                                   // :240
            const float4 pb = pos[j];
            const f3 d = A.pos - xyz(pb);
            const float reff = A.r * 0.5f + pb.w * 0.5f;
            if (!(reff - len(d) > 0.001f)) continue;                         // :253 (cheap reject)
            const float4 vb = vel[j], wb = omg[j];
            const Body B{xyz(pb), xyz(vb), xyz(wb), pb.w};
            f3 F, TA, TB;
            const int hit = contact_pair(c, A, B, F, TA, TB);
            if (hit == 0) continue;
            totalForce = add_exact(totalForce, F);                           // :261
            if (hit == 2) {
                totalTorque = add_exact(totalTorque, TA);                    // :289
                const f3 sc = TA * dt * TORQUE_SCALE;                        // b's scatter into a, :291
                tq[0] += (uint32_t)ftoi(sc.x);
                tq[1] += (uint32_t)ftoi(sc.y);
                tq[2] += (uint32_t)ftoi(sc.z);
            }
        }
    }
    v = A.vel + (totalForce / va.w) * dt;                                    // :302-306
    w = A.omg + (totalTorque / wa.w) * dt;
}

// Team form of contact_accumulate: T lanes (T | 64) share target a and take the candidates of a
// row T at a time, lane t taking j = base + t. That gives T times more lanes in flight at the
// reference's scale (a few thousand dense particles, hundreds of candidates each), where one lane
// per target leaves the chip idle and serialises every candidate load.
// The float totals keep the serial order bit for bit: the team walks its hit mask lowest lane first
// and every lane adds the hit lane's F and TA, which is exactly contact_accumulate's order
// (rows k in order, j increasing; adding TA = +0 for a repulsion-only hit changes nothing since
// the total starts at +0 and can never become −0). The int torque is a wrapping sum, so the
// team reduces it in any order. Every team lane returns the same v, w, tq.
template <int T>
__device__ __forceinline__ void contact_accumulate_team(const float4* __restrict__ pos,
                                                        const float4* __restrict__ vel,
                                                        const float4* __restrict__ omg,
                                                        const uint32_t* __restrict__ cs, const GridDesc& g,
                                                        const ContactConst& c, int32_t a, float4 pa, float4 va,
                                                        float4 wa, f3& v, f3& w, uint32_t tq[3]) {
    static_assert(T == 16 || T == 64, "team size (lanes 0..8 fetch the rows)");
    const int lane = (int)(threadIdx.x & 63u);
    const int t = lane & (T - 1);
    const int team0 = lane & ~(T - 1);
    const Body A{xyz(pa), xyz(va), xyz(wa), pa.w};
    const float dt = c.dt;
    f3 totalForce = mk(0, 0, 0), totalTorque = mk(0, 0, 0);
    uint32_t q0 = 0u, q1 = 0u, q2 = 0u;
    const int32_t cx = cell_cx(g, pa.x);
    const int32_t cy = cell_coord(pa.y, g.oy, g.inv_cell, g.gy);
    const int32_t cz = cell_coord(pa.z, g.oz, g.inv_cz, g.gz);
    const CellReach cr = cell_reach(g, c, pa, cx, cy, cz);
    // lanes 0..8 of the team fetch the nine row ranges at once; rows are read back by shuffle
    uint32_t rj0 = 0u, rj1 = 0u;
    if (t < 9) {
        const int32_t xx = cx + t / 3 - 1, yy = cy + t % 3 - 1;
        int32_t z0, z1;
        if (xx >= 0 && xx < g.gx && yy >= 0 && yy < g.gy && reach_row(cr, t / 3 - 1, t % 3 - 1, cz, g.gz, z0, z1)) {
            const uint32_t rowk = ((uint32_t)xx * (uint32_t)g.gy + (uint32_t)yy) * (uint32_t)g.gz;
            rj0 = cs[rowk + (uint32_t)z0];
            rj1 = cs[rowk + (uint32_t)z1 + 1u];
        }
    }
#pragma unroll 1
    for (int k = 0; k < 9; ++k) {
        const uint32_t j0 = (uint32_t)__shfl((int)rj0, k, T), j1 = (uint32_t)__shfl((int)rj1, k, T);
#pragma unroll 1
        for (uint32_t base = j0; base < j1; base += T) {
            const uint32_t j = base + (uint32_t)t;
            f3 F = mk(0, 0, 0), TA = mk(0, 0, 0);
            bool hit = false;
            if (j < j1 && (int32_t)j != a) {                                   // :240
                const float4 pb = pos[j];
                const f3 d = A.pos - xyz(pb);
                const float reff = A.r * 0.5f + pb.w * 0.5f;
                if (reff - len(d) > 0.001f) {                                   // :253 (cheap reject)
                    const float4 vb = vel[j], wb = omg[j];
                    const Body B{xyz(pb), xyz(vb), xyz(wb), pb.w};
                    f3 TB;
                    const int h = contact_pair(c, A, B, F, TA, TB);
                    hit = h != 0;
                    if (h == 2) {                                               // b's scatter into a, :291
                        const f3 sc = TA * dt * TORQUE_SCALE;
                        q0 += (uint32_t)ftoi(sc.x);
                        q1 += (uint32_t)ftoi(sc.y);
                        q2 += (uint32_t)ftoi(sc.z);
                    }
                    if (h != 2) TA = mk(0, 0, 0);
                    if (h == 0) F = mk(0, 0, 0);
                }
            }
            // this team's hits, lowest lane (= lowest j) first
            uint64_t m = (__ballot(hit) >> team0);
            if (T < 64) m &= (1ull << T) - 1ull;
            while (m) {
                const int src = __builtin_ctzll(m);
                m &= m - 1ull;
                totalForce = add_exact(totalForce, mk(__shfl(F.x, src, T), __shfl(F.y, src, T), __shfl(F.z, src, T)));
                totalTorque =
                    add_exact(totalTorque, mk(__shfl(TA.x, src, T), __shfl(TA.y, src, T), __shfl(TA.z, src, T)));
            }
        }
    }
#pragma unroll
    for (int o = T / 2; o > 0; o >>= 1) {
        q0 += (uint32_t)__shfl_xor((int)q0, o, T);
        q1 += (uint32_t)__shfl_xor((int)q1, o, T);
        q2 += (uint32_t)__shfl_xor((int)q2, o, T);
    }
    tq[0] = q0; tq[1] = q1; tq[2] = q2;
    v = A.vel + (totalForce / va.w) * dt;                                    // :302-306
    w = A.omg + (totalTorque / wa.w) * dt;
}

// Flat form (team code CT_FLAT): one wave per target over the target's candidates flattened across the nine rows
// (candidate f = row k's j = rj0_k + f − P_k, P the rows' exclusive length prefix), for the reference's scale where a
// target has ~100-800 candidates in up to 9 rows: the team form walks the rows one after another, a dependent global
// load of positions, then of the touching candidates' velocities, per row. Here one round prefetches the positions of
// CF_CHUNKS x 64 candidates and finds the touching ones (the reject test of :253, the same expressions); the touching
// candidates are then compacted over the wave's lanes in flattened order (chunk-major, lane-minor: rows in order and j
// increasing within a row, the serial order) through a per-wave LDS list, and each batch of 64 evaluates its pair
// bodies on all lanes and adds the hits' F and TA in list order: the serial order, bit for bit. r5 gave each lane its
// own touching candidates (up to three slots), so a round took as many body passes as its busiest lane touched
// candidates: 3.9 passes per wave at the rate table's 32,768-particle sphere against 1.85 compacted
// (scripts/contact_scene_stats.py), at ~280 VALU per pass.
constexpr int CT_FLAT = 65;
constexpr int CF_CHUNKS = 8;
constexpr int CF_WAVES = 16;   // waves per workgroup of k_contact_fused (1,024 lanes)
// The slot arrays as the contact pass reads them: cell starts and the slot holding sorted position j. DirectMap: the
// arrays are in sorted order (after the re-sort); FusedMap (below): the previous step's order, read through this
// step's permutation (the one-launch step at the reference's scale).
struct DirectMap {
    const uint32_t* cs;
    __device__ __forceinline__ uint32_t start(uint32_t k) const { return cs[k]; }
    __device__ __forceinline__ uint32_t old(uint32_t j) const { return j; }
};
template <int WAVES, class Map>
__device__ __forceinline__ void contact_accumulate_flat(const float4* __restrict__ pos, const float4* __restrict__ vel,
                                                        const float4* __restrict__ omg, const Map& M,
                                                        const GridDesc& g, const ContactConst& c, int32_t a, float4 pa,
                                                        float4 va, float4 wa, f3& v, f3& w, uint32_t tq[3]) {
    const int lane = (int)(threadIdx.x & 63u);
    const Body A{xyz(pa), xyz(va), xyz(wa), pa.w};
    const float dt = c.dt;
    f3 totalForce = mk(0, 0, 0), totalTorque = mk(0, 0, 0);
    uint32_t q0 = 0u, q1 = 0u, q2 = 0u;
    const int32_t cx = cell_cx(g, pa.x);
    const int32_t cy = cell_coord(pa.y, g.oy, g.inv_cell, g.gy);
    const int32_t cz = cell_coord(pa.z, g.oz, g.inv_cz, g.gz);
    const CellReach cr = cell_reach(g, c, pa, cx, cy, cz);
    uint32_t rj0 = 0u, rlen = 0u;
    if (lane < 9) {
        const int32_t xx = cx + lane / 3 - 1, yy = cy + lane % 3 - 1;
        int32_t z0, z1;
        if (xx >= 0 && xx < g.gx && yy >= 0 && yy < g.gy && reach_row(cr, lane / 3 - 1, lane % 3 - 1, cz, g.gz, z0, z1)) {
            const uint32_t rowk = ((uint32_t)xx * (uint32_t)g.gy + (uint32_t)yy) * (uint32_t)g.gz;
            rj0 = M.start(rowk + (uint32_t)z0);
            rlen = M.start(rowk + (uint32_t)z1 + 1u) - rj0;
        }
    }
    const uint32_t incl = row_scan_incl(rlen);   // inclusive prefix over lanes 0..8 (lanes >= 9 hold 0)
    const uint32_t excl = incl - rlen;
    // the rows' flattened starts, wave-uniform (scalar registers)
    uint32_t P[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) P[k] = (uint32_t)__builtin_amdgcn_readlane((int)excl, k);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 8);
    // candidate f -> sorted slot: its row k counts the starts at or below f; the row's first slot and flattened start
    // come from lane k (a per-lane select chain over P / J compiled to a scratch-memory table)
    auto slot_of = [&](uint32_t f) __attribute__((always_inline)) {
        int k = 0;
#pragma unroll
        for (int r = 1; r < 9; ++r) k += f >= P[r] ? 1 : 0;
        return (uint32_t)__shfl((int)rj0, k, 64) + (f - (uint32_t)__shfl((int)excl, k, 64));
    };
    // the hit's F and TA (TA = 0 for a repulsion-only contact) and the int torque b scatters into a (:291)
    auto body = [&](uint32_t j, f3& F, f3& TA) __attribute__((always_inline)) {
        const uint32_t o = M.old(j);
        const float4 pb = pos[o], vb = vel[o], wb = omg[o];
        const Body B{xyz(pb), xyz(vb), xyz(wb), pb.w};
        f3 TB;
        const int h = contact_pair(c, A, B, F, TA, TB);
        if (h == 2) {   // b's scatter into a (:291)
            const f3 sc = TA * dt * TORQUE_SCALE;
            q0 += (uint32_t)ftoi(sc.x);
            q1 += (uint32_t)ftoi(sc.y);
            q2 += (uint32_t)ftoi(sc.z);
        }
        if (h != 2) TA = mk(0, 0, 0);
        if (h == 0) F = mk(0, 0, 0);
    };
    // a batch's hits into the sums in lane order, transposed: the hit lanes write (F, TA) to the wave's LDS row and
    // lane c < 6 adds component c of each (F.x, F.y, F.z, TA.x, TA.y, TA.z), the same adds in the same order
    __shared__ float cf_rows[WAVES][64 * 6];
    __shared__ uint32_t cf_list[WAVES][64 * CF_CHUNKS];   // a round's touching candidates (sorted slots), in order
    float* row = cf_rows[threadIdx.x >> 6];
    uint32_t* list = cf_list[threadIdx.x >> 6];
    float comp = 0.0f;
    auto fold = [&](const f3& F, const f3& TA, bool hit) __attribute__((always_inline)) {
        uint64_t m = __ballot(hit);
        if (m == 0) return;   // wave-uniform
        if (hit) {
            float* e = row + 6 * lane;
            e[0] = F.x; e[1] = F.y; e[2] = F.z; e[3] = TA.x; e[4] = TA.y; e[5] = TA.z;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < 6) {
            while (__popcll(m) >= 4) {   // four reads in flight, then the four adds in order
                float x[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    x[u] = row[6 * __builtin_ctzll(m) + lane];
                    m &= m - 1ull;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) comp = comp + x[u];
            }
            for (; m; m &= m - 1ull) comp = comp + row[6 * __builtin_ctzll(m) + lane];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
#pragma unroll 1
    for (uint32_t round = 0; round < total; round += 64u * CF_CHUNKS) {
        // chunks holding candidates (wave-uniform): a round past the last candidate scans nothing (the reference's
        // R = 15 sphere: ~350 candidates, 6 of 8 chunks)
        const uint32_t nch = min((total - round + 63u) >> 6, (uint32_t)CF_CHUNKS);
        uint32_t jj[CF_CHUNKS];
        float4 pb[CF_CHUNKS];
#pragma unroll
        for (int ch = 0; ch < CF_CHUNKS; ++ch) {   // every position load of the round in flight together
            if ((uint32_t)ch >= nch) break;
            const uint32_t f = round + (uint32_t)(ch * 64 + lane);
            jj[ch] = slot_of(min(f, total - 1u));
            pb[ch] = pos[M.old(jj[ch])];
        }
        // bit ch: candidate (round, ch, lane) may touch a (:240, :253). A superset of the reference's test
        // reff − |d| > 0.001 without the square root: |d|² < t² with t = reff − 0.0009 + 1e-5·reff, whose margin
        // (1e-4 + 1e-5·reff) exceeds the few-ulp rounding of |d| and t for every reff; contact_pair's own first test
        // is that same reference test, and a candidate it rejects adds F = TA = +0 (no change to the sums, which
        // are never −0) and no torque.
        uint32_t touch = 0u;
#pragma unroll
        for (int ch = 0; ch < CF_CHUNKS; ++ch) {
            if ((uint32_t)ch >= nch) break;
            const uint32_t f = round + (uint32_t)(ch * 64 + lane);
            const f3 d = A.pos - xyz(pb[ch]);
            const float reff = A.r * 0.5f + pb[ch].w * 0.5f;
            const float t = (reff - 0.0009f) + reff * 1e-5f;
            if (f < total && (int32_t)jj[ch] != a && t > 0.0f && dot(d, d) < t * t) touch |= 1u << ch;
        }
        // compaction: candidate (ch, lane) goes to list position (touches of the chunks before) + (touching lanes
        // below it in its chunk); the rounds' positions are wave-uniform running counts
        uint32_t T = 0;
#pragma unroll
        for (int ch = 0; ch < CF_CHUNKS; ++ch) {
            if ((uint32_t)ch >= nch) break;
            const bool t = (touch >> ch) & 1u;
            const uint64_t b = __ballot(t);
            if (t) list[T + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u))] = jj[ch];
            T += (uint32_t)__popcll(b);
        }
        if (T == 0) continue;   // wave-uniform
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
        for (uint32_t b0 = 0; b0 < T; b0 += 64u) {   // a batch: every lane one body, then the adds in list order
            const bool hit = b0 + (uint32_t)lane < T;
            f3 F = mk(0, 0, 0), TA = mk(0, 0, 0);
            if (hit) body(list[b0 + (uint32_t)lane], F, TA);
            fold(F, TA, hit);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        q0 += (uint32_t)__shfl_xor((int)q0, o, 64);
        q1 += (uint32_t)__shfl_xor((int)q1, o, 64);
        q2 += (uint32_t)__shfl_xor((int)q2, o, 64);
    }
    tq[0] = q0; tq[1] = q1; tq[2] = q2;
    totalForce = mk(__shfl(comp, 0, 64), __shfl(comp, 1, 64), __shfl(comp, 2, 64));
    totalTorque = mk(__shfl(comp, 3, 64), __shfl(comp, 4, 64), __shfl(comp, 5, 64));
    v = A.vel + (totalForce / va.w) * dt;                                    // :302-306
    w = A.omg + (totalTorque / wa.w) * dt;
}

// T lanes per target: 16 or 64 (team form) or CT_FLAT (one wave, flat form); lanes of a target for the launch mapping
template <int T> constexpr int team_lanes() { return T == CT_FLAT ? 64 : T; }
template <int T>
__device__ __forceinline__ void contact_accumulate_lanes(const float4* __restrict__ pos, const float4* __restrict__ vel,
                                                         const float4* __restrict__ omg, const uint32_t* __restrict__ cs,
                                                         const GridDesc& g, const ContactConst& c, int32_t a, float4 pa,
                                                         float4 va, float4 wa, f3& v, f3& w, uint32_t tq[3]) {
    if constexpr (T == CT_FLAT)
        contact_accumulate_flat<CT_BLK / 64>(pos, vel, omg, DirectMap{cs}, g, c, a, pa, va, wa, v, w, tq);
    else
        contact_accumulate_team<T>(pos, vel, omg, cs, g, c, a, pa, va, wa, v, w, tq);
}

// ApplyDragForce (compute:316-323; selectedID is a particle index). The reference applies it
// to any particle below particleBuffer.Length, active or not.
__device__ __forceinline__ f3 apply_drag(const ContactConst& c, int32_t pid, f3 p, f3 v, float mass) {
    if (c.drag_id >= 0 && pid == c.drag_id) {
        const f3 toTarget = mk(c.drag_tx, c.drag_ty, c.drag_tz) - p;
        const f3 force = toTarget * c.drag_strength * c.dt;
        v = v + force / mass;
    }
    return v;
}

// Drag, UpdateMotion (compute:332-354) and UpdateRotation (:385-406) of an active particle.
__device__ __forceinline__ void contact_finish(const ContactConst& c, int32_t pid, float4 pa, f3 v, f3 w,
                                               float mass, float inertia, float drag, float4 qa,
                                               const uint32_t tq[3], f3& p_out, f3& v_out, f3& w_out,
                                               float4& q_out) {
    const float dt = c.dt;
    f3 p = xyz(pa);
    v = apply_drag(c, pid, p, v, mass);
    const float linearDamping = exp_r(-drag * c.global_drag * dt);
    const float angularDamping = exp_r(-c.torque_damping * dt);
    v = v * linearDamping;
    w = w * angularDamping;
    p = p + v * dt;
    if (len(p) > c.spawn_radius) {
        const f3 norm = normalize(p);
        p = norm * c.spawn_radius;
        v = v - norm * (2.0f * dot(v, norm));                              // reflect
        const f3 tangentialVel = v - norm * dot(v, norm);
        const f3 frictionDir = normalize(tangentialVel + mk(1e-6f, 1e-6f, 1e-6f));
        const float frictionMag = len(tangentialVel) * c.boundary_friction;
        const float effectiveRadius = pa.w * c.roll_mult;
        const f3 torque = cross(-norm * effectiveRadius, -frictionDir * frictionMag);
        w = w + (torque / inertia) * dt;
    }
    const f3 torque = mk((float)(int32_t)tq[0], (float)(int32_t)tq[1], (float)(int32_t)tq[2]) / TORQUE_SCALE;
    w = w + torque / inertia;
    w = w * exp_r(-c.torque_damping * dt);
    float4 q = qa;
    const float angle = len(w * dt);
    if (angle > 0.00001f) {
        const f3 axis = normalize(w);
        float s, co;
        sincos_r(angle * 0.5f, s, co);
        const float4 r = quat_mul(make_float4(axis.x * s, axis.y * s, axis.z * s, co), qa);
        const float l = sqrtf(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w);
        q = make_float4(r.x / l, r.y / l, r.z / l, r.w / l);
    }
    p_out = p; v_out = v; w_out = w; q_out = q;
}

// The whole frame without adhesion: ApplySPHForces + drag + motion + rotation in one pass.
__global__ __launch_bounds__(CT_BLK) void k_contact_step(
    const float4* __restrict__ pos, const float4* __restrict__ vel, const float4* __restrict__ omg,
    const float4* __restrict__ rot, const float4* __restrict__ aux, const int32_t* __restrict__ id,
    const uint32_t* __restrict__ cs, int32_t n_active, int32_t n, GridDesc g, ContactConst c,
    float4* __restrict__ pos_o, float4* __restrict__ vel_o, float4* __restrict__ omg_o,
    float4* __restrict__ rot_o, int32_t* __restrict__ torque_o, uint32_t* __restrict__ keys_o, MoverSink mv) {
    const int32_t a = blockIdx.x * CT_BLK + threadIdx.x;
    if (a >= n) return;
    rmax_load(c);
    const float4 pa = pos[a], va = vel[a], wa = omg[a], qa = rot[a];
    if (a >= n_active) {   // inactive slots (id >= activeParticleCount): drag only
        const f3 v = apply_drag(c, id[a], xyz(pa), xyz(va), va.w);
        pos_o[a] = pa; vel_o[a] = make_float4(v.x, v.y, v.z, va.w); omg_o[a] = wa; rot_o[a] = qa;
        if (torque_o) { torque_o[3 * a] = 0; torque_o[3 * a + 1] = 0; torque_o[3 * a + 2] = 0; }
        keys_o[a] = g.ncells;
        append_mover(mv, a, g.ncells);
        return;
    }
    f3 v, w;
    uint32_t tq[3];
    contact_accumulate(pos, vel, omg, cs, g, c, a, pa, va, wa, v, w, tq);
    f3 p;
    float4 q;
    contact_finish(c, id[a], pa, v, w, va.w, wa.w, aux[a].x, qa, tq, p, v, w, q);
    pos_o[a] = make_float4(p.x, p.y, p.z, pa.w);
    vel_o[a] = make_float4(v.x, v.y, v.z, va.w);
    omg_o[a] = make_float4(w.x, w.y, w.z, wa.w);
    rot_o[a] = q;
    if (torque_o) {
        torque_o[3 * a] = (int32_t)tq[0]; torque_o[3 * a + 1] = (int32_t)tq[1]; torque_o[3 * a + 2] = (int32_t)tq[2];
    }
    keys_o[a] = cell_key(g, p.x, p.y, p.z);
    append_mover(mv, a, keys_o[a]);
}

// k_contact_step with T lanes per target (contact_accumulate_team); team lane 0 finishes and writes.
template <int T>
__global__ __launch_bounds__(CT_BLK) void k_contact_step_team(
    const float4* __restrict__ pos, const float4* __restrict__ vel, const float4* __restrict__ omg,
    const float4* __restrict__ rot, const float4* __restrict__ aux, const int32_t* __restrict__ id,
    const uint32_t* __restrict__ cs, int32_t n_active, int32_t n, GridDesc g, ContactConst c,
    float4* __restrict__ pos_o, float4* __restrict__ vel_o, float4* __restrict__ omg_o,
    float4* __restrict__ rot_o, int32_t* __restrict__ torque_o, uint32_t* __restrict__ keys_o, MoverSink mv) {
    constexpr int L = team_lanes<T>();
    const int32_t a = blockIdx.x * (CT_BLK / L) + (int32_t)(threadIdx.x / L);
    const bool lead = (threadIdx.x & (L - 1)) == 0;
    if (a >= n) return;                                                      // team-uniform
    rmax_load(c);
    const float4 pa = pos[a], va = vel[a], wa = omg[a];
    if (a >= n_active) {
        if (!lead) return;
        const float4 qa = rot[a];
        const f3 v = apply_drag(c, id[a], xyz(pa), xyz(va), va.w);
        pos_o[a] = pa; vel_o[a] = make_float4(v.x, v.y, v.z, va.w); omg_o[a] = wa; rot_o[a] = qa;
        if (torque_o) { torque_o[3 * a] = 0; torque_o[3 * a + 1] = 0; torque_o[3 * a + 2] = 0; }
        keys_o[a] = g.ncells;
        append_mover(mv, a, g.ncells);
        return;
    }
    f3 v, w;
    uint32_t tq[3];
    contact_accumulate_lanes<T>(pos, vel, omg, cs, g, c, a, pa, va, wa, v, w, tq);
    if (!lead) return;
    f3 p;
    float4 q;
    contact_finish(c, id[a], pa, v, w, va.w, wa.w, aux[a].x, rot[a], tq, p, v, w, q);
    pos_o[a] = make_float4(p.x, p.y, p.z, pa.w);
    vel_o[a] = make_float4(v.x, v.y, v.z, va.w);
    omg_o[a] = make_float4(w.x, w.y, w.z, wa.w);
    rot_o[a] = q;
    if (torque_o) {
        torque_o[3 * a] = (int32_t)tq[0]; torque_o[3 * a + 1] = (int32_t)tq[1]; torque_o[3 * a + 2] = (int32_t)tq[2];
    }
    keys_o[a] = cell_key(g, p.x, p.y, p.z);
    append_mover(mv, a, keys_o[a]);
}

// k_contact_forces with T lanes per target.
template <int T>
__global__ __launch_bounds__(CT_BLK) void k_contact_forces_team(
    const float4* __restrict__ pos, const float4* __restrict__ vel, const float4* __restrict__ omg,
    const int32_t* __restrict__ id, const uint32_t* __restrict__ cs, int32_t n_active, int32_t n, GridDesc g,
    ContactConst c, float4* __restrict__ vel_o, float4* __restrict__ omg_o, int32_t* __restrict__ torque_o,
    int32_t* __restrict__ slot_of) {
    constexpr int L = team_lanes<T>();
    const int32_t a = blockIdx.x * (CT_BLK / L) + (int32_t)(threadIdx.x / L);
    const bool lead = (threadIdx.x & (L - 1)) == 0;
    if (a >= n) return;                                                      // team-uniform
    rmax_load(c);
    const float4 pa = pos[a], va = vel[a], wa = omg[a];
    f3 v = xyz(va), w = xyz(wa);
    uint32_t tq[3] = {0u, 0u, 0u};
    if (a < n_active) contact_accumulate_lanes<T>(pos, vel, omg, cs, g, c, a, pa, va, wa, v, w, tq);
    if (!lead) return;
    const int32_t pid = id[a];
    if ((uint32_t)pid < (uint32_t)n) slot_of[pid] = a;
    vel_o[a] = make_float4(v.x, v.y, v.z, va.w);
    omg_o[a] = make_float4(w.x, w.y, w.z, wa.w);
    torque_o[3 * a] = (int32_t)tq[0]; torque_o[3 * a + 1] = (int32_t)tq[1]; torque_o[3 * a + 2] = (int32_t)tq[2];
}

// With adhesion, phase 1: ApplySPHForces only (v1, ω1 and the int torque into *_o), plus the
// particle-index → slot map the bond pass reads particles through.
__global__ __launch_bounds__(CT_BLK) void k_contact_forces(
    const float4* __restrict__ pos, const float4* __restrict__ vel, const float4* __restrict__ omg,
    const int32_t* __restrict__ id, const uint32_t* __restrict__ cs, int32_t n_active, int32_t n, GridDesc g,
    ContactConst c, float4* __restrict__ vel_o, float4* __restrict__ omg_o, int32_t* __restrict__ torque_o,
    int32_t* __restrict__ slot_of) {
    const int32_t a = blockIdx.x * CT_BLK + threadIdx.x;
    if (a >= n) return;
    rmax_load(c);
    const float4 pa = pos[a], va = vel[a], wa = omg[a];
    const int32_t pid = id[a];
    if ((uint32_t)pid < (uint32_t)n) slot_of[pid] = a;
    f3 v = xyz(va), w = xyz(wa);
    uint32_t tq[3] = {0u, 0u, 0u};
    if (a < n_active) contact_accumulate(pos, vel, omg, cs, g, c, a, pa, va, wa, v, w, tq);
    vel_o[a] = make_float4(v.x, v.y, v.z, va.w);
    omg_o[a] = make_float4(w.x, w.y, w.z, wa.w);
    torque_o[3 * a] = (int32_t)tq[0]; torque_o[3 * a + 1] = (int32_t)tq[1]; torque_o[3 * a + 2] = (int32_t)tq[2];
}

// With adhesion, phase 3: ApplyAdhesionDeltas (compute:587-607) as a gather of this particle's
// bond terms (adhesion.hip), then drag, motion and rotation. vel_io / omg_io hold phase 1's
// v1, ω1 and are updated in place (each slot touches only its own element).
__global__ __launch_bounds__(CT_BLK) void k_contact_finish(
    const float4* __restrict__ pos, const float4* __restrict__ rot, const float4* __restrict__ aux,
    const int32_t* __restrict__ id, const int32_t* __restrict__ torque, int32_t n_active, int32_t n,
    GridDesc g, ContactConst c, BondView b, float4* __restrict__ vel_io, float4* __restrict__ omg_io,
    float4* __restrict__ pos_o, float4* __restrict__ rot_o, uint32_t* __restrict__ keys_o, MoverSink mv) {
    const int32_t a = blockIdx.x * CT_BLK + threadIdx.x;
    if (a >= n) return;
    const float4 pa = pos[a], va = vel_io[a], wa = omg_io[a], qa = rot[a];
    const int32_t pid = id[a];
    if (a >= n_active) {   // inactive: ApplyAdhesionDeltas and UpdateMotion skip it, drag does not
        const f3 v = apply_drag(c, pid, xyz(pa), xyz(va), va.w);
        vel_io[a] = make_float4(v.x, v.y, v.z, va.w);
        pos_o[a] = pa; rot_o[a] = qa;
        keys_o[a] = g.ncells;
        append_mover(mv, a, g.ncells);
        return;
    }
    f3 v = xyz(va);
    float4 q = qa;
    bond_gather(b, pid, v, q);
    const uint32_t tq[3] = {(uint32_t)torque[3 * a], (uint32_t)torque[3 * a + 1], (uint32_t)torque[3 * a + 2]};
    f3 p, w;
    contact_finish(c, pid, pa, v, xyz(wa), va.w, wa.w, aux[a].x, q, tq, p, v, w, q);
    pos_o[a] = make_float4(p.x, p.y, p.z, pa.w);
    vel_io[a] = make_float4(v.x, v.y, v.z, va.w);
    omg_io[a] = make_float4(w.x, w.y, w.z, wa.w);
    rot_o[a] = q;
    keys_o[a] = cell_key(g, p.x, p.y, p.z);
    append_mover(mv, a, keys_o[a]);
}

// ---------------------------------------------------------------- the one-launch step at the reference's scale
// Model R at N <= FZ_N (the reference runs 4-10,000 particles, ParticleSystemController.cs:12): the re-sort, ApplySPHForces,
// drag, motion and rotation of a step in ONE launch, with no grid barrier. Every workgroup rebuilds, in LDS, the step's
// permutation from the previous step's mover list (m <= N <= FZ_N movers fit whole): the movers sorted by (new key,
// slot), their new slots dst_r = (q − A(q)) + r (resort.hip's formulas, q the insertion slot, A the movers below a slot
// from a slot bitmap), so that any sorted position j maps to the slot of the previous order that holds it
// (FusedMap::old) and any cell start follows from the old table (FusedMap::start). The contact pass then reads the
// previous step's arrays through that map and writes its targets at their sorted positions: the outputs are the
// re-sorted arrays, bit-identical to re-sort + contact (tests/test_gpu_small.py). Each workgroup also writes an equal
// share of the new cell-start table. Movers of this step go to the other list; the counters rotate over three (the one
// this step appends to was zeroed by the step before).
constexpr int FZ_BLK = 1024;   // 16 targets (one per wave) per workgroup: the permutation is built once per 16
constexpr int FZ_T = FZ_BLK / 64;

// Test-only timing probe (scripts/contact_probe.py, a -DSPH_CONTACT_PROBE build): per workgroup the wall clock (100 MHz)
// at its start, after the permutation build, after the barrier and at its end, each wave's end of its neighbour sums
// (8-23), and in the finish: after its arithmetic (24) and after its plain stores, before the mover append (25).
#ifdef SPH_CONTACT_PROBE
constexpr int CT_PROBE_W = 32;
__device__ uint64_t g_ct_probe[256 * 32];
static_assert(CT_PROBE_W == 32, "FZ_PROBE's stride");
#define CT_PROBE(cond, slot)                                                                               \
    do {                                                                                                   \
        if ((cond) && blockIdx.x < 256) g_ct_probe[blockIdx.x * CT_PROBE_W + (slot)] = wall_clock64();    \
    } while (0)
extern "C" int sph_debug_contact_probe(uint64_t* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ct_probe), sizeof(g_ct_probe)) == hipSuccess ? 0 : -1;
}
#else
#define CT_PROBE(cond, slot) \
    do {                     \
    } while (0)
#endif

// A target's neighbour sums, handed from its wave to the lane that finishes it
struct FusedFin {
    float4 pa, va, wa, rot, aux;
    f3 v, w;
    uint32_t tq[3];
    uint32_t key_a;
    int32_t id, mode;
};

__global__ __launch_bounds__(FZ_BLK) void k_contact_fused(FusedIO io, int32_t n_active, int32_t n, GridDesc g,
                                                          ContactConst c) {
    __shared__ FusedLds L;
    __shared__ FusedFin fin[FZ_T];
    CT_PROBE(threadIdx.x == 0, 0);
    rmax_load(c);   // with the build's first loads
    const FusedMap M = fused_build<FZ_BLK>(L, io.count, io.mi, io.mk, io.cs, n, io.count_zero, io.host_count);
    CT_PROBE(threadIdx.x == 0, 1);
    {   // one target per wave: sorted position a, read from the previous order's slot o
        const int32_t a = blockIdx.x * FZ_T + (int32_t)(threadIdx.x >> 6);
        if (a < n) {   // wave-uniform
            bool mv;
            uint32_t key_mv;
            const uint32_t o = M.old_at((uint32_t)a, mv, key_mv);
            const float4 pa = io.pos[o], va = io.vel[o], wa = io.omg[o];
            // the finishing lane's inputs, loaded under the neighbour sums; the old key loaded whether or not the
            // target moved (a load under a branch had the compiler wait for it before issuing the others)
            const float4 rot = io.rot[o], aux = io.aux[o];
            const int32_t id = io.id[o], mode = io.mode[o];
            const uint32_t sko = io.sk[o];
            const uint32_t key_a = mv ? key_mv : sko;
            f3 v = xyz(va), w = xyz(wa);
            uint32_t tq[3] = {0u, 0u, 0u};
            if (a < n_active) contact_accumulate_flat<CF_WAVES>(io.pos, io.vel, io.omg, M, g, c, a, pa, va, wa, v, w, tq);
            if ((threadIdx.x & 63u) == 0) {
                FusedFin& f = fin[threadIdx.x >> 6];
                f.pa = pa; f.va = va; f.wa = wa; f.v = v; f.w = w;
                f.tq[0] = tq[0]; f.tq[1] = tq[1]; f.tq[2] = tq[2];
                f.rot = rot; f.aux = aux;
                f.key_a = key_a; f.id = id; f.mode = mode;
            }
        }
        CT_PROBE((threadIdx.x & 63u) == 0, 8 + (threadIdx.x >> 6));
    }
    __syncthreads();
    CT_PROBE(threadIdx.x == 0, 2);
    // drag, motion and rotation of the workgroup's 16 targets on 16 lanes of wave 0: the per-target tail (double-
    // evaluated exp, sin, cos) costs one wave's issue instead of sixteen. Waves 1-15 meanwhile write the workgroup's
    // share of the new cell-start table.
    if (threadIdx.x >= 64u) {
        fused_cs_share(M, io.cs_o, g.ncells, threadIdx.x - 64u, FZ_BLK - 64u);
        return;
    }
    const int32_t a = blockIdx.x * FZ_T + (int32_t)threadIdx.x;
    if (threadIdx.x >= (uint32_t)FZ_T || a >= n) return;
    const FusedFin& f = fin[threadIdx.x];
    const uint32_t key_a = f.key_a;
    const float4 pa = f.pa, va = f.va, wa = f.wa;
    uint32_t key_n;
    f3 p, v, w;
    float4 q;
    if (a >= n_active) {   // inactive slots (id >= activeParticleCount): drag only
        v = apply_drag(c, f.id, xyz(pa), xyz(va), va.w);
        p = xyz(pa);
        w = xyz(wa);
        q = f.rot;
        key_n = g.ncells;
    } else {
        contact_finish(c, f.id, pa, f.v, f.w, va.w, wa.w, f.aux.x, f.rot, f.tq, p, v, w, q);
        key_n = cell_key(g, p.x, p.y, p.z);
    }
    CT_PROBE(threadIdx.x == 0, 24);
    io.pos_o[a] = a >= n_active ? pa : make_float4(p.x, p.y, p.z, pa.w);
    io.vel_o[a] = make_float4(v.x, v.y, v.z, va.w);
    io.omg_o[a] = a >= n_active ? wa : make_float4(w.x, w.y, w.z, wa.w);
    io.rot_o[a] = q;
    io.aux_o[a] = f.aux;
    io.id_o[a] = f.id;
    io.mode_o[a] = f.mode;
    if (io.torque_o) {
        io.torque_o[3 * a] = (int32_t)f.tq[0]; io.torque_o[3 * a + 1] = (int32_t)f.tq[1];
        io.torque_o[3 * a + 2] = (int32_t)f.tq[2];
    }
    io.sk_o[a] = key_a;
    io.keys_o[a] = key_n;
    CT_PROBE(threadIdx.x == 0, 25);
    if (key_n != key_a) {   // a mover of the next step's re-sort
        const uint32_t r = atomicAdd(io.count_o, 1u);
        if (r < io.cap) {
            io.mi_o[r] = (uint32_t)a;
            io.mk_o[r] = key_n;
            io.mo_o[r] = key_a;
        }
    }
    CT_PROBE(threadIdx.x == 0, 3);
}

int32_t contact_fused_max() { return FZ_N; }

void launch_contact_fused(const FusedIO& io, int32_t n_active, int32_t n, GridDesc g, ContactConst c, hipStream_t s) {
    if (n <= 0 || n > FZ_N) return;
    SPH_LAUNCH(k_contact_fused, (n + FZ_T - 1) / FZ_T, FZ_BLK, 0, s, io, n_active, n, g, c);
}

// Lanes per target: enough teams to fill the chip (256 CUs × 8 waves × 64 lanes ≈ 131k lanes) without
// splitting thin candidate lists. A forced choice (1, 16, 64, CT_FLAT) wins; every choice gives bit-identical
// results (contact_accumulate_team).
static int contact_team(int32_t n, int forced) {
    if (forced == 1 || forced == 16 || forced == 64 || forced == CT_FLAT) return forced;
    // the flat form: 32.2 -> 26.5 us per step at 4,096 particles, 334 -> 315 us at 32,768 (scripts/small_n_timing.py,
    // profiles/r05_small_n.log)
    if (n <= 32768) return CT_FLAT;
    if (n <= 262144) return 16;
    return 1;
}

void launch_contact_step(const float4* pos, const float4* vel, const float4* omg, const float4* rot,
                         const float4* aux, const int32_t* id, const uint32_t* cs, int32_t n_active,
                         int32_t n, GridDesc g, ContactConst c, float4* pos_o, float4* vel_o,
                         float4* omg_o, float4* rot_o, int32_t* torque_o, uint32_t* keys_o, int team,
                         MoverSink mv, hipStream_t s) {
    if (n <= 0) return;
    switch (contact_team(n, team)) {
#define SPH_CT_STEP(T)                                                                                        \
    case T:                                                                                                   \
        k_contact_step_team<T><<<(n + CT_BLK / team_lanes<T>() - 1) / (CT_BLK / team_lanes<T>()), CT_BLK, 0, s>>>(  \
            pos, vel, omg, rot, aux, id, cs, n_active, n, g, c, pos_o, vel_o, omg_o, rot_o, torque_o, keys_o, mv);  \
        break;
        SPH_CT_STEP(CT_FLAT)
        SPH_CT_STEP(64)
        SPH_CT_STEP(16)
#undef SPH_CT_STEP
    default:
        k_contact_step<<<(n + CT_BLK - 1) / CT_BLK, CT_BLK, 0, s>>>(pos, vel, omg, rot, aux, id, cs, n_active, n, g,
                                                                    c, pos_o, vel_o, omg_o, rot_o, torque_o, keys_o, mv);
    }
}

void launch_contact_forces(const float4* pos, const float4* vel, const float4* omg, const int32_t* id,
                           const uint32_t* cs, int32_t n_active, int32_t n, GridDesc g, ContactConst c,
                           float4* vel_o, float4* omg_o, int32_t* torque_o, int32_t* slot_of, int team,
                           hipStream_t s) {
    if (n <= 0) return;
    switch (contact_team(n, team)) {
#define SPH_CT_FORCES(T)                                                                                      \
    case T:                                                                                                   \
        k_contact_forces_team<T><<<(n + CT_BLK / team_lanes<T>() - 1) / (CT_BLK / team_lanes<T>()), CT_BLK, 0, s>>>( \
            pos, vel, omg, id, cs, n_active, n, g, c, vel_o, omg_o, torque_o, slot_of);                         \
        break;
        SPH_CT_FORCES(CT_FLAT)
        SPH_CT_FORCES(64)
        SPH_CT_FORCES(16)
#undef SPH_CT_FORCES
    default:
        k_contact_forces<<<(n + CT_BLK - 1) / CT_BLK, CT_BLK, 0, s>>>(pos, vel, omg, id, cs, n_active, n, g, c,
                                                                      vel_o, omg_o, torque_o, slot_of);
    }
}

void launch_contact_finish(const float4* pos, const float4* rot, const float4* aux, const int32_t* id,
                           const int32_t* torque, int32_t n_active, int32_t n, GridDesc g, ContactConst c,
                           BondView b, float4* vel_io, float4* omg_io, float4* pos_o, float4* rot_o,
                           uint32_t* keys_o, MoverSink mv, hipStream_t s) {
    if (n > 0)
        k_contact_finish<<<(n + CT_BLK - 1) / CT_BLK, CT_BLK, 0, s>>>(pos, rot, aux, id, torque, n_active, n, g, c,
                                                                      b, vel_io, omg_io, pos_o, rot_o, keys_o, mv);
}

}  // namespace sph
