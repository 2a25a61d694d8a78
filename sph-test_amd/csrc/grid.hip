// grid.hip — hash, cell-start, reorder and boundary-format kernels (gfx950).
//
// Reference counterparts:
//   keys          GetGridCoord/GridHash + BuildHashGrid (SimulateParticles.compute:102-109,196-209)
//   cell_start    the reference has none: its gridHeads/gridNext lists are walked instead
//                 (compute:236-298); cell_start[k] = lower_bound(sorted keys, k), valid for
//                 empty cells too, so a row of 3 cells is one contiguous range
//   scatter_by_id CopyPositions/CopyRotationsToReadbackBuffer (compute:410-422), into
//                 particle-index order
//   aos84 <-> SoA particleBuffer's 84-byte Particle struct (compute:23-40,
//                 ParticleSystemController.cs:157-175) at the ABI; SoA float4 inside
//   lattice       dam-break / sloshing lattice with seeded jitter (SPEC_SPH.md §2)
#include "common.h"

namespace sph {

constexpr int BLK = 256;
static inline int nblk(int64_t n) { return (int)((n + BLK - 1) / BLK); }

// rmax (Model R, optional): the largest radius (pos.w) as float bits, atomicMax of the waves' maxima into a word the
// caller zeroed; a negative or NaN radius gives bits above +inf's, which the contact pass reads as "no bound".
__global__ __launch_bounds__(BLK) void k_keys(const float4* __restrict__ pos, int32_t n,
                                              const int32_t* __restrict__ id, int32_t n_active_id,
                                              GridDesc g, uint32_t* __restrict__ keys, bool window_sentinel,
                                              uint32_t* __restrict__ rmax) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i >= n) return;
    const float4 p = pos[i];
    uint32_t k = window_sentinel ? window_key(g, p.x, p.y, p.z) : cell_key(g, p.x, p.y, p.z);
    if (id != nullptr && id[i] >= n_active_id) k = g.ncells;   // inactive: sorts last
    keys[i] = k;
    if (rmax) {
        uint32_t r = __float_as_uint(p.w);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) r = max(r, (uint32_t)__shfl_xor((int)r, o, 64));
        if (lane_id() == __builtin_ctzll(__ballot(true))) atomicMax(rmax, r);
    }
}

constexpr uint32_t CS_SHORT = 32;
constexpr uint32_t CS_CHUNK = 8192;   // long gaps are queued in chunks so no workgroup fills more

// thread i in [0, n]: cells (key[i-1], key[i]] start at slot i (key[-1] = -1, key[n] = ncells).
// Thread n also writes cs[ncells + 1] = n: the re-sort reads cs_old[k + 1] for a mover whose key is
// the inactive sentinel ncells.
__global__ __launch_bounds__(BLK) void k_cell_start(const uint32_t* __restrict__ sk, int32_t n,
                                                    uint32_t* __restrict__ cs, uint32_t ncells,
                                                    uint4* __restrict__ gaps, uint32_t* __restrict__ gap_count,
                                                    uint32_t* __restrict__ gap_next) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i == 0) *gap_next = 0u;   // the next call's counter (ping-pong: no memset launch)
    if (i > n) return;
    if (i == n) cs[ncells + 1] = (uint32_t)n;
    const int64_t kp = i > 0 ? (int64_t)sk[i - 1] : -1;
    const int64_t kc = i < n ? (int64_t)sk[i] : (int64_t)ncells;
    if (kc <= kp) return;
    if (kc - kp <= CS_SHORT) {
        for (int64_t k = kp + 1; k <= kc; ++k) cs[k] = (uint32_t)i;
    } else {
        const uint32_t nch = (uint32_t)((kc - kp + CS_CHUNK - 1) / CS_CHUNK);
        const uint32_t slot = atomicAdd(gap_count, nch);
        for (uint32_t c = 0; c < nch; ++c) {
            const int64_t a = kp + 1 + (int64_t)c * CS_CHUNK;
            const int64_t b = a + CS_CHUNK - 1 < kc ? a + CS_CHUNK - 1 : kc;
            gaps[slot + c] = make_uint4((uint32_t)a, (uint32_t)b, (uint32_t)i, 0u);
        }
    }
}

__global__ __launch_bounds__(BLK) void k_cell_start_gaps(const uint4* __restrict__ gaps,
                                                         const uint32_t* __restrict__ gap_count,
                                                         uint32_t* __restrict__ cs) {
    const uint32_t ng = *gap_count;
    for (uint32_t gi = blockIdx.x; gi < ng; gi += gridDim.x) {
        const uint4 gp = gaps[gi];
        for (uint32_t k = gp.x + threadIdx.x; k <= gp.y; k += BLK) cs[k] = gp.z;
    }
}

// Model R's seven slot arrays in one launch (at the reference's few thousand particles each
// launch is a few µs of fixed cost and moves almost nothing)
__global__ __launch_bounds__(BLK) void k_gather_r(const uint32_t* __restrict__ perm, GatherR g, int32_t n) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = perm[i];
#pragma unroll
    for (int k = 0; k < 5; ++k) g.f4o[k][i] = g.f4[k][s];
#pragma unroll
    for (int k = 0; k < 2; ++k) g.i32o[k][i] = g.i32[k][s];
}

__global__ __launch_bounds__(BLK) void k_gather_s(const uint32_t* __restrict__ perm,
                                                  const float4* __restrict__ pos,
                                                  const float4* __restrict__ vel,
                                                  const int32_t* __restrict__ id,
                                                  float4* __restrict__ pos_o, float4* __restrict__ vel_o,
                                                  int32_t* __restrict__ id_o, int32_t n) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = perm[i];
    pos_o[i] = pos[s];
    vel_o[i] = vel[s];
    id_o[i] = id[s];
}

__global__ __launch_bounds__(BLK) void k_scatter_f4_by_id(const float4* __restrict__ src,
                                                          const int32_t* __restrict__ id, int32_t n,
                                                          float* __restrict__ dst, int32_t comps) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i >= n) return;
    const float4 v = src[i];
    float* d = dst + (int64_t)id[i] * comps;
    d[0] = v.x; d[1] = v.y; d[2] = v.z;
    if (comps == 4) d[3] = v.w;
}

__global__ __launch_bounds__(BLK) void k_scatter_f2x_by_id(const float2* __restrict__ src,
                                                           const int32_t* __restrict__ id, int32_t n,
                                                           float* __restrict__ dst, int32_t comp) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i < n) dst[id[i]] = comp ? src[i].y : src[i].x;
}

__global__ __launch_bounds__(BLK) void k_scatter_i3_by_id(const int32_t* __restrict__ src,
                                                          const int32_t* __restrict__ id, int32_t n,
                                                          int32_t* __restrict__ dst) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i >= n) return;
    const int64_t d = (int64_t)id[i] * 3;
    dst[d] = src[3 * (int64_t)i];
    dst[d + 1] = src[3 * (int64_t)i + 1];
    dst[d + 2] = src[3 * (int64_t)i + 2];
}

// 84-byte Particle (compute:23-40): 21 dwords.
//  0-2 position, 3 radius, 4-6 velocity, 7 mass, 8-10 angularVelocity, 11 momentOfInertia,
//  12 drag, 13 repulsionStrength, 14 padding1 (C#: uint genomeFlags), 15 padding2,
//  16-19 rotation (x,y,z,w), 20 modeIndex (int)
__global__ __launch_bounds__(BLK) void k_aos84_to_soa(const uint32_t* __restrict__ aos, int32_t n,
                                                      float4* __restrict__ pos, float4* __restrict__ vel,
                                                      float4* __restrict__ omg, float4* __restrict__ rot,
                                                      float4* __restrict__ aux, int32_t* __restrict__ mode,
                                                      int32_t* __restrict__ id) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i >= n) return;
    const uint32_t* p = aos + (int64_t)i * 21;
    uint32_t w[21];
#pragma unroll
    for (int k = 0; k < 21; ++k) w[k] = p[k];
    auto f = [&](int k) { return __uint_as_float(w[k]); };
    pos[i] = make_float4(f(0), f(1), f(2), f(3));
    vel[i] = make_float4(f(4), f(5), f(6), f(7));
    if (omg) omg[i] = make_float4(f(8), f(9), f(10), f(11));
    if (aux) aux[i] = make_float4(f(12), f(13), f(14), f(15));
    if (rot) rot[i] = make_float4(f(16), f(17), f(18), f(19));
    if (mode) mode[i] = (int32_t)w[20];
    id[i] = i;
}

__global__ __launch_bounds__(BLK) void k_soa_to_aos84(const float4* __restrict__ pos,
                                                      const float4* __restrict__ vel,
                                                      const float4* __restrict__ omg,
                                                      const float4* __restrict__ rot,
                                                      const float4* __restrict__ aux,
                                                      const int32_t* __restrict__ mode,
                                                      const int32_t* __restrict__ id, int32_t n,
                                                      uint32_t* __restrict__ aos) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i >= n) return;
    uint32_t* p = aos + (int64_t)id[i] * 21;
    const float4 a = pos[i], b = vel[i];
    const float4 c = omg ? omg[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 d = aux ? aux[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 e = rot ? rot[i] : make_float4(0.f, 0.f, 0.f, 1.f);
    const float v[20] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w,
                         d.x, d.y, d.z, d.w, e.x, e.y, e.z, e.w};
#pragma unroll
    for (int k = 0; k < 20; ++k) p[k] = __float_as_uint(v[k]);
    p[20] = mode ? (uint32_t)mode[i] : 0xFFFFFFFFu;
}

__global__ __launch_bounds__(BLK) void k_pack_sv(const float* __restrict__ pos3,
                                                 const float* __restrict__ vel3, int32_t n,
                                                 float4* __restrict__ pos, float4* __restrict__ vel,
                                                 int32_t* __restrict__ id) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i >= n) return;
    const int64_t b = 3 * (int64_t)i;
    pos[i] = make_float4(pos3[b], pos3[b + 1], pos3[b + 2], 0.f);
    vel[i] = vel3 ? make_float4(vel3[b], vel3[b + 1], vel3[b + 2], 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
    id[i] = i;
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__device__ __forceinline__ float lattice_jitter(uint32_t seed_mix, uint32_t id, uint32_t axis,
                                                float jitter) {
    const uint32_t u = mix32(seed_mix ^ (3u * id + axis));
    const float r = (float)(u >> 8) * (1.0f / 16777216.0f);
    return (2.0f * r - 1.0f) * jitter;
}

__global__ __launch_bounds__(BLK) void k_lattice(int32_t dim, int32_t nx, int32_t ny, int32_t n,
                                                 float dx, float x0, float y0, float z0,
                                                 uint32_t seed_mix, float jitter,
                                                 float4* __restrict__ pos, float4* __restrict__ vel,
                                                 int32_t* __restrict__ id) {
#pragma clang fp contract(off)   // the oracle's roundings: one fma, one multiply, one add
    const int32_t p = blockIdx.x * BLK + threadIdx.x;
    if (p >= n) return;
    const int32_t ix = p % nx, iy = (p / nx) % ny, iz = p / (nx * ny);
    const uint32_t u = (uint32_t)p;
    const float x = fmaf((float)ix + 0.5f, dx, x0) + lattice_jitter(seed_mix, u, 0, jitter);
    const float y = fmaf((float)iy + 0.5f, dx, y0) + lattice_jitter(seed_mix, u, 1, jitter);
    const float z = dim == 3 ? fmaf((float)iz + 0.5f, dx, z0) + lattice_jitter(seed_mix, u, 2, jitter) : 0.0f;
    pos[p] = make_float4(x, y, z, 0.f);
    vel[p] = make_float4(0.f, 0.f, 0.f, 0.f);
    id[p] = p;
}

__global__ __launch_bounds__(BLK) void k_iota(uint32_t* __restrict__ v, int32_t n) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

// ---------------------------------------------------------------- launchers
void launch_keys(const float4* pos, int32_t n, const int32_t* id, int32_t n_active_id, GridDesc g,
                 uint32_t* keys, hipStream_t s, bool window_sentinel, uint32_t* rmax) {
    if (n > 0) k_keys<<<nblk(n), BLK, 0, s>>>(pos, n, id, n_active_id, g, keys, window_sentinel, rmax);
}
void launch_cell_start(const uint32_t* sk, int32_t n, uint32_t* cs, uint32_t ncells, uint4* gaps,
                       uint32_t* gap_count, int* par, hipStream_t s) {
    uint32_t* cur = gap_count + *par;
    uint32_t* next = gap_count + (1 - *par);
    k_cell_start<<<nblk((int64_t)n + 1), BLK, 0, s>>>(sk, n, cs, ncells, gaps, cur, next);
    k_cell_start_gaps<<<1024, BLK, 0, s>>>(gaps, cur, cs);
    *par = 1 - *par;
}
void launch_gather_r(const uint32_t* perm, const GatherR& g, int32_t n, hipStream_t s) {
    if (n > 0) k_gather_r<<<nblk(n), BLK, 0, s>>>(perm, g, n);
}
void launch_gather_s(const uint32_t* perm, const float4* pos, const float4* vel, const int32_t* id,
                     float4* pos_o, float4* vel_o, int32_t* id_o, int32_t n, hipStream_t s) {
    if (n > 0) k_gather_s<<<nblk(n), BLK, 0, s>>>(perm, pos, vel, id, pos_o, vel_o, id_o, n);
}
void launch_scatter_f4_by_id(const float4* src, const int32_t* id, int32_t n, float* dst, int32_t comps,
                             hipStream_t s) {
    if (n > 0) k_scatter_f4_by_id<<<nblk(n), BLK, 0, s>>>(src, id, n, dst, comps);
}
void launch_scatter_f2x_by_id(const float2* src, const int32_t* id, int32_t n, float* dst, hipStream_t s, int32_t comp) {
    if (n > 0) k_scatter_f2x_by_id<<<nblk(n), BLK, 0, s>>>(src, id, n, dst, comp);
}
void launch_scatter_i3_by_id(const int32_t* src, const int32_t* id, int32_t n, int32_t* dst, hipStream_t s) {
    if (n > 0) k_scatter_i3_by_id<<<nblk(n), BLK, 0, s>>>(src, id, n, dst);
}
void launch_aos84_to_soa(const void* aos, int32_t n, float4* pos, float4* vel, float4* omg, float4* rot,
                         float4* aux, int32_t* mode, int32_t* id, hipStream_t s) {
    if (n > 0)
        k_aos84_to_soa<<<nblk(n), BLK, 0, s>>>((const uint32_t*)aos, n, pos, vel, omg, rot, aux, mode, id);
}
void launch_soa_to_aos84(const float4* pos, const float4* vel, const float4* omg, const float4* rot,
                         const float4* aux, const int32_t* mode, const int32_t* id, int32_t n, void* aos,
                         hipStream_t s) {
    if (n > 0)
        k_soa_to_aos84<<<nblk(n), BLK, 0, s>>>(pos, vel, omg, rot, aux, mode, id, n, (uint32_t*)aos);
}
// Test hook (sph_debug_kick): every slot in [0, n) that holds particle `target` gets dv added to its velocity.
__global__ void k_kick(const int32_t* __restrict__ id, float4* __restrict__ vel, int32_t n, int32_t target, float dvx,
                       float dvy, float dvz) {
    const int32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i < n && id[i] == target) {
        const float4 v = vel[i];
        vel[i] = make_float4(v.x + dvx, v.y + dvy, v.z + dvz, v.w);
    }
}
void launch_kick(const int32_t* id, float4* vel, int32_t n, int32_t target, const float dv[3], hipStream_t s) {
    if (n > 0) k_kick<<<nblk(n), BLK, 0, s>>>(id, vel, n, target, dv[0], dv[1], dv[2]);
}
void launch_pack_sv(const float* pos3, const float* vel3, int32_t n, float4* pos, float4* vel, int32_t* id,
                    hipStream_t s) {
    if (n > 0) k_pack_sv<<<nblk(n), BLK, 0, s>>>(pos3, vel3, n, pos, vel, id);
}
void launch_lattice(int32_t dim, int32_t nx, int32_t ny, int32_t nz, float dx, float x0, float y0, float z0,
                    uint32_t seed, float jitter, float4* pos, float4* vel, int32_t* id, hipStream_t s) {
    const int32_t n = nx * ny * (dim == 3 ? nz : 1);
    // mix32(seed) on the host: the same integer hash as oracle/sph_oracle.c
    uint32_t x = seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    if (n > 0) k_lattice<<<nblk(n), BLK, 0, s>>>(dim, nx, ny, n, dx, x0, y0, z0, x, jitter, pos, vel, id);
}
void launch_iota(uint32_t* v, int32_t n, hipStream_t s) {
    if (n > 0) k_iota<<<nblk(n), BLK, 0, s>>>(v, n);
}

}  // namespace sph
