// particles.hip — Model R particle lifecycle on the device, gfx950.
//
//   k_init_sphere  InitParticles (SimulateParticles.compute:118-194), bit-reproducible: the
//                  HLSL sin / pow are evaluated in double and rounded once to float (the
//                  correctly rounded float result, which the D3D spec leaves to the hardware),
//                  with fp contraction off, so the C oracle computes the same bits.
//   k_split        the buffer half of ProcessPendingSplits (ParticleSystemController.cs:832-959):
//                  child A overwrites the parent's record, child B is a copy of it at index
//                  activeParticleCount + k. The reference reads the whole particle buffer back,
//                  edits it on the CPU and writes it all again (:793-794, :959); here only the
//                  split records travel (92 bytes each) and the edit is a device scatter.
//   k_get_range / k_set_range   particleBuffer.GetData/SetData(array, managedStart, bufferStart,
//                  count) on an index range (controller:519-522, 535, 736), through the index→slot
//                  map (the device keeps particles cell-sorted).
#include "common.h"

namespace sph {

constexpr int PL_BLK = 256;

static inline int nblk_pl(int32_t n) { return (n + PL_BLK - 1) / PL_BLK; }

__device__ __forceinline__ float hsin(float x) { return (float)sin((double)x); }
__device__ __forceinline__ float hpow(float x, float y) { return (float)pow((double)x, (double)y); }
// Contraction is off in every helper the init uses: frac(s·b) fused into fma(s, b, −floor(s·b))
// would return the exact fraction instead of the HLSL one (rounded product first).
__device__ __forceinline__ float frac(float x) {
#pragma clang fp contract(off)
    return x - floorf(x);
}
// frac(sin(seed * a) * b) * 2 - 1
__device__ __forceinline__ float sgn_hash(float seedf, float a, float b) {
#pragma clang fp contract(off)
    const float s = hsin(seedf * a) * b;
    return frac(s) * 2.0f - 1.0f;
}

__global__ __launch_bounds__(PL_BLK) void k_slot_map(const int32_t* __restrict__ id, int32_t n,
                                                    int32_t* __restrict__ slot_of) {
    const int32_t s = blockIdx.x * PL_BLK + threadIdx.x;
    if (s >= n) return;
    const int32_t i = id[s];
    if ((uint32_t)i < (uint32_t)n) slot_of[i] = s;
}

__global__ __launch_bounds__(PL_BLK) void k_init_sphere(int32_t n, int32_t active, InitConst c,
                                                       float4* __restrict__ pos, float4* __restrict__ vel,
                                                       float4* __restrict__ omg, float4* __restrict__ rot,
                                                       float4* __restrict__ aux, int32_t* __restrict__ mode,
                                                       int32_t* __restrict__ id, int32_t* __restrict__ torque) {
#pragma clang fp contract(off)
    const int32_t i = blockIdx.x * PL_BLK + threadIdx.x;
    if (i >= n) return;
    id[i] = i;
    if (torque) { torque[3 * i] = 0; torque[3 * i + 1] = 0; torque[3 * i + 2] = 0; }   // :193
    if (i >= active) {   // never written by InitParticles: a fresh ComputeBuffer is zero
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        pos[i] = z; vel[i] = z; omg[i] = z; rot[i] = z; aux[i] = z; mode[i] = 0;
        return;
    }
    const uint32_t seed = (uint32_t)i * 65537u + 17u;                                   // :123
    const float sf = (float)seed;
    float px = 0.f, py = 0.f, pz = 0.f;
    if (i != 0) {
        float dx = sgn_hash(sf, 12.9898f, 43758.5453f), dy = sgn_hash(sf, 78.233f, 43758.5453f),
              dz = sgn_hash(sf, 91.934f, 43758.5453f);
        float l = sqrtf(dx * dx + dy * dy + dz * dz);
        dx = dx / l; dy = dy / l; dz = dz / l;
        const float randVal = frac(hsin(sf * 1.2345f) * 10000.0f);                        // :141
        const float dist = hpow(randVal, 1.0f / 3.0f) * c.spawn_radius;
        px = dx * dist; py = dy * dist; pz = dz * dist;
        if (i > 1) {                                                                     // :147-155
            const float repelDist = hpow(0.5f * (float)i / (float)c.length, 1.0f / 3.0f) * c.spawn_radius * 0.1f;
            float ex = sgn_hash(sf, 45.678f, 43758.5453f), ey = sgn_hash(sf, 67.890f, 43758.5453f),
                  ez = sgn_hash(sf, 12.345f, 43758.5453f);
            const float m = sqrtf(ex * ex + ey * ey + ez * ez);
            ex = ex / m; ey = ey / m; ez = ez / m;
            px = px + ex * repelDist; py = py + ey * repelDist; pz = pz + ez * repelDist;
        }
    }
    const float radius = c.min_radius + frac(hsin(sf * 3.456f) * 999.0f) * (c.max_radius - c.min_radius); // :160
    const float volume = (4.0f / 3.0f) * 3.1415926f * hpow(radius, 3.0f);
    const float mass = c.density * volume;
    const float inertia = (2.0f / 5.0f) * mass * radius * radius;
    const float drag = 0.5f + frac(hsin(sf * 5.6789f) * 888.0f) * (1.0f - 0.5f);           // :166
    int32_t modeIndex = -1;                                                              // :172-186
    if (c.genome_modes > 0) {
        if (frac(hsin(sf * 78.123f) * 5432.1f) < 0.5f)
            modeIndex = c.default_mode;
        else
            modeIndex = (int32_t)(frac(hsin(sf * 43.21f) * 8765.43f) * (float)c.genome_modes);
        modeIndex = modeIndex < 0 ? 0 : (modeIndex > c.genome_modes - 1 ? c.genome_modes - 1 : modeIndex);
    }
    pos[i] = make_float4(px, py, pz, radius);
    vel[i] = make_float4(0.f, 0.f, 0.f, mass);
    omg[i] = make_float4(0.f, 0.f, 0.f, inertia);
    aux[i] = make_float4(drag, 1.0f, 0.f, 0.f);
    rot[i] = make_float4(0.f, 0.f, 0.f, 1.f);
    mode[i] = modeIndex;
}

// One split per lane. Parents are distinct and < active (checked on the host), children B
// have indices >= active, so no lane reads a record another lane writes.
__global__ __launch_bounds__(PL_BLK) void k_split(const SplitRec* __restrict__ sp, int32_t count, int32_t active,
                                                 int32_t n_old, const int32_t* __restrict__ slot_of,
                                                 float4* __restrict__ pos, float4* __restrict__ vel,
                                                 float4* __restrict__ omg, float4* __restrict__ rot,
                                                 float4* __restrict__ aux, int32_t* __restrict__ mode,
                                                 int32_t* __restrict__ id) {
    const int32_t k = blockIdx.x * PL_BLK + threadIdx.x;
    if (k >= count) return;
    const SplitRec r = sp[k];
    const int32_t sa = slot_of[r.parent];
    const float4 pa = pos[sa], va = vel[sa];
    // child A overwrites the parent (:853-857)
    pos[sa] = make_float4(r.posA[0], r.posA[1], r.posA[2], pa.w);
    vel[sa] = make_float4(r.velA[0], r.velA[1], r.velA[2], va.w);
    rot[sa] = make_float4(r.rotA[0], r.rotA[1], r.rotA[2], r.rotA[3]);
    mode[sa] = r.modeA;
    // child B = copy of child A with B's position, velocity, rotation and mode (:864-869)
    const int32_t ib = active + k;
    const int32_t sb = ib < n_old ? slot_of[ib] : ib;   // indices past the old count are new slots
    pos[sb] = make_float4(r.posB[0], r.posB[1], r.posB[2], pa.w);
    vel[sb] = make_float4(r.velB[0], r.velB[1], r.velB[2], va.w);
    omg[sb] = omg[sa];
    aux[sb] = aux[sa];
    rot[sb] = make_float4(r.rotB[0], r.rotB[1], r.rotB[2], r.rotB[3]);
    mode[sb] = r.modeB;
    id[sb] = ib;
}

// 84-byte records of particle indices [first, first+count) (grid.hip's dword layout).
__global__ __launch_bounds__(PL_BLK) void k_get_range(const float4* __restrict__ pos, const float4* __restrict__ vel,
                                                     const float4* __restrict__ omg, const float4* __restrict__ rot,
                                                     const float4* __restrict__ aux, const int32_t* __restrict__ mode,
                                                     const int32_t* __restrict__ slot_of, int32_t first, int32_t count,
                                                     uint32_t* __restrict__ aos) {
    const int32_t k = blockIdx.x * PL_BLK + threadIdx.x;
    if (k >= count) return;
    const int32_t s = slot_of[first + k];
    const float4 a = pos[s], b = vel[s], c = omg[s], d = aux[s], e = rot[s];
    const float v[20] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w,
                         d.x, d.y, d.z, d.w, e.x, e.y, e.z, e.w};
    uint32_t* p = aos + (int64_t)k * 21;
#pragma unroll
    for (int j = 0; j < 20; ++j) p[j] = __float_as_uint(v[j]);
    p[20] = (uint32_t)mode[s];
}

__global__ __launch_bounds__(PL_BLK) void k_set_range(const uint32_t* __restrict__ aos, const int32_t* __restrict__ slot_of,
                                                     int32_t first, int32_t count, float4* __restrict__ pos,
                                                     float4* __restrict__ vel, float4* __restrict__ omg,
                                                     float4* __restrict__ rot, float4* __restrict__ aux,
                                                     int32_t* __restrict__ mode) {
    const int32_t k = blockIdx.x * PL_BLK + threadIdx.x;
    if (k >= count) return;
    const int32_t s = slot_of[first + k];
    const uint32_t* p = aos + (int64_t)k * 21;
    uint32_t w[21];
#pragma unroll
    for (int j = 0; j < 21; ++j) w[j] = p[j];
    auto f = [&](int j) { return __uint_as_float(w[j]); };
    pos[s] = make_float4(f(0), f(1), f(2), f(3));
    vel[s] = make_float4(f(4), f(5), f(6), f(7));
    omg[s] = make_float4(f(8), f(9), f(10), f(11));
    aux[s] = make_float4(f(12), f(13), f(14), f(15));
    rot[s] = make_float4(f(16), f(17), f(18), f(19));
    mode[s] = (int32_t)w[20];
}

void launch_slot_map(const int32_t* id, int32_t n, int32_t* slot_of, hipStream_t s) {
    if (n > 0) k_slot_map<<<nblk_pl(n), PL_BLK, 0, s>>>(id, n, slot_of);
}
void launch_init_sphere(int32_t n, int32_t active, InitConst c, float4* pos, float4* vel, float4* omg, float4* rot,
                        float4* aux, int32_t* mode, int32_t* id, int32_t* torque, hipStream_t s) {
    if (n > 0) k_init_sphere<<<nblk_pl(n), PL_BLK, 0, s>>>(n, active, c, pos, vel, omg, rot, aux, mode, id, torque);
}
void launch_split(const SplitRec* sp, int32_t count, int32_t active, int32_t n_old, const int32_t* slot_of,
                  float4* pos, float4* vel, float4* omg, float4* rot, float4* aux, int32_t* mode, int32_t* id,
                  hipStream_t s) {
    if (count > 0)
        k_split<<<nblk_pl(count), PL_BLK, 0, s>>>(sp, count, active, n_old, slot_of, pos, vel, omg, rot, aux, mode, id);
}
void launch_get_range(const float4* pos, const float4* vel, const float4* omg, const float4* rot, const float4* aux,
                      const int32_t* mode, const int32_t* slot_of, int32_t first, int32_t count, void* aos,
                      hipStream_t s) {
    if (count > 0)
        k_get_range<<<nblk_pl(count), PL_BLK, 0, s>>>(pos, vel, omg, rot, aux, mode, slot_of, first, count,
                                                      (uint32_t*)aos);
}
void launch_set_range(const void* aos, const int32_t* slot_of, int32_t first, int32_t count, float4* pos,
                      float4* vel, float4* omg, float4* rot, float4* aux, int32_t* mode, hipStream_t s) {
    if (count > 0)
        k_set_range<<<nblk_pl(count), PL_BLK, 0, s>>>((const uint32_t*)aos, slot_of, first, count, pos, vel, omg,
                                                      rot, aux, mode);
}

}  // namespace sph
