// wcsph.hip — Model S neighbour passes (SPEC_SPH.md §2) for gfx950.
//
// The reference has no SPH arithmetic. Its only neighbour pass,
// ApplySPHForces (SimulateParticles.compute:211-309), walks 27 linked lists per particle.
// Here every particle walks the 9 contiguous rows of its 3x3x3 cell block in the
// cell-sorted arrays (SPEC_SPH.md §0), so candidates come in index order from a few
// cache lines. No MFMA: the neighbour sum is a gather.
//
//   k_density          ρ_i = Σ m W, Tait EOS → (ρ, P/ρ²)            reads x (16 B), writes 8 B
//   k_force_integrate  pressure + Monaghan viscosity + XSPH, KDK kick-drift, box walls,
//                      and the next step's cell key                 reads x,v,ρ,P/ρ² (40 B),
//                                                                    writes x,v,key (36 B)
#include "common.h"

namespace sph {

constexpr int NB_BLK = 256;

// The 9 neighbour rows (SPEC_SPH.md §0) of a particle at (x,y,z), each trimmed to its z window.
struct RowIter {
    int32_t cx, cy;
    float fx, fy, gzf;
};

__device__ __forceinline__ RowIter row_iter(const GridDesc& g, float x, float y, float z) {
    RowIter it;
    it.cx = cell_cx(g, x);
    it.cy = cell_coord(y, g.oy, g.inv_cell, g.gy);
    cell_fracs(g, x, y, z, it.cx, it.cy, it.fx, it.fy, it.gzf);
    return it;
}

// Row k (0..8, dx-major) as a sorted-index range; false if the row is outside the grid or ≥ 2h away.
__device__ __forceinline__ bool row_range(const GridDesc& g, const uint32_t* __restrict__ cs,
                                          const RowIter& it, int k, uint32_t& j0, uint32_t& j1) {
    const int dx = k / 3 - 1, dy = k % 3 - 1;
    const int32_t xx = it.cx + dx, yy = it.cy + dy;
    if (xx < 0 || xx >= g.gx || yy < 0 || yy >= g.gy) return false;
    int32_t zlo, zhi;
    if (!row_window(g, it.fx, it.fy, it.gzf, dx, dy, zlo, zhi)) return false;
    const uint32_t rowk = ((uint32_t)xx * (uint32_t)g.gy + (uint32_t)yy) * (uint32_t)g.gz;
    j0 = cs[rowk + (uint32_t)zlo];
    j1 = cs[rowk + (uint32_t)zhi + 1u];
    return true;
}

// cubic spline W and F = (1/r) dW/dr (SPEC_SPH.md §2); fast v_sqrt / v_rcp
__device__ __forceinline__ void spline(const SphConst& c, float r2, float& W, float& F) {
    const float r = __builtin_amdgcn_sqrtf(r2);
    const float q = r * c.inv_h;
    const float t = 2.0f - q;
    if (q < 1.0f) {
        W = c.sigma * (1.0f + q * q * (-1.5f + 0.75f * q));
        F = c.sigma_h2 * (-3.0f + 2.25f * q);
    } else {
        W = c.sigma * (0.25f * t * t * t);
        F = -c.sigma_h * 0.75f * t * t * __builtin_amdgcn_rcpf(r);
    }
}

__global__ __launch_bounds__(NB_BLK) void k_density(const float4* __restrict__ pos,
                                                    const uint32_t* __restrict__ cs, int32_t ib, int32_t n,
                                                    GridDesc g, SphConst c, float2* __restrict__ rp, DevRange dr) {
    if (dr.lo) {
        ib = (int32_t)*dr.lo;
        n = (int32_t)*dr.hi;
    }
    const int32_t i = ib + blockIdx.x * NB_BLK + threadIdx.x;
    if (i >= n) return;
    const float4 pi = pos[i];
    const RowIter it = row_iter(g, pi.x, pi.y, pi.z);
    float s = 0.0f;
#pragma unroll 1
    for (int k = 0; k < 9; ++k) {
        uint32_t j0, j1;
        if (!row_range(g, cs, it, k, j0, j1)) continue;
#pragma unroll 2
        for (uint32_t j = j0; j < j1; ++j) {
            const float4 pj = pos[j];
            const float dx = pi.x - pj.x, dy = pi.y - pj.y, dz = pi.z - pj.z;
            const float r2 = dx * dx + dy * dy + dz * dz;
            if (r2 < c.four_h2) {
                const float r = __builtin_amdgcn_sqrtf(r2);
                const float q = r * c.inv_h;
                const float t = 2.0f - q;
                const float w = q < 1.0f ? 1.0f + q * q * (-1.5f + 0.75f * q) : 0.25f * t * t * t;
                s += w;
            }
        }
    }
    const float d = c.mass * (c.sigma * s);
    const float tr = d * c.inv_rho0;
    const float t2 = tr * tr, t4 = t2 * t2;
    const float P = c.B * (t4 * t2 * tr - 1.0f);
    rp[i] = make_float2(d, P / (d * d));
}

__global__ __launch_bounds__(NB_BLK) void k_force_integrate(
    const float4* __restrict__ pos, const float4* __restrict__ vel, const float2* __restrict__ rp,
    const uint32_t* __restrict__ cs, int32_t ib, int32_t n, GridDesc g, SphConst c, float dt, float fext_x,
    float4* __restrict__ pos_o, float4* __restrict__ vel_o, uint32_t* __restrict__ keys_o, MoverSink mv) {
    const int32_t i = ib + blockIdx.x * NB_BLK + threadIdx.x;
    if (i >= n) return;
    const float4 pi = pos[i];
    const float4 vi = vel[i];
    const float2 ri = rp[i];
    const RowIter it = row_iter(g, pi.x, pi.y, pi.z);
    float ax = 0.f, ay = 0.f, az = 0.f, sx = 0.f, sy = 0.f, sz = 0.f;
    const float m = c.mass;
#pragma unroll 1
    for (int k = 0; k < 9; ++k) {
        uint32_t j0, j1;
        if (!row_range(g, cs, it, k, j0, j1)) continue;
#pragma unroll 2
        for (uint32_t j = j0; j < j1; ++j) {
            const float4 pj = pos[j];
            const float dx = pi.x - pj.x, dy = pi.y - pj.y, dz = pi.z - pj.z;
            const float r2 = dx * dx + dy * dy + dz * dz;
            if (r2 < c.four_h2 && (int32_t)j != i) {
                const float4 vj = vel[j];
                const float2 rj = rp[j];
                float W, F;
                spline(c, r2, W, F);
                const float du = vi.x - vj.x, dv = vi.y - vj.y, dw = vi.z - vj.z;
                const float vr = du * dx + dv * dy + dw * dz;
                const float inv_rbar = __builtin_amdgcn_rcpf(0.5f * (ri.x + rj.x));
                const float mu = c.h * vr * __builtin_amdgcn_rcpf(r2 + c.eta2);
                const float pij = vr < 0.0f ? -c.ac0 * mu * inv_rbar : 0.0f;
                const float cf = -m * (ri.y + rj.y + pij) * F;
                ax += cf * dx; ay += cf * dy; az += cf * dz;
                const float cx = c.eps * m * inv_rbar * W;
                sx -= cx * du; sy -= cx * dv; sz -= cx * dw;
            }
        }
    }
    // KDK leapfrog, kick-drift form (SPEC_SPH.md §2), then box walls
    float nv[3] = {vi.x + (ax + c.gx + fext_x) * dt, vi.y + (ay + c.gy) * dt, vi.z + (az + c.gz) * dt};
    float np[3] = {pi.x + (nv[0] + sx) * dt, pi.y + (nv[1] + sy) * dt, pi.z + (nv[2] + sz) * dt};
    const float L[3] = {c.Lx, c.Ly, c.Lz};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (np[a] < 0.0f) { np[a] = 0.0f; if (nv[a] < 0.0f) nv[a] = -c.wall_e * nv[a]; }
        if (np[a] > L[a]) { np[a] = L[a]; if (nv[a] > 0.0f) nv[a] = -c.wall_e * nv[a]; }
    }
    pos_o[i] = make_float4(np[0], np[1], np[2], 0.f);
    vel_o[i] = make_float4(nv[0], nv[1], nv[2], 0.f);
    const uint32_t key = cell_key(g, np[0], np[1], np[2]);
    keys_o[i] = key;
    // the mover list takes the window key: in a slab, a particle that left the held columns sorts
    // last (window_key = cell_key in a single domain); it changed iff the clamped key changed
    append_mover(mv, i, window_key(g, np[0], np[1], np[2]));
}

// dr set: [ib, ie) only sizes the grid (an upper bound); the kernel reads its bounds from dr
void launch_density(const float4* pos, const uint32_t* cs, int32_t ib, int32_t ie, GridDesc g, SphConst c,
                    float2* rp, hipStream_t s, DevRange dr) {
    if (ie > ib) k_density<<<(ie - ib + NB_BLK - 1) / NB_BLK, NB_BLK, 0, s>>>(pos, cs, ib, ie, g, c, rp, dr);
}

void launch_force_integrate(const float4* pos, const float4* vel, const float2* rp, const uint32_t* cs, int32_t ib,
                            int32_t ie, GridDesc g, SphConst c, float dt, float fext_x, float4* pos_o,
                            float4* vel_o, uint32_t* keys_o, MoverSink mv, hipStream_t s) {
    if (ie > ib)
        k_force_integrate<<<(ie - ib + NB_BLK - 1) / NB_BLK, NB_BLK, 0, s>>>(pos, vel, rp, cs, ib, ie, g, c, dt,
                                                                             fext_x, pos_o, vel_o, keys_o, mv);
}

}  // namespace sph
