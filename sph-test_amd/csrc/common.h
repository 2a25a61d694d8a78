// common.h — internal declarations shared by the HIP kernels and the C ABI (libsphhip.so).
// Not part of the public ABI (that is include/sphhip.h). gfx950 / wave64 only.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

namespace sph {

// Uniform grid (SPEC_SPH.md §0). key = (cx*gy + cy)*gz + cz, x slowest.
// A context may hold an x-window [cx0, cx0+gx) of a global grid of gx_all columns (slab
// decomposition, SPEC_SPH.md §3). The column is computed globally then shifted, so all
// ranks agree bit for bit on which column a particle is in.
// Model S splits z into zsub sub-cells (cells 2h × 2h × 2h/zsub, SPEC_SPH.md §0): each of the
// neighbour rows is then walked over a z window trimmed to the row's xy distance. It may also split
// each column into xsub x sub-columns (cells cell/xsub wide in x): keys then count sub-columns,
// key = ((cxs*gy + cy)*gz + cz with cxs = xsub*cx + the sub-column, so a column is still one
// contiguous run of xsub*gy*gz keys (col_keys) and the slab decomposition keeps whole columns.
struct GridDesc {
    float ox, oy, oz;
    float inv_cell;      // 1 / cell (x, y)
    float inv_cz;        // 1 / (cell / zsub) (z)
    int32_t gx, gy, gz;  // gx counts columns (cell wide), gz z sub-cells
    uint32_t ncells;     // gx*xsub*gy*gz (keys == ncells mark inactive particles)
    int32_t cx0;         // first global column held (0 without decomposition)
    int32_t gx_all;      // global column count (== gx without decomposition)
    int32_t zsub;        // z sub-cells per cell (Model S 3D 6, Model R and 2D 1)
    int32_t zwin;        // max |Δ z sub-cell| of a neighbour (zsub + 1; Model R 1)
    int32_t xsub;        // x sub-columns per column (Model S 3D: SPH_XSUB; Model R and 2D 1)
    float inv_cxs;       // xsub / cell (x sub-column coordinate; == inv_cell when xsub = 1)
};
#if defined(__HIPCC__)
#define SPH_HD __host__ __device__
#else
#define SPH_HD
#endif
// keys per column (the slab decomposition's column of keys)
template <int XS = 0>
SPH_HD inline uint32_t col_keys(const GridDesc& g) { return (uint32_t)(XS ? XS : g.xsub) * (uint32_t)g.gy * (uint32_t)g.gz; }

// Model S constants (SPEC_SPH.md §2), derived on the host from sph_params.
struct SphConst {
    float mass, four_h2, inv_h, sigma, sigma_h, sigma_h2;
    float B, inv_rho0, h, eta2, ac0, eps;
    float gx, gy, gz;
    float Lx, Ly, Lz;
    float wall_e;
    float inv_h2;   // 1/h², the neighbour passes' q = sqrt(r²/h²)
    // the neighbour passes in units of r (wcsph_tiled.hip SPH_RUNITS): 2h, −6h, 4h³ and the density scale m·σ/(4h³)
    float two_h, m6h, four_h3, rho_scale;
};

// Model R uniforms (SimulateParticles.compute:89-100) + DragInput (:70-74).
struct ContactConst {
    float dt, spawn_radius, global_drag, torque_factor, torque_damping, boundary_friction;
    float roll_mult, repulsion_strength;
    int32_t drag_id;
    float drag_tx, drag_ty, drag_tz, drag_strength;
    // device word: an upper bound of every radius (float bits, k_keys on the full sort after any change of the
    // particles; +inf until then). The contact pass skips the cells of its 27 that lie beyond rA/2 + rmax/2. null: none
    const uint32_t* rmax = nullptr;
    // its value, read by each contact kernel at its start with its first loads (contact.hip rmax_load): read where the
    // cell reach is computed, the load waited one more memory round trip in every target's chain
    float rmv = __builtin_inff();
};
constexpr int SDEV_RMAX = 15;   // sph_ctx::sdev word holding ContactConst::rmax (Model R)

#if defined(__HIPCC__)
// A word another launch wrote (a count, a range key), read through the vector memory path with the default cache policy.
// A uniform address otherwise becomes a scalar load, and the wait for the kernel arguments' scalar loads (lgkmcnt,
// which cannot tell them apart) then also waits for it: the loads that follow issued one memory round trip late.
// The zero offset comes from a VGPR the compiler cannot see through (vzero; one for several loads keeps them together).
__device__ __forceinline__ uint32_t vzero() {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}
__device__ __forceinline__ uint32_t ld_vec(const uint32_t* p) { return p[vzero()]; }

__device__ __forceinline__ int32_t cell_coord(float x, float o, float inv, int32_t G) {
    // GetGridCoord (compute:102-105): (uint)((p - origin) * inv) with ftou (neg/NaN -> 0), clamp
    float g = (x - o) * inv;
    if (!(g > 0.0f)) return 0;
    if (g >= (float)(G - 1)) return G - 1;
    return (int32_t)g;
}

// local x column of a position (global column - cx0, clamped to the held window)
__device__ __forceinline__ int32_t cell_cx(const GridDesc& g, float x) {
    const int32_t c = cell_coord(x, g.ox, g.inv_cell, g.gx_all) - g.cx0;
    return c < 0 ? 0 : (c >= g.gx ? g.gx - 1 : c);
}

// local x sub-column of a position (xsub per column). inv_cxs = xsub · inv_cell exactly, so the global
// sub-column is xsub · (global column) + [0, xsub) for every x, clamping included: keys / col_keys
// give the column of cell_cx. XS: xsub as a compile-time constant (0: read it from the grid).
template <int XS = 0>
__device__ __forceinline__ int32_t cell_cxs(const GridDesc& g, float x) {
    const int32_t xs = XS ? XS : g.xsub;
    const float inv = XS == 1 ? g.inv_cell : g.inv_cxs;
    const int32_t c = cell_coord(x, g.ox, inv, g.gx_all * xs) - g.cx0 * xs;
    const int32_t m = g.gx * xs;
    return c < 0 ? 0 : (c >= m ? m - 1 : c);
}

template <int XS = 0>
__device__ __forceinline__ uint32_t cell_key(const GridDesc& g, float x, float y, float z) {
    int32_t cx = cell_cxs<XS>(g, x);
    int32_t cy = cell_coord(y, g.oy, g.inv_cell, g.gy);
    int32_t cz = cell_coord(z, g.oz, g.inv_cz, g.gz);
    return ((uint32_t)cx * (uint32_t)g.gy + (uint32_t)cy) * (uint32_t)g.gz + (uint32_t)cz;
}

// slab: a particle outside the held columns (already sent away) gets key ncells: it sorts last
template <int XS = 0>
__device__ __forceinline__ uint32_t window_key(const GridDesc& g, float x, float y, float z) {
    const int32_t c = cell_coord(x, g.ox, g.inv_cell, g.gx_all) - g.cx0;
    return (c < 0 || c >= g.gx) ? g.ncells : cell_key<XS>(g, x, y, z);
}

// One of the (2·xsub+1)·3 neighbour rows of a Model S particle (SPEC_SPH.md §0): the z sub-cell window
// [zlo, zhi] of row (cxs+dx, cy+dy) (dx in sub-columns, |dx| <= xsub) that can hold a particle within
// 2h, or false when the row's column is ≥ 2h away in xy. fx: the particle's position inside its
// sub-column, fy inside its cell, in [0,1]. The x gap is counted in sub-columns and scaled by 1/xsub
// (exact; with xsub = 1 the arithmetic is the 3 x 3 rows' of SPEC_SPH.md §0 to the bit).
// XS: the grid's xsub as a compile-time constant (the neighbour passes are instantiated per xsub).
template <int XS>
__device__ __forceinline__ bool row_window(const GridDesc& g, float fx, float fy, float gzf, int dx, int dy,
                                           int32_t& zlo, int32_t& zhi) {
    float gxg;
    if constexpr (XS == 1) {
        gxg = dx < 0 ? fx : (dx > 0 ? 1.0f - fx : 0.0f);
    } else {
        gxg = (dx < 0 ? fx + (float)(-dx - 1) : (dx > 0 ? (1.0f - fx) + (float)(dx - 1) : 0.0f)) * (1.0f / XS);
    }
    const float gyg = dy < 0 ? fy : (dy > 0 ? 1.0f - fy : 0.0f);
    const float d2 = fmaf(gyg, gyg, gxg * gxg);   // explicit: both passes must trim every window identically
    if (!(d2 < 1.0f)) return false;
    const float hz = __builtin_amdgcn_sqrtf(1.0f - d2) * (float)g.zsub + 1e-3f;
    const float a = gzf - hz, b = gzf + hz;
    zlo = a > 0.0f ? (int32_t)a : 0;
    zhi = b < (float)(g.gz - 1) ? (int32_t)b : g.gz - 1;
    if (zhi < 0) zhi = 0;
    return true;
}

// The particle's in-cell fractions (x in its sub-column cxs, y) and z sub-cell coordinate for row_window.
template <int XS = 0>
__device__ __forceinline__ void cell_fracs(const GridDesc& g, float x, float y, float z, int32_t cxs, int32_t cy,
                                           float& fx, float& fy, float& gzf) {
    const int32_t xs = XS ? XS : g.xsub;
    const float inv = XS == 1 ? g.inv_cell : g.inv_cxs;
    fx = fminf(fmaxf((x - g.ox) * inv - (float)(cxs + g.cx0 * xs), 0.0f), 1.0f);
    fy = fminf(fmaxf((y - g.oy) * g.inv_cell - (float)cy, 0.0f), 1.0f);
    gzf = (z - g.oz) * g.inv_cz;
}

// Workgroups are dispatched round-robin over the 8 XCDs, each with its own L2
// (MI355X_MICROARCH.md). Remapped so that each XCD runs groups of SPH_XCD_CHUNK consecutive logical
// blocks: neighbouring blocks stage the same neighbour rows and then share one L2 instead of
// fetching them 8 times, while dealing the runs round-robin keeps the eight XCDs on equally dense
// parts of the fluid. One contiguous range per XCD (SPH_XCD_CHUNK=0) left XCDs with sparse or
// surface-heavy ranges idle at the end: C3 force pass 250 -> 238 us with runs of 16
// (profiles/r01_xcd_map_ab.log; 8 and 32 are within noise of 16, 4 and 64 are slower).
#ifndef SPH_XCD_CHUNK
#define SPH_XCD_CHUNK 16
#endif
__device__ __forceinline__ int32_t xcd_block(int32_t b, int32_t nb) {
    constexpr int32_t NX = 8;
#if SPH_XCD_CHUNK < 0   // A/B: dispatch order
    return b;
#elif SPH_XCD_CHUNK > 0   // runs of C consecutive blocks dealt round-robin to the XCDs (the tail: dispatch order)
    constexpr int32_t C = SPH_XCD_CHUNK;
    const int32_t full = nb / (NX * C) * (NX * C);
    if (b >= full) return b;
    const int32_t x = b % NX, k = b / NX;
    return ((k / C) * NX + x) * C + (k % C);
#else   // A/B: one contiguous range per XCD
    const int32_t x = b % NX, k = b / NX, per = nb / NX, rem = nb % NX;
    return x * per + (x < rem ? x : rem) + k;
#endif
}

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Inclusive sum inside each row of 16 lanes by DPP row shifts (lanes 0-15: the scan of lanes 0-15)
__device__ __forceinline__ uint32_t row_scan_incl(uint32_t x) {
    const uint32_t rl = lane_id() & 15u;
    uint32_t t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
    if (rl >= 1u) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x112, 0xf, 0xf, false);            // row_shr:2
    if (rl >= 2u) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x114, 0xf, 0xf, false);            // row_shr:4
    if (rl >= 4u) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x118, 0xf, 0xf, false);            // row_shr:8
    if (rl >= 8u) x += t;
    return x;
}

// Inclusive sum over the wave's 64 lanes by DPP moves (row shifts by 1, 2, 4, 8 inside rows of 16, then the row
// broadcasts of lanes 15 and 31): six VALU-latency steps, where a shuffle scan (ds_bpermute) waits an LDS round trip
// at each of its six steps
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    const uint32_t lane = lane_id(), rl = lane & 15u;
    uint32_t t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
    if (rl >= 1u) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x112, 0xf, 0xf, false);            // row_shr:2
    if (rl >= 2u) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x114, 0xf, 0xf, false);            // row_shr:4
    if (rl >= 4u) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x118, 0xf, 0xf, false);            // row_shr:8
    if (rl >= 8u) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x142, 0xf, 0xf, false);            // row_bcast:15
    if ((lane & 31u) >= 16u) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x143, 0xf, 0xf, false);            // row_bcast:31
    if (lane >= 32u) x += t;
    return x;
}

// Per-kernel timing without extra packets in the stream. While a timing scope (host.h KTimer,
// profiling on) is open, the launches inside it carry the scope's events in their own dispatch
// packets (hipExtLaunchKernel): the first launch the start event, every launch the stop event (the last
// one's end wins). Recording the events with hipEventRecord around each scope instead put ~10 us of
// idle time between consecutive kernels (0.373 -> 0.396 ms per C3 step with three scopes per step).
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
    int launches = 0;
};
extern thread_local LaunchEvents* g_launch_events;
#define SPH_LAUNCH(kernel, grid, block, shmem, stream, ...)                                                  \
    do {                                                                                                     \
        LaunchEvents* le_ = g_launch_events;                                                                 \
        if (le_) {                                                                                           \
            hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(block), (uint32_t)(shmem), stream,                \
                                  le_->launches == 0 ? le_->start : nullptr, le_->stop, 0u, __VA_ARGS__);    \
            ++le_->launches;                                                                                 \
        } else {                                                                                             \
            kernel<<<grid, block, shmem, stream>>>(__VA_ARGS__);                                             \
        }                                                                                                    \
    } while (0)

#endif

// Slot bounds held in device memory (slab mode: known on the device before the host reads
// them back). lo == nullptr: use the launch's host bounds.
struct DevRange {
    const uint32_t* lo = nullptr;
    const uint32_t* hi = nullptr;
};

// The slab step's send blocks: the count / pack pair takes SEND_SLOTS consecutive owned slots per workgroup (slab.hip):
// SPH_SL_PER slots per thread of 256.
#ifndef SPH_SL_PER
#define SPH_SL_PER 16
#endif
constexpr int32_t SEND_SLOTS = 256 * SPH_SL_PER;
// Early sends (abi_multi.cpp phase_boundary): the boundary force pass counts the next step's sends itself, per send
// block, into bins[side * nblk + block] (zeroed by the step's k_slab_lag after the pack has read them). Range r of the
// launch (0: dr, 1: dr2) starts a side's send range and counts for side[r] (−1: none): new column <= col_le (left)
// or >= col_ge (right).
struct SendBins {
    uint32_t* bins = nullptr;   // null: no count
    int32_t nblk = 0;
    int32_t side[2] = {-1, -1};
    int32_t col_le = 0, col_ge = 0;
};

// The in-library slab step (abi_multi.cpp) keeps every per-step size on the device: the counts of
// the halo messages arrive in their headers, the slot ranges come out of the re-sort's cell table,
// and every kernel reads them here (launch grids are host upper bounds). No host read per step.
struct SlabSizes {
    uint32_t nl, nr;          // records taken from the left / right message (clamped to capacity)
    uint32_t o0, o1;          // owned slots of the previous sorted order
    uint32_t no, n;           // o1 - o0; assembled slots nl + no + nr
    uint32_t pick[8];         // column starts of the new order (launch_resort's CsPick): columns 0, lo, lo+1,
                              // hi-1, hi, gx (local), then lo+2 and hi-2 (clamped into [lo, hi]): the send candidates
    uint32_t rg[10];          // ghost-left [0,1), owned [2,3), ghost-right [4,5), boundary columns [6,7), [8,9)
    uint32_t fr[6];           // force pass: interior [0,1), boundary [2,3) and [4,5)
    uint32_t dropped;         // own particles the assemble dropped (left the held window)
    uint32_t flags;           // sticky: SZ_* bits
    uint32_t jump;            // this step's force pass moved an own particle by more than one column (the next
                              // step's sends then scan every own slot; cleared when the sizes are derived)
    uint32_t hl_raw, hr_raw;  // this step's received message header counts (before clamping), for k_slab_lag
};
constexpr uint32_t SZ_OVF_MSG = 1u;     // a halo message held more records than its capacity
constexpr uint32_t SZ_OVF_CAP = 2u;     // the assembled slots exceed the context's capacity
constexpr uint32_t SZ_RHO_MISMATCH = 4u;  // a ghost column and the densities received differ in count
constexpr uint32_t SZ_OVF_MOVERS = 8u;    // a mover list or a re-sort destination past the slot capacity
constexpr uint32_t SZ_JUMP = 16u;         // an own particle left the held window in one step (two columns or more)
constexpr uint32_t SZ_JUMP_EARLY = 32u;   // early sends: an interior particle moved two or more columns in one step
constexpr int SZ_BITS = 6;
// Halo messages: one 32-byte header record, then the records. Header: (count, capacity, 0, 0 | 0...)
constexpr int MSG_HDR_F4 = 2;
// ρ halo messages: a 32-byte header (count, capacity) = 4 float2, then (ρ, P/ρ²) of the boundary column's slots
constexpr int RHO_HDR = 4;
// The slab step's ρ messages, written by the density pass itself (k_density_tiled): side s carries the own
// boundary column [pick[1 + 2s], pick[2 + 2s]) in slot order. msg[s] null: no neighbour on that side.
struct RhoOut {
    float2* msg[2] = {nullptr, nullptr};
    int32_t cap[2] = {0, 0};
    const SlabSizes* dz = nullptr;
    uint32_t* fbits = nullptr;   // RCCL step: dz->flags, one word per SZ_* bit, for the ranks' OR (abi_multi.cpp)
};
// What the assembled layout is computed from: the two message headers (null: no neighbour), the
// capacities they were sent with, and the context's slot capacity.
struct SizesIn {
    const float4* hl;
    const float4* hr;
    int32_t cap_l, cap_r, capacity;
};
#if defined(__HIPCC__)
__device__ __forceinline__ uint32_t header_count(const float4* msg) { return __float_as_uint(msg[0].x); }
// nl, no, nr and the flags of the assembled [left | own | right] (slab.hip k_slab_sizes; k_slab_rec)
__device__ __forceinline__ void slab_sizes_from(const SlabSizes* dz, const SizesIn& in, uint32_t& nl, uint32_t& no,
                                                uint32_t& nr, uint32_t& f, uint32_t& hl, uint32_t& hr) {
    hl = in.hl ? header_count(in.hl) : 0u;
    hr = in.hr ? header_count(in.hr) : 0u;
    nl = min(hl, (uint32_t)in.cap_l);
    nr = min(hr, (uint32_t)in.cap_r);
    f = dz->flags;
    if (hl > (uint32_t)in.cap_l || hr > (uint32_t)in.cap_r) f |= SZ_OVF_MSG;
    no = dz->o1 >= dz->o0 ? dz->o1 - dz->o0 : 0u;
    if ((uint64_t)nl + no + nr > (uint64_t)in.capacity) {   // never address past the slot arrays
        f |= SZ_OVF_CAP;
        nl = nr = 0;
        if (no > (uint32_t)in.capacity) no = 0;
    }
}
__device__ __forceinline__ void slab_sizes_store(SlabSizes* dz, uint32_t nl, uint32_t no, uint32_t nr, uint32_t f,
                                                 uint32_t hl, uint32_t hr) {
    dz->hl_raw = hl;
    dz->hr_raw = hr;
    dz->nl = nl;
    dz->nr = nr;
    dz->no = no;
    dz->n = nl + no + nr;
    dz->jump = 0u;             // read by this step's sends (before); set again by its force pass (after)
    atomicOr(&dz->flags, f);   // other workgroups of k_slab_rec may be setting SZ_OVF_MOVERS meanwhile
}
#endif

// Movers of a Model S step (resort.hip): particles whose new cell key differs from the sorted key
// of their slot. The force pass appends them (any order) for the incremental re-sort.
struct MoverSink {
    const uint32_t* sk;   // sorted keys of the slot order; nullptr: no append
    uint32_t* count;      // this step's mover counter (zero on entry)
    uint32_t* mi;         // slot index
    uint32_t* mk;         // new key
    uint32_t* mo;         // old key
    uint32_t cap;
    uint32_t* err = nullptr;   // SZ_OVF_MOVERS is or-ed here if the list would pass cap (entries dropped)
    uint32_t* jump = nullptr;  // slab step: SlabSizes.jump (a column jump > 1), SZ_JUMP into err (window exit)
    int32_t jump_err = 0;      // early sends (abi_multi.cpp): a column jump > 1 is SZ_JUMP_EARLY in err, not jump
};

#if defined(__HIPCC__)
// Called by every lane that holds a particle (lanes past n have returned): one atomic per wave.
__device__ __forceinline__ void append_mover(const MoverSink& s, int32_t i, uint32_t key) {
    if (!s.sk) return;
    const uint32_t ko = s.sk[i];
    const bool mv = key != ko;
    const uint64_t b = __ballot(mv);
    if (b == 0) return;
    const int leader = __builtin_ctzll(b);
    uint32_t base = 0;
    if ((int)lane_id() == leader) base = atomicAdd(s.count, (uint32_t)__popcll(b));
    base = __shfl(base, leader, 64);
    if (mv) {
        const uint32_t r = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        if (r >= s.cap) {   // a corrupted counter: never write past the lists
            if (s.err) atomicOr(s.err, SZ_OVF_MOVERS);
            return;
        }
        s.mi[r] = (uint32_t)i;
        s.mk[r] = key;
        s.mo[r] = ko;
    }
}
#endif

// ---- host-side launchers (each .hip file) ----
// radix sort (sort.hip)
size_t radix_hist_elems(int32_t capacity);
// Sort (keys_a, vals_a) by the low key_bits bits, stable. identity_vals: vals_a is not read,
// the input values are the slot indices. Ping-pongs between a and b; returns 1 if the
// result is in (keys_b, vals_b), 0 if in (keys_a, vals_a).
int radix_sort(uint32_t* keys_a, uint32_t* vals_a, uint32_t* keys_b, uint32_t* vals_b, int32_t n,
               int32_t key_bits, bool identity_vals, uint32_t* hist, uint32_t* bin_total,
               hipStream_t s);
// one-workgroup LDS sort (sort_small.hip), used by radix_sort for n <= SORT_SMALL_N, key_bits <= 16
// and identity values; the result goes to keys_out / vals_out
constexpr int32_t SORT_SMALL_N = 16384;
void launch_sort_small(const uint32_t* keys_in, int32_t n, int32_t key_bits, uint32_t* keys_out, uint32_t* vals_out,
                       hipStream_t s);

// incremental re-sort of a Model S step (resort.hip), from the movers the force pass appended.
// sk: sorted keys of the slot order; cs: its cell starts, updated in place; count: the movers'
// counter, count_other: the next step's counter (zeroed here). Writes the re-sorted state to *_o.
struct ResortScratch {
    uint32_t *mi, *mk, *mo;          // appended movers (MoverSink)
    uint64_t* ms;                    // movers by (new key, slot)
    uint32_t *mx, *mos;              // movers by slot: slot, old key
    uint32_t cap;
    int32_t mi_off;                  // slab step: an own mover's slot is mi + mi_off (MV_REC: records' slot)
    const SlabSizes* dz = nullptr;   // non-null: mi_off = nl - o0 from the device sizes
    uint32_t* err = nullptr;         // SZ_OVF_MOVERS if a destination would pass cap (never written)
    uint32_t* host_count = nullptr;  // mapped host memory: k_mv_rank stores the mover count there (the host's sort choice)
    uint32_t* stats = nullptr;       // [8] the re-sort's path counters (resort.hip RS_*; sph_read_resort_counts)
};
// a mover entry whose mi has this bit holds a slot of the assembled array (a halo record's);
// without it, mi is the force pass's slot and the assembled slot is mi + mi_off
constexpr uint32_t MV_REC = 0x80000000u;
// The slot array the re-sort reads, slot x in [0, n). Single domain: pos/vel/id/sk[x]. Slab step:
// the assembled [from left | own | from right] without copying it: x < nl is left record rl[x],
// x >= nre is right record rr[x - nre] (32-B halo records, old keys in skr[x]), and the own block
// is pos/vel/id/sk[x + o_off] (its slots in the previous sorted array).
struct AsmSrc {
    const float4* pos;
    const float4* vel;
    const int32_t* id;
    const uint32_t* sk;     // old (sorted) keys of the own slots
    const uint32_t* keys;   // new keys of the own slots (the force pass's)
    int32_t o_off;
    const float4* rl;
    const float4* rr;
    const uint32_t* skr;    // records: old keys, by assembled slot
    const uint32_t* keyr;   // records: new keys, by assembled slot
    int32_t nl, nre;
    const SlabSizes* dz;    // non-null: nl, nre, o_off (and the slot count) live on the device
};
// The old cell-start table of the assembled layout (slab.hip k_slab_cs_old), as extra workgroups of a launch.
struct CsOld {
    uint32_t* cs = nullptr;   // null: none
    uint32_t ncells = 0, gyz = 0, gx = 0;
    int32_t has_left = 0, has_right = 0;
    const uint32_t* src = nullptr;   // the previous table when it is not cs itself (then every cell is written)
};
#if defined(__HIPCC__)
// The cell-start table of the assembled old keys [left | own | right], for the incremental re-sort, made from the
// previous step's table in place (or, with CsOld.src, into a second table while passes still read the first), by the
// workgroup `blk` (four cells per lane; 1,024 per workgroup). Owned columns:
// the own block kept its order, so cs[k] shifts by nl − o0 (o0: the previous owned start), one 16-byte load and
// store per lane (the table is ~15 MB at C3). cs[ncells] = cs[ncells + 1] = n. Halo columns: the lower bound of
// cell k in its block's sorted old keys key(side, t): the workgroup stages every S-th key in LDS (S >= 64, at most
// CS_SAMP samples), finds from them a record window holding the lower bounds of all its cells, stages that
// window's keys (eight loads in flight per lane) and searches in LDS: about three global round trips. Measured
// against (profiles/r04_slab_trace.log, C3 x 4): a binary search per cell in global memory, 16 dependent loads
// (11 us per launch), and a gap fill by one lane per record (225 us: a lane before an empty stretch of rows
// writes thousands of cells alone).
constexpr int CS_SAMP = 1024;
constexpr int CS_WIN = 6144;
template <typename K>
__device__ __forceinline__ void cs_old_block(const CsOld& p, uint32_t blk, uint32_t nl, uint32_t no, uint32_t nr,
                                             int32_t shift, K key, uint32_t* samp, uint32_t* win) {
    const uint32_t n = nl + no + nr, ncells = p.ncells;
    const uint32_t owned_lo = p.has_left ? p.gyz : 0u, owned_hi = p.has_right ? (p.gx - 1u) * p.gyz : ncells;
    const uint32_t k0 = 4u * (blk * blockDim.x + threadIdx.x);
    const uint32_t kb0 = 4u * blk * blockDim.x, kb1 = kb0 + 4u * blockDim.x;   // this workgroup's cells
#pragma unroll 1
    for (int side = 0; side < 2; ++side) {   // workgroup-uniform
        const uint32_t r0 = side == 0 ? 0u : owned_hi, r1 = side == 0 ? owned_lo : ncells;   // halo cells
        if (!(side == 0 ? p.has_left : p.has_right) || kb1 <= r0 || kb0 >= r1) continue;
        const uint32_t c0 = max(kb0, r0), c1 = min(kb1, r1);
        const uint32_t base = side == 0 ? 0u : nl + no, len = side == 0 ? nl : nr;
        const uint32_t S = max(64u, (len + CS_SAMP - 1u) / CS_SAMP), ns = (len + S - 1u) / S;
        __syncthreads();
        for (uint32_t t0 = threadIdx.x; t0 < ns; t0 += 4u * blockDim.x) {
            uint32_t v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = key(side, min(t0 + u * blockDim.x, ns - 1u) * S);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (t0 + u * blockDim.x < ns) samp[t0 + u * blockDim.x] = v[u];
        }
        __syncthreads();
        uint32_t j0, j1;   // samples below c0 / c1: lb(c0) >= (j0 - 1)·S + 1 (or 0), lb(c1) <= min(j1·S, len)
        {
            uint32_t lo = 0u, hi = ns;
            while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (samp[m] < c0) lo = m + 1u; else hi = m; }
            j0 = lo;
            hi = ns;
            while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (samp[m] < c1) lo = m + 1u; else hi = m; }
            j1 = lo;
        }
        const uint32_t ws = j0 == 0u ? 0u : (j0 - 1u) * S + 1u, we = min(j1 * S, len);
        const uint32_t wn = we > ws ? we - ws : 0u;
        const bool staged = wn <= (uint32_t)CS_WIN;
        if (staged) {
            for (uint32_t t0 = threadIdx.x; t0 < wn; t0 += 8u * blockDim.x) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = key(side, ws + min(t0 + u * blockDim.x, wn - 1u));
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (t0 + u * blockDim.x < wn) win[t0 + u * blockDim.x] = v[u];
            }
        }
        __syncthreads();
        for (uint32_t k = max(k0, c0); k < min(k0 + 4u, c1); ++k) {
            uint32_t lo = ws, hi = we;
            if (staged) {
                lo = 0u;
                hi = wn;
                while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (win[m] < k) lo = m + 1u; else hi = m; }
                lo += ws;
            } else {
                while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (key(side, m) < k) lo = m + 1u; else hi = m; }
            }
            p.cs[k] = base + lo;
        }
    }
    if (k0 > ncells + 1u) return;
    const uint32_t* in = p.src ? p.src : p.cs;
    const bool write = shift != 0 || p.src != nullptr;   // in place, unshifted owned cells stay as they are
    if (k0 + 3u < owned_hi && k0 >= owned_lo) {   // four owned cells (cs is 16-byte aligned)
        if (write) {
            uint4 v = reinterpret_cast<const uint4*>(in)[k0 >> 2];
            v.x = (uint32_t)((int32_t)v.x + shift);
            v.y = (uint32_t)((int32_t)v.y + shift);
            v.z = (uint32_t)((int32_t)v.z + shift);
            v.w = (uint32_t)((int32_t)v.w + shift);
            reinterpret_cast<uint4*>(p.cs)[k0 >> 2] = v;
        }
        return;
    }
    for (uint32_t k = k0; k < k0 + 4u && k <= ncells + 1u; ++k) {
        if (k >= ncells) p.cs[k] = n;
        else if (k >= owned_lo && k < owned_hi && write) p.cs[k] = (uint32_t)((int32_t)in[k] + shift);
    }
}
inline int32_t cs_old_blocks(uint32_t ncells, int32_t blk) { return (int32_t)(((ncells + 2u + 3u) / 4u + blk - 1) / blk); }

// the device-sized slab step: the assembled array's layout from SlabSizes (see AsmSrc)
__device__ __forceinline__ void resolve_sizes(AsmSrc& a, ResortScratch& w, int32_t& n) {
    if (!a.dz) return;
    const uint32_t nl = a.dz->nl, no = a.dz->no;
    a.nl = (int32_t)nl;
    a.nre = (int32_t)(nl + no);
    a.o_off = (int32_t)a.dz->o0 - (int32_t)nl;
    w.mi_off = -a.o_off;
    n = (int32_t)a.dz->n;
}
#endif
inline AsmSrc asm_plain(const float4* pos, const float4* vel, const int32_t* id, const uint32_t* sk,
                        const uint32_t* keys, int32_t n) {
    return AsmSrc{pos, vel, id, sk, keys, 0, nullptr, nullptr, nullptr, nullptr, 0, n, nullptr};
}
// the slab step's halo records (slots [0, nl) and [nre, n)): new keys (window sentinel) into
// src.keyr, old keys moved into this window and clamped into src.skr, and every record whose key
// changed appended to the sink (mi = slot | MV_REC) after the own movers the force pass appended
// cs (optional): the device-sized step's old cell-start table in the same launch, from the messages' old keys
void launch_slab_rec(AsmSrc src, int32_t n, GridDesc g, uint32_t key_base, uint32_t* keyr, uint32_t* skr,
                     MoverSink sink, hipStream_t s, const SizesIn* sizes = nullptr, CsOld cs = CsOld{});
// cell-start values to pick once the table is final: out[t] = cs[idx[t]] (device), and the same
// into out_host (mapped pinned memory) when given; m = 0: none
struct CsPick {
    int32_t idx[8];
    int32_t m;
    uint32_t* out;
    uint32_t* out_host;
};
// Model R's further slot arrays, moved with pos / vel / id by the re-sort (all null for Model S)
struct ResortExtra {
    const float4 *omg, *rot, *aux;
    const int32_t* mode;
    float4 *omg_o, *rot_o, *aux_o;
    int32_t* mode_o;
};
// k_mv_rank's workgroups (key/slot ranges) for n slots
uint32_t resort_ranges(int32_t n);
// cs: the old cell-start table (read), cs_new: the new one (every entry written)
void launch_resort(AsmSrc src, uint32_t* cs, uint32_t* cs_new, uint32_t ncells, int32_t n, const uint32_t* count,
                   uint32_t* count_other, ResortScratch w, float4* pos_o, float4* vel_o, int32_t* id_o,
                   uint32_t* sk_o, hipStream_t s, CsPick pick = CsPick{{0}, 0, nullptr, nullptr},
                   ResortExtra ex = ResortExtra{});

// grid / data movement (grid.hip)
// window_sentinel (slab): a particle outside the held columns gets key ncells (sorts last)
// rmax (Model R): atomicMax of the radii's float bits into a word the caller zeroed (ContactConst::rmax)
void launch_keys(const float4* pos, int32_t n, const int32_t* id, int32_t n_active_id,
                 GridDesc g, uint32_t* keys, hipStream_t s, bool window_sentinel = false, uint32_t* rmax = nullptr);
// cell_start[k] = lower_bound(sorted keys, k) for k = 0..ncells, every cell written once:
// each particle boundary fills the cells up to its key; gaps longer than CS_SHORT cells are
// queued (gap list + counter, zeroed by the call) and filled by whole workgroups.
// gap_count: two counters used in turn (*par flips); each call zeroes the other one for the next call
void launch_cell_start(const uint32_t* sorted_keys, int32_t n, uint32_t* cs, uint32_t ncells,
                       uint4* gaps, uint32_t* gap_count, int* par, hipStream_t s);
// Model R's slot arrays (pos, vel, omg, rot, aux; id, mode) gathered by one launch
struct GatherR {
    const float4* f4[5];
    float4* f4o[5];
    const int32_t* i32[2];
    int32_t* i32o[2];
};
void launch_gather_r(const uint32_t* perm, const GatherR& g, int32_t n, hipStream_t s);
void launch_gather_s(const uint32_t* perm, const float4* pos, const float4* vel, const int32_t* id,
                     float4* pos_o, float4* vel_o, int32_t* id_o, int32_t n, hipStream_t s);
void launch_scatter_f4_by_id(const float4* src, const int32_t* id, int32_t n, float* dst,
                             int32_t comps, hipStream_t s);
// dst[id[i]] = src[i].x (comp 0) or .y (comp 1)
void launch_scatter_f2x_by_id(const float2* src, const int32_t* id, int32_t n, float* dst, hipStream_t s,
                              int32_t comp = 0);
void launch_scatter_i3_by_id(const int32_t* src, const int32_t* id, int32_t n, int32_t* dst, hipStream_t s);
void launch_aos84_to_soa(const void* aos, int32_t n, float4* pos, float4* vel, float4* omg,
                         float4* rot, float4* aux, int32_t* mode, int32_t* id, hipStream_t s);
void launch_soa_to_aos84(const float4* pos, const float4* vel, const float4* omg, const float4* rot,
                         const float4* aux, const int32_t* mode, const int32_t* id, int32_t n,
                         void* aos, hipStream_t s);
void launch_kick(const int32_t* id, float4* vel, int32_t n, int32_t target, const float dv[3], hipStream_t s);
void launch_pack_sv(const float* pos3, const float* vel3, int32_t n, float4* pos, float4* vel,
                    int32_t* id, hipStream_t s);
void launch_lattice(int32_t dim, int32_t nx, int32_t ny, int32_t nz, float dx, float x0, float y0,
                    float z0, uint32_t seed, float jitter, float4* pos, float4* vel, int32_t* id,
                    hipStream_t s);
void launch_iota(uint32_t* v, int32_t n, hipStream_t s);

// Model S, LDS-tiled (wcsph_tiled.hip): targets are the sorted slots [ib, ie). paths: 6 counters
// (density planes chunked / rows gathered from global memory, the same for the force pass, force
// planes scanned by distance because a target's candidates passed the hit mask, force blocks), once per
// block and event.
// The hit mask: pass 1 evaluates every candidate of a target's trimmed windows anyway, and writes
// bit k = "candidate k of the visit order is within 2h" (HM_WORDS words per target, word-major: word w
// of slot i at w[w * stride + i]). Pass 2 runs on the same positions and windows, so it reads its hits
// from the mask instead of recomputing every candidate's distance.
constexpr int HM_WORDS = 8;
struct HitMask {
    uint32_t* w = nullptr;   // HM_WORDS * stride words; nullptr: no mask (pass 2 scans by distance)
    uint32_t stride = 0;
};
// The neighbour passes' y-band schedule (schedule.hip): table[0] header, table[1 + d] workgroup d's target range;
// entries = the launch's workgroups. Single-context launches over [0, n) only.
constexpr int SCHED_BANDS = 8;
struct Sched {
    const uint2* table = nullptr;
    int32_t entries = 0;
};
int32_t schedule_entries(int32_t n, const GridDesc& g);
bool schedule_fits(const GridDesc& g);
void launch_schedule(const uint32_t* cs, GridDesc g, int32_t n, uint2* table, int32_t entries, hipStream_t s);
void launch_density_tiled(const float4* pos, const uint32_t* cs, int32_t ib, int32_t ie, GridDesc g,
                          SphConst c, float2* rp, HitMask hm, uint32_t* paths, hipStream_t s, DevRange dr = DevRange{},
                          RhoOut ro = RhoOut{}, Sched sch = Sched{});
// Model S at small N (wcsph_tiled.hip): one wave per target, the tiled passes' sums bit for bit; single context,
// targets [0, n); pass 2 takes its hits by distance (no hit mask)
constexpr int32_t SMALL_N = 16384;
void launch_density_small(const float4* pos, const uint32_t* cs, int32_t n, GridDesc g, SphConst c, float2* rp,
                          hipStream_t s);
void launch_force_small(const float4* pos, const float4* vel, const float2* rp, const uint32_t* cs, int32_t n, GridDesc g,
                        SphConst c, float dt, float fext_x, float4* pos_o, float4* vel_o, uint32_t* keys_o, MoverSink mv,
                        hipStream_t s);
void launch_force_tiled(const float4* pos, const float4* vel, const float2* rp, const uint32_t* cs,
                        int32_t ib, int32_t ie, GridDesc g, SphConst c, float dt, float fext_x,
                        float4* pos_o, float4* vel_o, uint32_t* keys_o, MoverSink mv, HitMask hm, uint32_t* paths,
                        hipStream_t s, DevRange dr = DevRange{}, DevRange dr2 = DevRange{}, int32_t ie2 = 0,
                        SendBins sb = SendBins{}, Sched sch = Sched{});

// slab decomposition (slab.hip)
// Order-preserving compaction of the sorted slots [b, e) whose key column satisfies
// col <= col_le (side 0) / col >= col_ge (side 1) into 32-byte records (x,y,z,id | u,v,w,0).
int32_t slab_compact_blocks(int32_t b, int32_t e);
void launch_slab_count(const uint32_t* keys, int32_t b, int32_t e, uint32_t gyz, int32_t col_le,
                       int32_t col_ge, uint32_t* blk /*[2][nblk]*/, uint32_t* totals /*[2]*/,
                       hipStream_t s,
                       int64_t* totals64 = nullptr);
// records carry the old sorted key as a global key (sk + key_base; sk null: none, see slab.hip)
void launch_slab_pack(const uint32_t* keys, const float4* pos, const float4* vel, const int32_t* id,
                      const uint32_t* sk, uint32_t key_base, int32_t b, int32_t e, uint32_t gyz, int32_t side,
                      int32_t col_le, int32_t col_ge, const uint32_t* blk, float4* out, hipStream_t s);
void launch_slab_unpack(const float4* rec, int32_t n, float4* pos, float4* vel, int32_t* id, hipStream_t s);
// cell starts of the assembled old keys, in place from the previous table (ncells + 2 entries)
void launch_slab_cs_old(uint32_t* cs, uint32_t ncells, uint32_t gyz, uint32_t gx, bool has_left, bool has_right,
                        int32_t shift, const uint32_t* sk, int32_t nl, int32_t no, int32_t nr, hipStream_t s,
                        const SlabSizes* dz = nullptr);
void launch_column_starts(const uint32_t* cs, uint32_t gyz, int32_t c0, int32_t m, uint32_t* out, hipStream_t s);
void launch_pick(const uint32_t* cs, const int32_t* idx, int32_t m, uint32_t* out, hipStream_t s,
                 uint32_t* out_host = nullptr);
// ---- the device-sized slab step (slab.hip; abi_multi.cpp drives it)
// count + pack over the owned slots [dz->o0, dz->o1): the same order-preserving compaction as above,
// into messages of a header and `cap[side]` records (header = true count; records past cap dropped and
// flagged by the receiver). nb_ub: count-block upper bound (slab_send_blocks of the slot bound).
// cand: steady state, scan only the columns a send can come from (slab.hip send_ranges)
// exact: also the totals (host-read before packing on exact-size steps). early: the sends of the NEXT step,
// packed right after this step's boundary force pass (slab.hip send_ranges)
void launch_slab_count_dev(const uint32_t* keys, const SlabSizes* dz, int32_t nb_ub, uint32_t gyz, int32_t col_le,
                           int32_t col_ge, uint32_t* blk, uint32_t* totals, hipStream_t s, bool cand, bool exact,
                           bool early = false);
// both sides in one launch from the raw per-block counts; headers and totals[2] written by the pack
void launch_slab_pack2_dev(const uint32_t* keys, const float4* pos, const float4* vel, const int32_t* id,
                           const uint32_t* sk, uint32_t key_base, const SlabSizes* dz, int32_t nb_ub, uint32_t gyz,
                           int32_t col_le, int32_t col_ge, const uint32_t* blk, float4* msg_l, int32_t cap_l,
                           float4* msg_r, int32_t cap_r, uint32_t* totals, hipStream_t s, bool cand,
                           bool early = false);
int32_t slab_send_blocks(int32_t b, int32_t e);
// the received messages' counts -> dz (nl, nr clamped to the capacities, no, n, overflow flags)
void launch_slab_sizes(SlabSizes* dz, const float4* msg_l, const float4* msg_r, int32_t cap_l, int32_t cap_r,
                       int32_t capacity, hipStream_t s);
// after the re-sort: dz->pick -> the ranges (rg, fr, o0/o1 of the new order, n and dropped)
// ρ, P/ρ² of boundary column `side` ([pick[1+2side], pick[2+2side])) -> message (header + cap entries)
// both sides' ρ messages in one launch each way (a null message: no neighbour on that side)
void launch_slab_pack_rho2(const float2* rp, SlabSizes* dz, float2* msg_l, int32_t cap_l, float2* msg_r, int32_t cap_r,
                           hipStream_t s);
// received densities -> the ghost column of `side` ([pick[4side], pick[4side+1])); mismatch -> SZ_RHO_MISMATCH
void launch_slab_unpack_rho2(float2* rp, SlabSizes* dz, const float2* msg_l, int32_t cap_l, const float2* msg_r,
                             int32_t cap_r, hipStream_t s);
// per-step counts for the host's lagged capacity choice, written to mapped pinned memory:
// out[0..1] sent records (left, right), out[2..3] received headers, out[4..5] ρ sent, out[6..7] ρ received,
// out[8] assembled slots, out[9] flags (gflags non-null: that word instead, every rank's flags reduced)
// totals: this step's send counts (k_slab_pack2 / k_slab_scan wrote them into the step's slot)
// zero/nzero: words to clear (the early sends' count bins, after the pack read them); null: none
void launch_slab_lag(SlabSizes* dz, int32_t has_left, int32_t has_right, const uint32_t* totals,
                     const float2* rho_in_l, const float2* rho_in_r, const uint32_t* gflags, uint32_t* out,
                     hipStream_t s, uint32_t* zero = nullptr, int32_t nzero = 0);

// owned slots [o0, o0+n) -> records of 8 floats (x,y,z,u,v,w,id-bits,ρ)
void launch_pack_owned(const float4* pos, const float4* vel, const int32_t* id, const float2* rp,
                       int32_t o0, int32_t n, float* out, hipStream_t s);
// keep the particles of global columns [lo, hi) (order-preserving) — slab init
void launch_slab_select_columns(const float4* pos, const float4* vel, const int32_t* id, int32_t n,
                                GridDesc gglobal, int32_t lo, int32_t hi, uint32_t* blk,
                                uint32_t* total, float4* pos_o, float4* vel_o, int32_t* id_o,
                                hipStream_t s);

// Adhesion bonds (§8f-1), SoA of the reference's 84-byte AdhesionConnection (compute:43-55).
struct BondSet {
    const int2* ends;       // (particleA, particleB): particle indices
    const float4* spring;   // (restLength, springStiffness, springDamping, anchorConstraintStiffness)
    const float4* relq;     // initialRelOrientation
    const float4* anc_a;    // anchorLocalPosA, w = enableAnchorConstraint (int bits)
    const float4* anc_b;    // anchorLocalPosB
    int32_t count;
};
// Per-bond int terms and the per-particle incidence lists the finishing pass gathers them by.
struct BondView {
    int32_t count;          // bonds this step; 0: ApplyAdhesionDeltas is not dispatched
    int32_t n_index;        // particle indices covered by off[]
    const uint32_t* off;    // [n_index + 1] CSR offsets by particle index
    const uint32_t* ent;    // bond << 1 | side (0: particleA, 1: particleB)
    const int4* terms;      // [4 * count]: Δv_A, Δv_B, Δq_A, Δq_B (fixed point ×1e6)
};

// Model R particle lifecycle (particles.hip)
struct InitConst {   // InitParticles uniforms (compute:89-100) + genome selection (:64-68)
    float spawn_radius, min_radius, max_radius, density;
    int32_t length;          // particleBuffer.Length
    int32_t genome_modes;    // genomeModesCount
    int32_t default_mode;    // defaultGenomeMode
};
struct SplitRec {    // CellSplitData (ParticleSystemController.cs:136-147) == sph_split (sphhip.h)
    int32_t parent;
    float posA[3], posB[3], velA[3], velB[3], rotA[4], rotB[4];
    int32_t modeA, modeB;
};
void launch_slot_map(const int32_t* id, int32_t n, int32_t* slot_of, hipStream_t s);
void launch_init_sphere(int32_t n, int32_t active, InitConst c, float4* pos, float4* vel, float4* omg, float4* rot,
                        float4* aux, int32_t* mode, int32_t* id, int32_t* torque, hipStream_t s);
void launch_split(const SplitRec* sp, int32_t count, int32_t active, int32_t n_old, const int32_t* slot_of,
                  float4* pos, float4* vel, float4* omg, float4* rot, float4* aux, int32_t* mode, int32_t* id,
                  hipStream_t s);
void launch_get_range(const float4* pos, const float4* vel, const float4* omg, const float4* rot, const float4* aux,
                      const int32_t* mode, const int32_t* slot_of, int32_t first, int32_t count, void* aos,
                      hipStream_t s);
void launch_set_range(const void* aos, const int32_t* slot_of, int32_t first, int32_t count, float4* pos,
                      float4* vel, float4* omg, float4* rot, float4* aux, int32_t* mode, hipStream_t s);

// Model R (contact.hip). team: lanes per target (0 = by size, else 1, 16 or 64; any choice gives
// bit-identical results).
// The one-launch Model R step at the reference's scale (contact.hip k_contact_fused): re-sort + contact + drag +
// motion + rotation for n <= contact_fused_max(), reading the previous step's arrays through this step's permutation.
struct FusedIO {
    const float4 *pos, *vel, *omg, *rot, *aux;
    const int32_t *id, *mode;
    const uint32_t *sk, *cs;
    const uint32_t *mi, *mk;
    const uint32_t* count;
    float4 *pos_o, *vel_o, *omg_o, *rot_o, *aux_o;
    int32_t *id_o, *mode_o, *torque_o;
    uint32_t *sk_o, *keys_o, *cs_o;
    uint32_t *mi_o, *mk_o, *mo_o, *count_o, *count_zero, *host_count;
    uint32_t cap;
    // (cs[k], cs[k + 1]) of each mover's new key k as the step before computed it, or ~0: that step's own table (null:
    // the build loads them); mc_o: this step's, for the next (fused_perm.h)
    const uint32_t* mc;
    uint32_t* mc_o;
};
int32_t contact_fused_max();
// Model S's counterpart (wcsph_tiled.hip k_density_fused): re-sort + pass 1 in one launch, then k_force_small
struct FusedIOS {
    const float4 *pos, *vel;
    const int32_t* id;
    const uint32_t *sk, *cs;
    const uint32_t *mi, *mk;
    const uint32_t* count;
    float4 *pos_o, *vel_o;
    int32_t* id_o;
    uint32_t *sk_o, *cs_o;
    float2* rp_o;
    uint32_t *count_zero, *host_count;
};
int32_t density_fused_max();
void launch_density_fused(const FusedIOS& io, int32_t n, GridDesc g, SphConst c, hipStream_t s);
void launch_contact_fused(const FusedIO& io, int32_t n_active, int32_t n, GridDesc g, ContactConst c, hipStream_t s);
void launch_contact_step(const float4* pos, const float4* vel, const float4* omg, const float4* rot,
                         const float4* aux, const int32_t* id, const uint32_t* cs, int32_t n_active,
                         int32_t n, GridDesc g, ContactConst c, float4* pos_o, float4* vel_o,
                         float4* omg_o, float4* rot_o, int32_t* torque_o, uint32_t* keys_o, int team,
                         MoverSink mv, hipStream_t s);
void launch_contact_forces(const float4* pos, const float4* vel, const float4* omg, const int32_t* id,
                           const uint32_t* cs, int32_t n_active, int32_t n, GridDesc g, ContactConst c,
                           float4* vel_o, float4* omg_o, int32_t* torque_o, int32_t* slot_of, int team,
                           hipStream_t s);
void launch_contact_finish(const float4* pos, const float4* rot, const float4* aux, const int32_t* id,
                           const int32_t* torque, int32_t n_active, int32_t n, GridDesc g, ContactConst c,
                           BondView b, float4* vel_io, float4* omg_io, float4* pos_o, float4* rot_o,
                           uint32_t* keys_o, MoverSink mv, hipStream_t s);
// ApplyAdhesionConstraints (compute:424-584), one lane per bond: reads the start-of-step
// position and rotation and the post-contact velocity, writes the bond's four int terms.
void launch_bond_terms(BondSet bs, const int32_t* slot_of, int32_t n, const float4* pos, const float4* vel1,
                       const float4* rot, float dt, int4* terms, hipStream_t s);

}  // namespace sph
