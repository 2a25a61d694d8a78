// wcsph_tiled.hip — LDS-tiled Model S neighbour passes (SPEC_SPH.md §2), gfx950.
//
// A workgroup owns 256 consecutive cell-sorted targets. Their keys span [kf, kl]. For each of
// the 9 (dx,dy) row offsets `off`, the block's candidates are the ONE contiguous sorted
// interval of keys [kf+off-zwin, kl+off+zwin], and every target's own trimmed row window
// lies inside it (SPEC_SPH.md §0). The three intervals of one dx plane are staged into LDS
// together: one barrier pair per plane, three coalesced streams in flight. Every target then
// walks its own three windows out of LDS, and lanes of one cell read the same address
// (broadcast). The visit order is the §0 order.
//
// Pass 1 scans 4 candidates per iteration, branchless (clamped LDS reads, predicated
// accumulation), and records every candidate's q = r/h ≤ 2 as one bit in visit order (the hit mask,
// common.h HitMask; the sign bit of 2 − q, see spline_w4). Only ~30% of the trimmed candidates are within
// 2h. Pass 2 runs on the same positions and windows, so it takes its hits from the mask instead of
// re-reading every candidate from LDS and recomputing its distance: per staged plane it walks the
// plane's bits (its three row windows back to back) in one pair loop, one hit per iteration (find-first-
// set, LDS slot = bit + its row's offset, pair body). A target with more than HM_WORDS·32 candidates
// falls back to a distance loop for the plane in question (wave-uniform); both give the same hits
// in the same order, so results do not depend on the path.
// A plane whose intervals exceed the LDS budget (sparse blocks spanning many rows) is processed
// offset by offset in chunks, and an offset beyond the fallback length is gathered directly from
// global memory.
#include "common.h"
#include "fused_perm.h"

namespace sph {

constexpr int TT_BLK = 256;     // targets per workgroup (128 / 192 / 512 measured 13-25% slower)
// Candidates staged per plane (LDS), density pass: 1350 (21.7 KB) with the kernel held to 72 VGPRs
// (amdgpu_waves_per_eu(7)) gives seven workgroups per CU. Against six at 1500 (74 VGPRs): -0.5 us from rest,
// -2 us mid-collapse; eight at 1200 (64 VGPRs, spills) +1 to +19 us, five +8 us, four +17 us
// (profiles/r02_density_waves_ab.log). 1500
// against 1024 at six per CU: 143.5 -> 141.4 us from rest (profiles/r02_density_budget_ab.log).
#ifndef SPH_TT_GCAP
#define SPH_TT_GCAP 1350
#endif
#ifndef SPH_DWAVES
#define SPH_DWAVES 7
#endif
constexpr int TT_GCAP = SPH_TT_GCAP;
constexpr int TT_FALLBACK = 4 * TT_GCAP;
// The force pass stages 32 B per candidate (no hit lists since the mask walk). With 124 VGPRs four
// workgroups fit a CU, so the plane budget takes what four leave of the LDS: 1270 candidates (40.6 KB);
// more of the C3 planes (~840 candidates on average) are then staged at once, not row by row in chunks.
// Interleaved A/B (profiles/r02_nolist_budget_ab.log): 1000 -> 1270 cut the force pass 205 -> 192 us
// from rest and 233 -> 222 us mid-collapse; five waves per SIMD (96 VGPRs, spills) cost 80 us.
#ifndef SPH_TF_GCAP
#define SPH_TF_GCAP 1270
#endif
constexpr int TF_GCAP = SPH_TF_GCAP;
#ifndef SPH_WALK_UNROLL
#define SPH_WALK_UNROLL 4
#endif
constexpr int TF_FALLBACK = 4 * TF_GCAP;
#ifndef SPH_TF_BLK
#define SPH_TF_BLK 256
#endif
constexpr int TF_BLK = SPH_TF_BLK;
static_assert(SEND_SLOTS % TF_BLK == 0, "a force workgroup lies in one send block (SendBins)");
// Slots each thread stages per round (loads in flight together): pass 1 up to 1,350 slots in 256 threads
// takes all of a plane in one or two rounds; pass 2 holds 40 B per slot in registers.
#ifndef SPH_TT_STAGE_U
#define SPH_TT_STAGE_U 3
#endif
#ifndef SPH_TF_STAGE_U
#define SPH_TF_STAGE_U 2
#endif
constexpr int TT_STAGE_U = SPH_TT_STAGE_U;
constexpr int TF_STAGE_U = SPH_TF_STAGE_U;
struct Staged {
    float4 p, v;
    float2 r;
};

struct BlockRows {
    int64_t kf, kl;           // key range of the block's targets
    int32_t cx, cy;           // this lane's sub-column (x, GridDesc::xsub per column) and cell (y)
    float fx, fy, gzf;        // in-sub-column / in-cell fractions and z sub-cell coordinate (row_window)
};

template <int XS>
__device__ __forceinline__ BlockRows block_rows(const GridDesc& g, const float4* __restrict__ pos, int32_t i0,
                                                int32_t ilast, float4 pi) {
    BlockRows b;
    const float4 pf = pos[i0], pl = pos[ilast];
    b.kf = cell_key<XS>(g, pf.x, pf.y, pf.z);
    b.kl = cell_key<XS>(g, pl.x, pl.y, pl.z);
    b.cx = cell_cxs<XS>(g, pi.x);
    b.cy = cell_coord(pi.y, g.oy, g.inv_cell, g.gy);
    cell_fracs<XS>(g, pi.x, pi.y, pi.z, b.cx, b.cy, b.fx, b.fy, b.gzf);
    return b;
}

// Row k = 3·plane + r: sub-column offset plane − XS, y offset r − 1 (planes 0..2·XS; XS = the grid's
// xsub, a template parameter of both passes so that the default grid compiles to the plain 3 x 3 rows).
// Block interval of row offset k ([c0,c1) sorted slots; uniform over the block).
template <int XS>
__device__ __forceinline__ void block_interval(const GridDesc& g, const uint32_t* __restrict__ cs, const BlockRows& b,
                                               int k, int32_t& c0, int32_t& c1) {
    const int32_t dxk = k / 3 - XS, dyk = k % 3 - 1;
    const int64_t off = ((int64_t)dxk * g.gy + dyk) * g.gz;
    int64_t ka = b.kf + off - g.zwin, kb = b.kl + off + g.zwin;
    const int64_t last = (int64_t)g.ncells - 1;
    if (kb < 0 || ka > last) {
        c0 = c1 = 0;
        return;
    }
    ka = ka < 0 ? 0 : ka;
    kb = kb > last ? last : kb;
    c0 = (int32_t)cs[ka];
    c1 = (int32_t)cs[kb + 1];
}

// This lane's trimmed window of row offset k ([r0,r1) sorted slots, empty if out of range).
template <int XS>
__device__ __forceinline__ void lane_window(const GridDesc& g, const uint32_t* __restrict__ cs, const BlockRows& b,
                                            bool valid, int k, int32_t& r0, int32_t& r1) {
    const int32_t dxk = k / 3 - XS, dyk = k % 3 - 1;
    const int32_t xx = b.cx + dxk, yy = b.cy + dyk;
    r0 = r1 = 0;
    int32_t zlo, zhi;
    if (valid && xx >= 0 && xx < g.gx * XS && yy >= 0 && yy < g.gy &&
        row_window<XS>(g, b.fx, b.fy, b.gzf, dxk, dyk, zlo, zhi)) {
        const uint32_t rowk = ((uint32_t)xx * (uint32_t)g.gy + (uint32_t)yy) * (uint32_t)g.gz;
        r0 = (int32_t)cs[rowk + (uint32_t)zlo];
        r1 = (int32_t)cs[rowk + (uint32_t)zhi + 1u];
    }
}

// Sparse-path counters (tests: sph_read_path_counts): [0] density planes chunked, [1] density rows
// gathered from global memory, [2] / [3] the same for the force pass. One atomic per block and event.
__device__ __forceinline__ void count_path(uint32_t* paths, int k) {
    if (paths && threadIdx.x == 0) atomicAdd(paths + k, 1u);
}
// per wave; paths is null unless a test armed the counters (one address: contended atomics)
__device__ __forceinline__ void count_wave(uint32_t* paths, int k) {
    if (paths && lane_id() == 0) atomicAdd(paths + k, 1u);
}

#ifdef SPH_BTIME
// Diagnostic builds only (-DSPH_BTIME): each workgroup's start and end (s_memrealtime, 100 MHz) of the last
// launch of each pass, read by sph_debug_block_times (scripts/block_times.py).
constexpr int BT_MAX = 16384;
__device__ uint64_t g_btime[2][BT_MAX][2];
#define SPH_BT_START const uint64_t bt0_ = __builtin_amdgcn_s_memrealtime()
#define SPH_BT_END(kid)                                                                                      \
    do {                                                                                                     \
        __syncthreads();                                                                                     \
        if (threadIdx.x == 0 && blockIdx.x < BT_MAX) {                                                       \
            g_btime[kid][blockIdx.x][0] = bt0_;                                                              \
            g_btime[kid][blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();                                  \
        }                                                                                                    \
    } while (0)
#else
#define SPH_BT_START ((void)0)
#define SPH_BT_END(kid) ((void)0)
#endif

#ifdef SPH_DIAG
// Diagnostic builds only (-DSPH_DIAG): lane-utilisation counters in paths[8..16) (sph_debug_pass_counts).
__device__ __forceinline__ int wave_max(int v) {
    for (int o = 32; o; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_sum(int v) {
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
#define SPH_DIAG_ADD(k, v)                                                                   \
    do {                                                                                     \
        const int v_ = (v);                                                                  \
        if (paths && lane_id() == 0) atomicAdd(paths + (k), (uint32_t)v_);                   \
    } while (0)
#else
#define SPH_DIAG_ADD(k, v) ((void)0)
#endif

// Sums of products are written as explicit fmaf chains: left to the compiler's contraction, dx·dx + dy·dy
// + dz·dz became fma(dx, dx, dy·dy) in the LDS scans but fma(dy, dy, dx·dx) in the global-gather path, so a
// candidate at q = 2 to the last ulp could be a hit on one path and not on the other, and results depended
// on which path a block took (on the plane budget and block size; tests/test_gpu_slab.py decompositions).
__device__ __forceinline__ float dist2(float4 a, float4 b) {
    const float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
    return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
}

// SPH_RUNITS (default 1): both passes evaluate the kernel in units of r instead of q = r/h: the powers of h go
// into per-launch constants (SphConst two_h, m6h, four_h3, rho_scale; PairK), which takes the r²·(1/h²) multiply
// out of pass 1's candidate loop and q, q² and one h factor out of pass 2's pair body. 0: the q forms below.
#ifndef SPH_RUNITS
#define SPH_RUNITS 1
#endif

#if SPH_RUNITS
// h³·4·w(q) of the unnormalised cubic spline (W = σ·w), r = |x_i − x_j|: min(4h³ + r²(3r − 6h), max(2h − r, 0)³),
// the q form below times h³. v = 2h − r comes back: its sign bit is set exactly for the candidates that are NOT
// neighbours (r > 2h, with r = sqrt(r²) rounded as here), the hit bit pass 1 records and is_hit tests.
__device__ __forceinline__ float spline_w4(const SphConst& c, float r2, float& v) {
    const float r = __builtin_amdgcn_sqrtf(r2);
    v = c.two_h - r;
    const float t = __builtin_amdgcn_fmed3f(v, 0.0f, c.two_h);   // max(v, 0) (v ≤ 2h); fmaxf adds a canonicalize
    return fminf(fmaf(r2, fmaf(3.0f, r, c.m6h), c.four_h3), t * t * t);
}

// The neighbour test of both passes, for paths without the hit mask: the bit pass 1 records.
__device__ __forceinline__ bool is_hit(const SphConst& c, float r2) {
    return (__float_as_uint(c.two_h - __builtin_amdgcn_sqrtf(r2)) >> 31) == 0u;
}
#else
// 4·w(q) of the unnormalised cubic spline (W = σ·w) for q ≤ 2, else 0. Branchless: both arms
// are computed and selected (a ?: over expressions compiles to an exec branch per candidate).
// Scaling by 4 (and the final 0.25) is exact in binary floating point: no rounding is added.
// 4w = (2−q)₊³ − 4(1−q)₊³: the outer arm (2−q)₊³ lies below the inner polynomial exactly where
// q ≥ 1 (their difference is 4(1−q)³), and (2−q)₊ is 0 past the support, where the polynomial is ≥ 4.
// So one min replaces both selects (18 VALU slots per candidate instead of 20; C3 pass 1 −5%).
// q = sqrt(r²/h²) (q² is then r²/h², no square), and v = 2 − q comes back: its sign bit is set exactly
// for the candidates that are NOT neighbours (q > 2), so the hit test costs no instruction of its own
// (pass 1 records the complement and inverts each word once). A neighbour is q ≤ 2 with q rounded as
// here; r = 2h exactly adds 0 in both passes. Against sqrt(r²)·(1/h), q·q and r² − 4h² for the bit: two
// VALU fewer per candidate.
__device__ __forceinline__ float spline_w4(const SphConst& c, float r2, float& v) {
    const float r2h = r2 * c.inv_h2;
    const float q = __builtin_amdgcn_sqrtf(r2h);
    v = 2.0f - q;
    const float t = __builtin_amdgcn_fmed3f(v, 0.0f, 4.0f);   // max(v, 0) (v ≤ 2); fmaxf adds a canonicalize here
    return fminf(fmaf(r2h, fmaf(3.0f, q, -6.0f), 4.0f), t * t * t);
}

// The neighbour test of both passes, for paths without the hit mask: the bit pass 1 records.
__device__ __forceinline__ bool is_hit(const SphConst& c, float r2) {
    return (__float_as_uint(2.0f - __builtin_amdgcn_sqrtf(r2 * c.inv_h2)) >> 31) == 0u;
}
#endif

// ρ and P/ρ² from the kernel sum (Tait EOS, SPEC_SPH.md §2), both forms of pass 1
__device__ __forceinline__ float2 density_eos(const SphConst& c, float s) {
#if SPH_RUNITS
    const float d = c.rho_scale * s;   // m·σ·(h³·4w)/(4h³)
#else
    const float d = c.mass * (c.sigma * (0.25f * s));
#endif
    const float tr = d * c.inv_rho0;
    const float t2 = tr * tr, t4 = t2 * t2;
    const float P = c.B * (t4 * t2 * tr - 1.0f);
    return make_float2(d, P / (d * d));
}

// The scans use x, y, z only, and the compiler then narrows the float4 LDS read to
// ds_read_b96: 8 LDS cycles per wave with 32-bank grouping, against 4 for ds_read_b128
// (MI355X_MICROARCH.md §LDS). The empty asm consumes .w at no instruction cost so the 16-B read stays.
__device__ __forceinline__ void keep_b128(float4 a, float4 b, float4 c, float4 d) {
    asm volatile("" ::"v"(a.w), "v"(b.w), "v"(c.w), "v"(d.w));
}

// Stage the plane's three intervals back to back: slot t of interval r sits at off[r] + t, from sorted
// slot c0[r] + (t − off[r]). U slots per thread per round, all U loads issued before the LDS writes, so
// they are in flight together; the source interval is picked by selects (indexing c0[] by a computed r
// put the array in scratch memory: one scratch load and one global load, serialised, per staged slot).
template <int U, int BLK = TT_BLK, typename L, typename W>
__device__ __forceinline__ void stage_plane(const int32_t (&c0)[3], const int32_t (&len)[3], int32_t total, L&& load,
                                            W&& write) {
    const int32_t e0 = len[0], e1 = len[0] + len[1];
    const int32_t d0 = c0[0], d1 = c0[1] - e0, d2 = c0[2] - e1;
    for (int32_t base = threadIdx.x; base < total; base += U * BLK) {
        decltype(load(0)) v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t t = base + u * BLK;
            if (t < total) v[u] = load(t + (t < e0 ? d0 : (t < e1 ? d1 : d2)));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t t = base + u * BLK;
            if (t < total) write(t, v[u]);
        }
    }
}

// One contiguous run [src0, src0 + ln) into slots [0, ln) (the chunked rows), the same way.
template <int U, int BLK = TT_BLK, typename L, typename W>
__device__ __forceinline__ void stage_run(int32_t src0, int32_t ln, L&& load, W&& write) {
    const int32_t c0[3] = {src0, 0, 0}, len[3] = {ln, 0, 0};
    stage_plane<U, BLK>(c0, len, ln, load, write);
}

// a[r] for a runtime r in 0..2 as selects: an array indexed by a runtime value lives in scratch memory for the whole
// kernel (pass 1 kept its lane windows there: three scratch stores per plane and a scratch load after each staging
// barrier, before the scan could start)
__device__ __forceinline__ int32_t pick3(const int32_t (&a)[3], int r) { return r == 0 ? a[0] : (r == 1 ? a[1] : a[2]); }

// A plane whose three intervals exceed the LDS budget: consecutive rows that fit together are staged as
// one group (rows 0+1 or 1+2), the others one by one; a row past the budget goes to big_row (chunks or
// global memory). Groups run in visit order, so the hit mask's bits are taken in order. At C3 ~10% of
// the block-planes from rest exceed the budgets: a block in a column of 2 x 2 lattice lines spans ~64
// layers, and its side rows in columns of 3 lattice lines hold ~1.5x its own count each.
template <typename G, typename B>
__device__ __forceinline__ void plane_groups(const int32_t (&len)[3], int32_t cap, G&& group, B&& big_row) {
    const bool f0 = len[0] <= cap, f1 = len[1] <= cap, f2 = len[2] <= cap;
    if (f0 && f1 && len[0] + len[1] <= cap) {
        group(3u);
        if (f2) group(4u); else big_row(2);
    } else if (f1 && f2 && len[1] + len[2] <= cap) {
        if (f0) group(1u); else big_row(0);
        group(6u);
    } else {
        if (f0) group(1u); else big_row(0);
        if (f1) group(2u); else big_row(1);
        if (f2) group(4u); else big_row(2);
    }
}

// Lanes of one wave take targets of one in-cell quadrant (fx < ½, fy < ½). A side row's trimmed z
// window and a plane's hit count grow with the target's distance to the neighbour column, so lanes
// with alike windows idle less in the wave-wide scan and flush loops. Stable within a quadrant;
// every target keeps its own visit order, so results are bit-identical. Returns the lane's slot
// (>= n for the padding lanes of the last block, which sort last).
template <int XS>
__device__ __forceinline__ int32_t quadrant_target(const GridDesc& g, const float4* __restrict__ pos, int32_t i0,
                                                   int32_t n, int32_t* perm, uint32_t (*cnt)[5]) {
    static_assert(TT_BLK % 64 == 0, "whole waves");
    const int32_t i = i0 + threadIdx.x;
    int bin = 4;
    if (i < n) {
        const float4 p = pos[i];
        const int32_t cx = cell_cxs<XS>(g, p.x), cy = cell_coord(p.y, g.oy, g.inv_cell, g.gy);
        float fx, fy, gzf;
        cell_fracs<XS>(g, p.x, p.y, p.z, cx, cy, fx, fy, gzf);
        bin = (fx >= 0.5f ? 1 : 0) + (fy >= 0.5f ? 2 : 0);
    }
    const int w = threadIdx.x >> 6;
    uint64_t mine = 0;
#pragma unroll
    for (int b = 0; b < 5; ++b) {
        const uint64_t m = __ballot(bin == b);
        if (bin == b) mine = m;
        if (lane_id() == 0) cnt[w][b] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    uint32_t off = 0;
    for (int b = 0; b < bin; ++b)
#pragma unroll
        for (int v = 0; v < TT_BLK / 64; ++v) off += cnt[v][b];
    for (int v = 0; v < w; ++v) off += cnt[v][bin];
    off += __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
    perm[off] = i;
    __syncthreads();
    return perm[threadIdx.x];
}

// This workgroup's targets [i0, iend): entry blockIdx.x of the y-band table (schedule.hip) when one is given and fits,
// else runs of blocks dealt to the XCDs (xcd_block) over [ib, n). false: no targets (exit before any barrier).
template <int BLK>
__device__ __forceinline__ bool block_range(const uint2* __restrict__ sch, int32_t ib, int32_t n, int32_t& i0,
                                            int32_t& iend) {
    int32_t nb = (int32_t)gridDim.x;
    if (sch) {
        const uint2 h = sch[0];
        if (h.x) {
            const uint2 e = sch[1 + blockIdx.x];
            i0 = (int32_t)e.x;
            iend = (int32_t)e.y;
            return i0 < iend;
        }
        nb = (n - ib + BLK - 1) / BLK;   // the table did not fit: the plain mapping over the first nb workgroups
        if ((int32_t)blockIdx.x >= nb) return false;
    }
    i0 = ib + xcd_block((int32_t)blockIdx.x, nb) * BLK;
    iend = min(i0 + BLK, n);
    return i0 < n;
}

template <int XS>
__global__ __launch_bounds__(TT_BLK) __attribute__((amdgpu_waves_per_eu(SPH_DWAVES))) void k_density_tiled(
    const float4* __restrict__ pos, const uint32_t* __restrict__ cs, int32_t ib, int32_t n, GridDesc g, SphConst c,
    float2* __restrict__ rp, DevRange dr, HitMask hm, uint32_t* __restrict__ paths, RhoOut ro,
    const uint2* __restrict__ sch) {
    __shared__ float4 sp[TT_GCAP + 4];
    __shared__ int32_t perm[TT_BLK];
    __shared__ uint32_t qcnt[TT_BLK / 64][5];
    if (ro.dz && blockIdx.x == 0 && threadIdx.x < 2 && ro.msg[threadIdx.x]) {   // ρ message headers (slab step)
        const int sd = (int)threadIdx.x;
        const uint32_t cnt = ro.dz->pick[2 + 2 * sd] - ro.dz->pick[1 + 2 * sd];
        float2* m = ro.msg[sd];
        m[0] = make_float2(__uint_as_float(cnt), __uint_as_float((uint32_t)ro.cap[sd]));
        m[1] = m[2] = m[3] = make_float2(0.f, 0.f);
    }
    if (ro.fbits && ro.dz && blockIdx.x == 0 && threadIdx.x == 0) {   // every earlier kernel of the step has set its flags
        const uint32_t f = ro.dz->flags;
#pragma unroll
        for (int k = 0; k < SZ_BITS; ++k) ro.fbits[k] = (f >> k) & 1u;
    }
    if (dr.lo) {   // device-resident bounds (slab mode); the grid is an upper bound
        ib = (int32_t)*dr.lo;
        n = (int32_t)*dr.hi;
    }
    int32_t i0, iend;
    if (!block_range<TT_BLK>(sch, ib, n, i0, iend)) return;   // whole workgroup: before any barrier
    SPH_BT_START;
    // quadrant order, measured against plain sorted order (138 -> 154 us) and halves by fx or by fy
    // (+1 to +2 us) at C3 (profiles/r02_pass1_lane_order_ab.log)
    const int32_t i = quadrant_target<XS>(g, pos, i0, iend, perm, qcnt);
    const bool valid = i < iend;
    const int32_t ilast = iend - 1;
    const float4 pi = pos[valid ? i : ilast];
    const BlockRows b = block_rows<XS>(g, pos, i0, ilast, pi);
    float s = 0.0f;
    auto load_p = [&](int32_t src) { return pos[src]; };
    auto write_p = [&](int32_t t, float4 e) { sp[t] = e; };
    // hit-mask writer: a 64-bit shift register (mh:ml) takes the newest bit at bit 0 (one v_alignbit per
    // candidate: ml = ml << 1 | sign(r² − 4h²)); the mn unwritten bits sit at [0, mn). A word leaves once 32
    // are pending: the oldest 32 (one v_alignbit), bit-reversed so that the oldest lands at bit 0.
    // The mask's words are stored while wp < wend (HM_WORDS of them; none without a mask).
    uint32_t mh = 0, ml = 0;
    int32_t mn = 0;
    const bool rec = valid && hm.w != nullptr;
    uint32_t* wp = rec ? hm.w + i : nullptr;
    uint32_t* const wend = rec ? hm.w + i + (size_t)HM_WORDS * hm.stride : nullptr;
    // the register pair takes sign(2 − q): 1 for a candidate that is NOT a neighbour; words are inverted
    auto bit = [&](float v) { ml = __builtin_amdgcn_alignbit(ml, __float_as_uint(v), 31u); };
    // the oldest 32 pending bits, sh newer ones above them. Words past the HM_WORDS budget all go to the extra
    // row at wend (allocated, never read), so the budget test sits inside the store and not in every group.
    // Only lanes with a target scan candidates, so wp is set wherever a store runs; hm.w is uniform.
    auto store = [&](uint32_t sh) {
        if (hm.w != nullptr) {
            *wp = __builtin_bitreverse32(~__builtin_amdgcn_alignbit(mh, ml, sh));
            if (wp < wend) wp += hm.stride;
        }
    };
    auto one = [&](float r2) {   // a single candidate (scalar tail, global gather)
        float v;
        s += spline_w4(c, r2, v);
        mh = __builtin_amdgcn_alignbit(mh, ml, 31u);
        bit(v);
        if (++mn >= 32) {
            mn -= 32;
            store((uint32_t)mn);
        }
    };
    // Four candidates per iteration, through an LDS pointer. mn advances by 4, so the iterations that
    // complete a word are known before the loop: the first at k0 = (31 − mn)/4, then every eighth, each
    // with mn mod 4 newer bits above the word. One compare per iteration (pointer against the next
    // word's iteration) replaces the counter update and compare, and the loop bound is the pointer too.
    auto scan = [&](int32_t lo, int32_t ln) {
        SPH_DIAG_ADD(8, wave_sum(ln));          // candidates
        SPH_DIAG_ADD(9, wave_max(ln >> 2));     // 4-candidate iterations
        SPH_DIAG_ADD(10, wave_max(ln & 3));     // tail iterations
        const int32_t n4 = ln >> 2;
        const float4* p = sp + lo;
        const float4* const pe = p + 4 * n4;
        int32_t it = 0;   // the group index: the same in every lane still scanning (uniform, a scalar register)
        for (; p < pe; p += 4, ++it) {
            const float4 a = p[0], bb = p[1], cc = p[2], d = p[3];
            const float ra = dist2(pi, a), rb = dist2(pi, bb), rc = dist2(pi, cc), rd = dist2(pi, d);
            float ua, ub, uc, ud;
            s += spline_w4(c, ra, ua);
            s += spline_w4(c, rb, ub);
            s += spline_w4(c, rc, uc);
            s += spline_w4(c, rd, ud);
            mh = __builtin_amdgcn_alignbit(mh, ml, 28u);
            bit(ua); bit(ub); bit(uc); bit(ud);
            // every eighth iteration the lanes still running (all of them at the same iteration, so the test is
            // wave-uniform) hold mn + 32 bits: store the oldest 32
            if ((it & 7) == 7) store((uint32_t)mn);
            keep_b128(a, bb, cc, d);
        }
        const int32_t pend = mn + 4 * (n4 & 7);   // the bits since the last store
        if (pend >= 32) store((uint32_t)(pend - 32));
        mn = pend & 31;
        // the 0–3 remaining candidates as one group of three (wave-uniform branch): the reads past the window
        // stay inside sp (the window ends at most at the staged data's end, and sp has 4 slots to spare) and
        // those candidates add a selected +0 and no bit; the k = ln mod 4 bits join the register pair in one
        // 64-bit shift. Sums and bits are those of k single steps (one), in the same order.
        const int32_t k = ln & 3;
        if (__any(k > 0)) {
            const float4* q = sp + lo + 4 * n4;
            const float4 a = q[0], bb = q[1], cc = q[2];
            float ua, ub, uc;
            const float wa = spline_w4(c, dist2(pi, a), ua);
            const float wb = spline_w4(c, dist2(pi, bb), ub);
            const float wc = spline_w4(c, dist2(pi, cc), uc);
            s += k > 0 ? wa : 0.0f;
            s += k > 1 ? wb : 0.0f;
            s += k > 2 ? wc : 0.0f;
            // sign bits (1: not a neighbour), oldest highest, then the k oldest kept
            const uint32_t f = ((__float_as_uint(ua) >> 31) << 2 | (__float_as_uint(ub) >> 31) << 1 |
                                (__float_as_uint(uc) >> 31)) >> (3 - k);
            const uint64_t m = ((uint64_t)mh << 32 | ml) << k | f;
            mh = (uint32_t)(m >> 32);
            ml = (uint32_t)m;
            mn += k;
            if (mn >= 32) {
                mn -= 32;
                store((uint32_t)mn);
            }
            keep_b128(a, bb, cc, cc);
        }
    };
    constexpr int nplanes = 2 * XS + 1;
#pragma unroll 1
    for (int p = 0; p < nplanes; ++p) {
        int32_t c0[3], c1[3], len[3], r0[3], r1[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            block_interval<XS>(g, cs, b, 3 * p + r, c0[r], c1[r]);
            len[r] = c1[r] - c0[r];
            lane_window<XS>(g, cs, b, valid, 3 * p + r, r0[r], r1[r]);
        }
        const int32_t total = len[0] + len[1] + len[2];
        // rows of mask gm staged back to back (they fit the budget together), each window scanned
        auto group = [&](uint32_t gm) {
            int32_t lg[3], tot = 0;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                lg[r] = (gm >> r & 1u) ? len[r] : 0;
                tot += lg[r];
            }
            __syncthreads();
            stage_plane<TT_STAGE_U>(c0, lg, tot, load_p, write_p);
            __syncthreads();
            int32_t o = 0;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                if (gm >> r & 1u) scan(o + (r0[r] - c0[r]), r1[r] - r0[r]);
                o += lg[r];
            }
        };
        // a row past the budget: in chunks, or straight from global memory
        auto big_row = [&](int r) {
            const int32_t lr = pick3(len, r), a0 = pick3(r0, r), a1 = pick3(r1, r), b0 = pick3(c0, r), b1 = pick3(c1, r);
            if (lr > TT_FALLBACK) {
                count_path(paths, 1);
                for (int32_t j = a0; j < a1; ++j) one(dist2(pi, pos[j]));
                return;
            }
#pragma unroll 1
            for (int32_t base = b0; base < b1; base += TT_GCAP) {
                const int32_t ln = min(TT_GCAP, b1 - base);
                __syncthreads();
                stage_run<TT_STAGE_U>(base, ln, load_p, write_p);
                __syncthreads();
                const int32_t lo = max(a0, base) - base;
                scan(lo, max(min(a1, base + ln) - base - lo, 0));
            }
        };
        if (total <= TT_GCAP) {
            group(7u);
            continue;
        }
        count_path(paths, 0);
        plane_groups(len, TT_GCAP, group, big_row);
    }
    SPH_BT_END(0);
    if (!valid) return;
    if (mn > 0 && wp < wend)   // the last, partial word: bits [0, mn), zeros above
        *wp = __builtin_bitreverse32(~ml << (32 - mn));
    const float2 out = density_eos(c, s);
    rp[i] = out;
    if (ro.dz) {   // slab step: a target of an own boundary column is also an entry of that side's ρ message
#pragma unroll
        for (int sd = 0; sd < 2; ++sd) {
            const uint32_t b = ro.dz->pick[1 + 2 * sd], e = ro.dz->pick[2 + 2 * sd];
            const uint32_t t = (uint32_t)i - b;
            if (ro.msg[sd] && (uint32_t)i >= b && (uint32_t)i < e && t < (uint32_t)ro.cap[sd]) ro.msg[sd][RHO_HDR + t] = out;
        }
    }
}

struct ForceAcc {
    float ax, ay, az, sx, sy, sz;
};

// Per-launch constants of the pair body, folded on the host from SphConst (SPEC_SPH.md §2), q = r/h:
//   W = σ·w4/4 with w4 = 4 + q²(3q − 6) (q < 1) or (2 − q)³;  G = −m·F (the kernel-gradient factor)
//   = 3mσ/h²·(1 − 0.75q) (q < 1) or 0.75mσ/h·(2 − q)²/r = kf·g with kf = 0.75mσ/h² and g = 4 − 3q or
//   (2 − q)²·h/r;  Π_ij·ρ̄ = 2·α·c0·h·min(v·r, 0)/(r² + η²);  XSPH ε·m·W/ρ̄ = kx·w4/(ρi + ρj).
// The pair body adds g- and w4-weighted terms; kf and kx scale the target's sums once, at the end, and
// g_in = −2 − (3q − 6) reuses w4's 3q − 6: two VALU fewer per pair than kin_a·q + kin_b (two SGPR operands:
// one move) and kx·(1/ρ̄)·w4. q itself is r²·rsq(r²)·(1/h), the oracle's sqrt(r²)·(1/h) to an ulp: near the
// support edge 2 − q cancels, and a q rounded another way (sqrt(r²/h²), measured) moves single-neighbour
// splash particles past the parity bound (tests/test_gpu_parity_headline.py).
struct PairK {
    float inv_h, h, kvisc, eta2, kf, kx;
    float two_h, m6h, four_h3, m2h;
};

static PairK pair_constants(const SphConst& c) {
    PairK k;
    k.inv_h = c.inv_h;
    k.h = c.h;
    k.kvisc = -2.0f * c.ac0 * c.h;            // inv_rbar = 2/(ρi + ρj)
    k.eta2 = c.eta2;
#if SPH_RUNITS
    // r units: the pair body's G and w4 carry one and three more factors of h than their q forms
    k.kf = 0.75f * c.mass * c.sigma_h2 * c.inv_h;
    k.kx = 0.5f * c.eps * c.mass * c.sigma / c.four_h3 * 4.0f;
#else
    k.kf = 0.75f * c.mass * c.sigma_h2;
    k.kx = 0.5f * c.eps * c.mass * c.sigma;
#endif
    k.two_h = c.two_h;
    k.m6h = c.m6h;
    k.four_h3 = c.four_h3;
    k.m2h = -c.two_h;
    return k;
}

// Pair body (SPEC_SPH.md §2). pj = (x, y, z, ρ_j), vj = (u, v, w, P_j/ρ_j²). Branchless, for
// pairs with q ≤ 2: one rsq gives r and 1/r; r = 0 (the target itself, or coincident distinct
// particles) gives q = 0 and adds ±0 along dx = 0. pair_terms evaluates a pair, pair_add adds it to the target's
// sums (the small-N pass evaluates pairs on many lanes and adds them in visit order on one, with the same roundings).
struct PairTerms {
    float cf, dx, dy, dz, cx, du, dv, dw;
};
__device__ __forceinline__ PairTerms pair_terms(const PairK& k, float4 pi, float4 vi, float rhoi, float prhoi, float4 pj,
                                                float4 vj) {
    const float dx = pi.x - pj.x, dy = pi.y - pj.y, dz = pi.z - pj.z;
    const float r2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));   // explicit chains: the same rounding on every path
    const float rs = __builtin_amdgcn_rsqf(fmaxf(r2, 1e-30f));
#if SPH_RUNITS
    // r units: w4·h³ = 4h³ + r²(3r − 6h) or (2h − r)³, G·h = 4h − 3r or (2h − r)²/r
    const float r = r2 * rs;
    const float t = k.two_h - r;
    const float t2 = t * t;
    const bool inner = r < k.h;
    const float c36 = fmaf(3.0f, r, k.m6h);
    const float w_in = fmaf(r2, c36, k.four_h3), w_out = t2 * t;
    const float g_in = k.m2h - c36, g_out = t2 * rs;
#else
    const float q = r2 * rs * k.inv_h;
    const float t = 2.0f - q;
    const float t2 = t * t;
    const bool inner = q < 1.0f;
    // both arms first, then a plain select (a ?: over expressions compiles to an exec branch)
    const float c36 = fmaf(3.0f, q, -6.0f);
    const float w_in = fmaf(q * q, c36, 4.0f), w_out = t2 * t;
    const float g_in = -2.0f - c36, g_out = t2 * rs * k.h;
#endif
    const float w4 = inner ? w_in : w_out;
    const float G = inner ? g_in : g_out;
    const float du = vi.x - vj.x, dv = vi.y - vj.y, dw = vi.z - vj.z;
    const float vr = fmaf(dw, dz, fmaf(dv, dy, du * dx));
    // one reciprocal for both 1/(ρi + ρj) and 1/((r² + η²)(ρi + ρj))
    const float e = r2 + k.eta2;
    const float inv_es = __builtin_amdgcn_rcpf(e * (rhoi + pj.w));
    const float inv_s = e * inv_es;
    const float pij = fminf(vr, 0.0f) * k.kvisc * inv_es;
    const float cf = (prhoi + vj.w + pij) * G;
    const float cx = inv_s * w4;
    return PairTerms{cf, dx, dy, dz, cx, du, dv, dw};
}
// the sums (the compiler contracts each into one fma: one rounding per term, in both forms)
__device__ __forceinline__ void pair_add(const PairTerms& t, ForceAcc& a) {
    a.ax += t.cf * t.dx; a.ay += t.cf * t.dy; a.az += t.cf * t.dz;
    a.sx -= t.cx * t.du; a.sy -= t.cx * t.dv; a.sz -= t.cx * t.dw;
}
__device__ __forceinline__ void pair_force(const PairK& k, float4 pi, float4 vi, float rhoi, float prhoi, float4 pj,
                                           float4 vj, ForceAcc& a) {
    pair_add(pair_terms(k, pi, vi, rhoi, prhoi, pj, vj), a);
}

// The end of pass 2 for target i in the small-N form (single context: no slab guard): the arithmetic of
// k_force_tiled's tail, expression for expression (the sums scaled once, KDK with the box walls, the next cell key).
template <int XS>
__device__ __forceinline__ uint32_t integrate_target(ForceAcc acc, const PairK& pk, const SphConst& c, const GridDesc& g,
                                                     float4 pi, float4 vi, float dt, float fext_x, int32_t i,
                                                     float4* __restrict__ pos_o, float4* __restrict__ vel_o,
                                                     uint32_t* __restrict__ keys_o) {
    acc.ax *= pk.kf; acc.ay *= pk.kf; acc.az *= pk.kf;
    acc.sx *= pk.kx; acc.sy *= pk.kx; acc.sz *= pk.kx;
    float nv[3] = {vi.x + (acc.ax + c.gx + fext_x) * dt, vi.y + (acc.ay + c.gy) * dt, vi.z + (acc.az + c.gz) * dt};
    float np[3] = {pi.x + (nv[0] + acc.sx) * dt, pi.y + (nv[1] + acc.sy) * dt, pi.z + (nv[2] + acc.sz) * dt};
    const float L[3] = {c.Lx, c.Ly, c.Lz};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (np[a] < 0.0f) { np[a] = 0.0f; if (nv[a] < 0.0f) nv[a] = -c.wall_e * nv[a]; }
        if (np[a] > L[a]) { np[a] = L[a]; if (nv[a] > 0.0f) nv[a] = -c.wall_e * nv[a]; }
    }
    pos_o[i] = make_float4(np[0], np[1], np[2], 0.f);
    vel_o[i] = make_float4(nv[0], nv[1], nv[2], 0.f);
    const uint32_t key = cell_key<XS>(g, np[0], np[1], np[2]);
    keys_o[i] = key;
    return key;
}

template <int XS>
__global__ __launch_bounds__(TF_BLK) __attribute__((amdgpu_waves_per_eu(4))) void k_force_tiled(
    const float4* __restrict__ pos, const float4* __restrict__ vel, const float2* __restrict__ rp,
    const uint32_t* __restrict__ cs, int32_t ib, int32_t n, GridDesc g, SphConst c, PairK pk, float dt,
    float fext_x, float4* __restrict__ pos_o, float4* __restrict__ vel_o, uint32_t* __restrict__ keys_o, MoverSink mv,
    HitMask hm, uint32_t* __restrict__ paths, DevRange dr, DevRange dr2, int32_t nb_a, SendBins sb,
    const uint2* __restrict__ sch) {
    __shared__ float4 sp[TF_GCAP + 4];     // (x, y, z, ρ)
    __shared__ float4 sv[TF_GCAP + 4];     // (u, v, w, P/ρ²)
    const int tid = threadIdx.x;
    int32_t blk = 0, i0, iend;
    int32_t rng = 0;       // which range (SendBins.side)
    if (sch) {   // single context: the y-band table (schedule.hip)
        if (!block_range<TF_BLK>(sch, ib, n, i0, iend)) return;   // whole workgroup: before any barrier
    } else {
        blk = xcd_block(blockIdx.x, gridDim.x);
        int32_t nb_r = nb_a;   // this range's workgroups
        if (dr2.lo && blk >= nb_a) {   // a second range in the same launch (the slab step's two boundary columns)
            blk -= nb_a;
            nb_r = (int32_t)gridDim.x - nb_a;
            dr = dr2;
            rng = 1;
        }
        if (dr.lo) {   // device-resident bounds (slab step); the grid is an upper bound
            ib = (int32_t)*dr.lo;
            n = (int32_t)*dr.hi;
            // a range past its grid (a bound from an earlier step's count) stops every rank, as a message overflow does
            if (blk == 0 && tid == 0 && mv.err && n - ib > nb_r * TF_BLK) atomicOr(mv.err, SZ_OVF_CAP);
        }
        i0 = ib + blk * TF_BLK;
        if (i0 >= n) return;   // whole workgroup: before any barrier
        iend = min(i0 + TF_BLK, n);
    }
    SPH_BT_START;
    // Targets stay in sorted order here. Lanes ordered by quarters of fx (a dx plane's hit count follows
    // fx) fill the plane loop better (66% -> 80% of lanes busy at C3) but run slower, 206 -> 246 us, and
    // by halves of fx (83%) 190 -> 229 us: the lanes of a wave then come from more z layers and read
    // scattered LDS slots (profiles/r02_direct_plane_ab.log, r02_fx2_noself_ab.log).
    const int32_t i = i0 + tid;
    const bool valid = i < iend;
    const int32_t ilast = iend - 1;
    const int32_t ii = valid ? i : ilast;
    const float4 pi = pos[ii], vi = vel[ii];
    const float2 ri = rp[ii];
    const BlockRows b = block_rows<XS>(g, pos, i0, ilast, pi);
    ForceAcc acc{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // hit-mask reader (pass 1's bits of this target, in visit order): rb holds rn bits, LSB next;
    // the remaining words wait in a queue of registers (static indices only). Measured against a
    // one-word prefetch from global memory (with and without 5 waves per SIMD): the queue is 2-3%
    // faster on the force pass (profiles/r02_hitmask_ab.log).
    uint32_t q[HM_WORDS];
#pragma unroll
    for (int w = 0; w < HM_WORDS; ++w) q[w] = (valid && hm.w) ? hm.w[(size_t)w * hm.stride + i] : 0u;
    uint64_t rb = (uint64_t)q[0] | ((uint64_t)q[1] << 32);
    int32_t rn = 64, kb = 0;   // kb: candidates of this target so far (the bit index of the next window)
    auto take = [&](int32_t len) -> uint32_t {   // the next len (0..32) bits
        const uint32_t v = (uint32_t)rb & (len >= 32 ? 0xffffffffu : ((1u << len) - 1u));
        rb >>= len;
        rn -= len;
        if (rn <= 32) {
            rb |= (uint64_t)q[2] << rn;
            rn += 32;
#pragma unroll
            for (int w = 2; w + 1 < HM_WORDS; ++w) q[w] = q[w + 1];
            q[HM_WORDS - 1] = 0u;
        }
        return v;
    };
    auto skip = [&](int32_t ln) {
        for (int32_t off = 0; __any(off < ln); off += 32) (void)take(max(0, min(32, ln - off)));
    };
    // The pair loop over the next nb bits of the mask, 128 at a time (four words), one hit per
    // iteration: bit b is candidate b of up to three windows back to back (lengths l0, e2 − l0 and the
    // rest), at LDS slot b + d0, d1 or d2. Lanes idle only at the end of a piece (one piece per plane
    // at C3: 54% -> 66% of lanes busy against the 16-entry hit lists this replaced, 36% -> 53%
    // mid-collapse). Words are consumed from w0; an emptied w0 takes the next word (an all-zero word
    // in the middle costs the lane one idle iteration).
    auto walk = [&](int32_t nb, int32_t l0, int32_t e2, int32_t d0, int32_t d1, int32_t d2) {
        for (int32_t off = 0; __any(off < nb); off += 128) {
            const int32_t rem = nb - off;
            uint32_t w0 = take(min(max(rem, 0), 32)), w1 = take(min(max(rem - 32, 0), 32));
            uint32_t w2 = take(min(max(rem - 64, 0), 32)), w3 = take(min(max(rem - 96, 0), 32));
            int32_t nh = (int32_t)(__popc(w0) + __popc(w1) + __popc(w2) + __popc(w3));
            int32_t base = off;
            SPH_DIAG_ADD(11, wave_sum(nh));   // pairs
            SPH_DIAG_ADD(12, wave_max(nh));   // loop iterations
            SPH_DIAG_ADD(13, 1);              // loops
            // SPH_WALK_UNROLL hits per loop trip: fewer loop and exec-mask instructions per hit, and the next
            // hit's slot and LDS reads can issue before the current pair body ends. Force pass 189 -> 181 us
            // from rest, 214 -> 203 us mid-collapse at 4 (2: 184, 3: 182 us; the word shift as selects instead
            // of a branch: no change; profiles/r02_walk_unroll_ab.log). The trip test sits at the bottom
            // (do-while): with it at the top the compiler copied the six accumulators twice per trip (12 moves
            // for 4 hits); force pass 171.3 -> 167.6 us from rest, 193.2 -> 189.1 mid-collapse
            // (profiles/r03_walk_dowhile_ab.log).
            if (__any(nh > 0)) do {
#pragma unroll
                for (int u = 0; u < SPH_WALK_UNROLL; ++u) {
                    if (w0 != 0u) {
                        const int32_t bi = base + (int32_t)__builtin_ctz(w0);
                        w0 &= w0 - 1u;
                        --nh;
                        const int32_t slot = bi + (bi < l0 ? d0 : (bi < e2 ? d1 : d2));
                        pair_force(pk, pi, vi, ri.x, ri.y, sp[slot], sv[slot], acc);
                    }
                    // the next word moves up, as selects: as a branch the compiler copied each queue word into a
                    // new register every step (3 moves + 4 masked moves per step; force pass 189.2 -> 187.7 us
                    // mid-collapse, profiles/r03_walk_select_shift_ab.log)
                    const bool z = w0 == 0u;
                    w0 = z ? w1 : w0;
                    w1 = z ? w2 : w1;
                    w2 = z ? w3 : w2;
                    w3 = z ? 0u : w3;
                    base += z ? 32 : 0;
                }
            } while (__any(nh > 0));
        }
    };
    // Planes the mask does not cover (a target past its 256 bits): LDS slots [lo, lo+ln) by distance,
    // in visit order. The target itself is a hit: its pair adds exactly ±0 (dx = du = 0, q = 0 finite).
    auto dscan = [&](int32_t lo, int32_t ln) {
        for (int32_t t = 0; __any(t < ln); ++t) {
            if (t < ln) {
                const float4 pj = sp[lo + t];
                if (is_hit(c, dist2(pi, pj))) pair_force(pk, pi, vi, ri.x, ri.y, pj, sv[lo + t], acc);
            }
        }
    };
    auto load_f = [&](int32_t src) { return Staged{pos[src], vel[src], rp[src]}; };
    auto write_f = [&](int32_t t, const Staged& e) {
        sp[t] = make_float4(e.p.x, e.p.y, e.p.z, e.r.x);
        sv[t] = make_float4(e.v.x, e.v.y, e.v.z, e.r.y);
    };
    constexpr int nplanes = 2 * XS + 1;
#pragma unroll 1
    for (int p = 0; p < nplanes; ++p) {
        int32_t c0[3], c1[3], len[3], r0[3], r1[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            block_interval<XS>(g, cs, b, 3 * p + r, c0[r], c1[r]);
            len[r] = c1[r] - c0[r];
            lane_window<XS>(g, cs, b, valid, 3 * p + r, r0[r], r1[r]);
        }
        const int32_t total = len[0] + len[1] + len[2];
        const int32_t plen = (r1[0] - r0[0]) + (r1[1] - r0[1]) + (r1[2] - r0[2]);
        // the mask covers this plane for every lane of the wave (wave-uniform)
        const bool by_mask = hm.w != nullptr && !__any(kb + plen > HM_WORDS * 32);
        kb += plen;
        if (!by_mask) {   // this plane scans by distance (its bits, if any, are passed over)
            count_wave(paths, 4);
            if (hm.w != nullptr) skip(plen);
        }
        // rows of mask gm staged back to back (they fit the budget together); the mask walk takes their
        // windows' bits in visit order (rows outside gm count zero bits)
        auto group = [&](uint32_t gm) {
            int32_t lg[3], wg[3], tot = 0;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                lg[r] = (gm >> r & 1u) ? len[r] : 0;
                wg[r] = (gm >> r & 1u) ? r1[r] - r0[r] : 0;
                tot += lg[r];
            }
            __syncthreads();
            stage_plane<TF_STAGE_U, TF_BLK>(c0, lg, tot, load_f, write_f);
            __syncthreads();
            if (by_mask) {
                const int32_t l0 = wg[0], e2 = l0 + wg[1];
                walk(e2 + wg[2], l0, e2, r0[0] - c0[0], lg[0] + (r0[1] - c0[1]) - l0,
                     lg[0] + lg[1] + (r0[2] - c0[2]) - e2);
            } else {
                int32_t o = 0;
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    if (gm >> r & 1u) dscan(o + (r0[r] - c0[r]), wg[r]);
                    o += lg[r];
                }
            }
        };
        // a row past the budget: in chunks (the chunks take the row's bits in order), or straight from
        // global memory
        auto big_row = [&](int r) {
            const int32_t lr = pick3(len, r), a0 = pick3(r0, r), a1 = pick3(r1, r), b0 = pick3(c0, r), b1 = pick3(c1, r);
            if (lr > TF_FALLBACK) {
                count_path(paths, 3);
                if (by_mask) skip(a1 - a0);
                for (int32_t j = a0; j < a1; ++j) {
                    const float4 pj = pos[j];
                    if (j != i && is_hit(c, dist2(pi, pj))) {
                        const float4 vj = vel[j];
                        const float2 rj = rp[j];
                        pair_force(pk, pi, vi, ri.x, ri.y, make_float4(pj.x, pj.y, pj.z, rj.x),
                                   make_float4(vj.x, vj.y, vj.z, rj.y), acc);
                    }
                }
                return;
            }
#pragma unroll 1
            for (int32_t base = b0; base < b1; base += TF_GCAP) {
                const int32_t ln = min(TF_GCAP, b1 - base);
                __syncthreads();
                stage_run<TF_STAGE_U, TF_BLK>(base, ln, load_f, write_f);
                __syncthreads();
                const int32_t lo = max(a0, base) - base;
                const int32_t wl = max(min(a1, base + ln) - base - lo, 0);
                if (by_mask)
                    walk(wl, wl, wl, lo, 0, 0);
                else
                    dscan(lo, wl);
            }
        };
        if (total <= TF_GCAP) {
            group(7u);
            continue;
        }
        count_path(paths, 2);
        plane_groups(len, TF_GCAP, group, big_row);
    }
    count_wave(paths, 5);   // waves (3 planes each)
    SPH_BT_END(1);
    if (!valid) return;
    // integrate_target's arithmetic, kept inline here: as a call the kernel's scalar arguments spilled to lanes
    acc.ax *= pk.kf; acc.ay *= pk.kf; acc.az *= pk.kf;
    acc.sx *= pk.kx; acc.sy *= pk.kx; acc.sz *= pk.kx;
    float nv[3] = {vi.x + (acc.ax + c.gx + fext_x) * dt, vi.y + (acc.ay + c.gy) * dt, vi.z + (acc.az + c.gz) * dt};
    float np[3] = {pi.x + (nv[0] + acc.sx) * dt, pi.y + (nv[1] + acc.sy) * dt, pi.z + (nv[2] + acc.sz) * dt};
    const float L[3] = {c.Lx, c.Ly, c.Lz};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (np[a] < 0.0f) { np[a] = 0.0f; if (nv[a] < 0.0f) nv[a] = -c.wall_e * nv[a]; }
        if (np[a] > L[a]) { np[a] = L[a]; if (nv[a] > 0.0f) nv[a] = -c.wall_e * nv[a]; }
    }
    pos_o[i] = make_float4(np[0], np[1], np[2], 0.f);
    vel_o[i] = make_float4(nv[0], nv[1], nv[2], 0.f);
    const uint32_t key = cell_key<XS>(g, np[0], np[1], np[2]);
    keys_o[i] = key;
    // the mover list takes the window key: in a slab, a particle that left the held columns sorts
    // last (window_key = cell_key in a single domain); it changed iff the clamped key changed
    const uint32_t wk = window_key<XS>(g, np[0], np[1], np[2]);
    if (mv.jump && mv.sk) {   // slab step: the next sends assume moves of at most one column (slab.hip send_ranges)
        const uint32_t gyz = col_keys<XS>(g);
        const int32_t d = (int32_t)(wk / gyz) - (int32_t)(mv.sk[i] / gyz);
        if (wk >= g.ncells) {
            if (mv.err) atomicOr(mv.err, SZ_JUMP);   // left the held window: it reaches no neighbour
        } else if (d > 1 || d < -1) {
            if (mv.jump_err) atomicOr(mv.err, SZ_JUMP_EARLY);
            else *mv.jump = 1u;
        }
    }
    if (sb.bins && sb.side[rng] >= 0) {   // early sends: this wave's count for its send block (workgroup-uniform test)
        const int32_t sd = sb.side[rng], col = (int32_t)(key / col_keys<XS>(g));
        const bool snd = sd == 0 ? col <= sb.col_le : col >= sb.col_ge;
        const uint64_t act = __ballot(1), m = __ballot(snd);
        if (m != 0ull && lane_id() == (uint32_t)(__ffsll((long long)act) - 1))
            atomicAdd(sb.bins + sd * sb.nblk + (blk * TF_BLK) / SEND_SLOTS, (uint32_t)__popcll(m));
    }
    append_mover(mv, i, wk);
}

// ---------------------------------------------------------------- small N
// At the reference's own scale (a few thousand particles, ParticleSystemController.cs:12) the tiled passes run a
// handful of 256-target workgroups on a 256-CU chip (C1: 16), each walking its planes one after another. The small
// form gives every target one wave: lane k < rows finds row k's trimmed window (lane_window, the tiled passes'
// windows), the rows' windows back to back are the visit order, and each 64-candidate chunk of it is evaluated one
// candidate per lane, its loads in flight together. The sums are then taken in visit order from the lanes
// (readlane): pass 1 adds every candidate's w (non-neighbours add +0), pass 2 adds the hits' pair terms, each with
// the tiled passes' expression, so the results are bit-identical to theirs (tests/test_gpu_small.py). Pass 2 takes
// its hits by distance (is_hit: the bit pass 1 records), so no hit mask passes between the two.
template <int XS>
struct SmallRows {
    static constexpr int NR = 3 * (2 * XS + 1);   // rows in visit order
    uint32_t rj0 = 0u, excl = 0u, total = 0u;     // lane k < NR: row k's first slot and flattened start
    uint32_t P[NR];                               // the rows' flattened starts (wave-uniform)
    __device__ __forceinline__ SmallRows(const GridDesc& g, const uint32_t* __restrict__ cs, float4 pi, int lane) {
        BlockRows b;
        b.cx = cell_cxs<XS>(g, pi.x);
        b.cy = cell_coord(pi.y, g.oy, g.inv_cell, g.gy);
        cell_fracs<XS>(g, pi.x, pi.y, pi.z, b.cx, b.cy, b.fx, b.fy, b.gzf);
        uint32_t len = 0u;
        if (lane < NR) {
            int32_t r0, r1;
            lane_window<XS>(g, cs, b, true, lane, r0, r1);
            rj0 = (uint32_t)r0;
            len = (uint32_t)(r1 - r0);
        }
        prefix(len, lane);
    }
    // the same rows from a permutation's cell starts (fused_perm.h: the one-launch steps)
    __device__ __forceinline__ SmallRows(const GridDesc& g, const FusedMap& M, float4 pi, int lane) {
        BlockRows b;
        b.cx = cell_cxs<XS>(g, pi.x);
        b.cy = cell_coord(pi.y, g.oy, g.inv_cell, g.gy);
        cell_fracs<XS>(g, pi.x, pi.y, pi.z, b.cx, b.cy, b.fx, b.fy, b.gzf);
        // both table reads of a row first, then the map's searches: one memory round trip, not two
        uint32_t len = 0u, ka = 0u, kb = 0u;
        bool in_row = false;
        if (lane < NR) {
            const int32_t dxk = lane / 3 - XS, dyk = lane % 3 - 1;
            const int32_t xx = b.cx + dxk, yy = b.cy + dyk;
            int32_t zlo, zhi;
            if (xx >= 0 && xx < g.gx * XS && yy >= 0 && yy < g.gy &&
                row_window<XS>(g, b.fx, b.fy, b.gzf, dxk, dyk, zlo, zhi)) {
                const uint32_t rowk = ((uint32_t)xx * (uint32_t)g.gy + (uint32_t)yy) * (uint32_t)g.gz;
                ka = rowk + (uint32_t)zlo;
                kb = rowk + (uint32_t)zhi + 1u;
                in_row = true;
            }
        }
        const uint32_t ca = M.cs[ka], cb = M.cs[kb];   // (key 0 for lanes without a row: in bounds, unused)
        if (in_row) {
            rj0 = M.start_c(ka, ca);
            len = M.start_c(kb, cb) - rj0;
        }
        prefix(len, lane);
    }
    __device__ __forceinline__ void prefix(uint32_t len, int) {
        const uint32_t incl = row_scan_incl(len);   // rows on lanes 0..NR-1 (NR <= 15)
        excl = incl - len;
#pragma unroll
        for (int k = 0; k < NR; ++k) P[k] = (uint32_t)__builtin_amdgcn_readlane((int)excl, k);
        total = (uint32_t)__builtin_amdgcn_readlane((int)incl, NR - 1);
    }
    // flattened candidate f -> sorted slot (the row's first slot and start from its lane, not a per-lane select
    // chain: that compiles to a scratch-memory table)
    __device__ __forceinline__ uint32_t slot(uint32_t f) const {
        int k = 0;
#pragma unroll
        for (int r = 1; r < NR; ++r) k += f >= P[r] ? 1 : 0;
        return (uint32_t)__shfl((int)rj0, k, 64) + (f - (uint32_t)__shfl((int)excl, k, 64));
    }
};

__device__ __forceinline__ float lanef(float v, uint32_t src) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)src));
}

// s + w over the wave's lanes in lane (visit) order, taking only the lanes whose w is not ±0: s starts at +0 and the
// weights are ≥ +0, so s is never −0 and adding a zero term leaves it unchanged bit for bit (NaN terms are kept).
__device__ __forceinline__ float visit_sum(float s, float w) {
    for (uint64_t m = __ballot(w != 0.0f); m; m &= m - 1ull) s += lanef(w, (uint32_t)__builtin_ctzll(m));
    return s;
}

// The force sums of a wave's hits in visit order, transposed: lane c < 6 accumulates component c (the a = cf·d and
// s = −cx·du products of pair_add, the same fused multiply-adds in the same order), reading each hit's terms from
// the wave's LDS row instead of eight lane reads per hit.
struct HitTerms {
    float4 a, b;   // (cf, dx, dy, dz), (cx, du, dv, dw)
};
__device__ __forceinline__ float hit_fold(float acc, const HitTerms* row, uint64_t m, int lane) {
    const float* base = reinterpret_cast<const float*>(row);
    const int pi = lane < 3 ? 0 : 4;                      // cf or cx
    const int qi = lane < 3 ? 1 + lane : 5 + (lane - 3);  // dx, dy, dz or du, dv, dw
    const float sg = lane < 3 ? 1.0f : -1.0f;
    while (__popcll(m) >= 4) {   // four hits' reads in flight, then their four multiply-adds in order
        float p[4], q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int su = __builtin_ctzll(m);
            m &= m - 1ull;
            p[u] = sg * base[8 * su + pi];
            q[u] = base[8 * su + qi];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = fmaf(p[u], q[u], acc);
    }
    while (m) {
        const int s0 = __builtin_ctzll(m);
        m &= m - 1ull;
        acc = fmaf(sg * base[8 * s0 + pi], base[8 * s0 + qi], acc);
    }
    return acc;
}

template <int XS>
__global__ __launch_bounds__(256) void k_density_small(const float4* __restrict__ pos, const uint32_t* __restrict__ cs,
                                                       int32_t n, GridDesc g, SphConst c, float2* __restrict__ rp) {
    const int lane = (int)lane_id();
    const int32_t i = (int32_t)blockIdx.x * 4 + (int32_t)(threadIdx.x >> 6);
    if (i >= n) return;   // wave-uniform
    const float4 pi = pos[i];
    const SmallRows<XS> R(g, cs, pi, lane);
    float s = 0.0f;
#pragma unroll 1
    for (uint32_t base = 0; base < R.total; base += 64u) {
        const uint32_t f = base + (uint32_t)lane;
        float v;
        const float w4 = spline_w4(c, dist2(pi, pos[R.slot(min(f, R.total - 1u))]), v);
        const float w = f < R.total ? w4 : 0.0f;
        s = visit_sum(s, w);
    }
    if (lane == 0) rp[i] = density_eos(c, s);
}

template <int XS>
__global__ __launch_bounds__(256) void k_force_small(const float4* __restrict__ pos, const float4* __restrict__ vel,
                                                     const float2* __restrict__ rp, const uint32_t* __restrict__ cs,
                                                     int32_t n, GridDesc g, SphConst c, PairK pk, float dt, float fext_x,
                                                     float4* __restrict__ pos_o, float4* __restrict__ vel_o,
                                                     uint32_t* __restrict__ keys_o, MoverSink mv) {
    const int lane = (int)lane_id();
    const int32_t i = (int32_t)blockIdx.x * 4 + (int32_t)(threadIdx.x >> 6);
    if (i >= n) return;   // wave-uniform
    const float4 pi = pos[i], vi = vel[i];
    const float2 ri = rp[i];
    const SmallRows<XS> R(g, cs, pi, lane);
    __shared__ HitTerms rows[4][64];
    HitTerms* row = rows[threadIdx.x >> 6];
    float comp = 0.0f;   // lane c < 6: component c of the sums (pair_add's ax, ay, az, sx, sy, sz)
#pragma unroll 1
    for (uint32_t base = 0; base < R.total; base += 64u) {
        const uint32_t f = base + (uint32_t)lane;
        const uint32_t j = R.slot(min(f, R.total - 1u));
        // a candidate's velocity and pass-1 terms load with its position whether or not it is a hit: one memory round
        // trip per round instead of two (the hit test waited for the position before the others issued)
        const float4 pj = pos[j], vj = vel[j];
        const float2 rj = rp[j];
        const bool hit = f < R.total && is_hit(c, dist2(pi, pj));
        if (hit) {
            const PairTerms t =
                pair_terms(pk, pi, vi, ri.x, ri.y, make_float4(pj.x, pj.y, pj.z, rj.x), make_float4(vj.x, vj.y, vj.z, rj.y));
            row[lane] = HitTerms{make_float4(t.cf, t.dx, t.dy, t.dz), make_float4(t.cx, t.du, t.dv, t.dw)};
        }
        const uint64_t m = __ballot(hit);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < 6) comp = hit_fold(comp, row, m, lane);   // the hits in visit order
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const ForceAcc acc{lanef(comp, 0), lanef(comp, 1), lanef(comp, 2), lanef(comp, 3), lanef(comp, 4), lanef(comp, 5)};
    if (lane != 0) return;
    const uint32_t key = integrate_target<XS>(acc, pk, c, g, pi, vi, dt, fext_x, i, pos_o, vel_o, keys_o);
    append_mover(mv, i, key);   // one lane: window_key = cell_key in a single domain
}

// The one-launch re-sort + pass 1 at the reference's scale (n <= FZ_N, fused_perm.h): each workgroup rebuilds the
// step's permutation from the previous step's movers, every wave takes one target at its sorted position, reads the
// previous order through the permutation, sums pass 1 exactly as k_density_small and writes the target's (x, v, id,
// sorted key) at its sorted position, so pass 2 (k_force_small) runs on the sorted arrays as after the re-sort. Two
// launches per step instead of three, bit-identical (tests/test_gpu_small.py).
constexpr int FZS_BLK = 1024;
template <int XS>
__device__ __forceinline__ void density_fused_target(const FusedIOS& io, const FusedMap& M, int32_t i, int lane,
                                                     const GridDesc& g, const SphConst& c) {
    bool mv;
    uint32_t key_mv;
    const uint32_t o = M.old_at((uint32_t)i, mv, key_mv);
    const float4 pi = io.pos[o];
    const float4 vi = io.vel[o];   // written at the end: loaded under the sums
    const int32_t idi = io.id[o];
    const uint32_t sko = io.sk[o];   // whether or not a mover: a load under a branch was waited before the others issued
    const uint32_t key = mv ? key_mv : sko;
    const SmallRows<XS> R(g, M, pi, lane);
    float s = 0.0f;
#pragma unroll 1
    for (uint32_t base = 0; base < R.total; base += 64u) {
        const uint32_t f = base + (uint32_t)lane;
        float v;
        const float w4 = spline_w4(c, dist2(pi, io.pos[M.old(R.slot(min(f, R.total - 1u)))]), v);
        const float w = f < R.total ? w4 : 0.0f;
        s = visit_sum(s, w);
    }
    if (lane != 0) return;
    io.rp_o[i] = density_eos(c, s);
    io.pos_o[i] = pi;
    io.vel_o[i] = vi;
    io.id_o[i] = idi;
    io.sk_o[i] = key;
}

template <int XS>
__global__ __launch_bounds__(FZS_BLK) void k_density_fused(FusedIOS io, int32_t n, GridDesc g, SphConst c) {
    __shared__ FusedLds L;
    const FusedMap M = fused_build<FZS_BLK>(L, io.count, io.mi, io.mk, io.cs, n, io.count_zero, io.host_count);
    const int lane = (int)lane_id();
    const int32_t i = (int32_t)blockIdx.x * (FZS_BLK / 64) + (int32_t)(threadIdx.x >> 6);
    if (i < n) {   // wave-uniform
        density_fused_target<XS>(io, M, i, lane, g, c);
    }
    // the workgroup's share of the new cell-start table, each wave after its target
    fused_cs_share(M, io.cs_o, g.ncells, threadIdx.x, FZS_BLK);
}

int32_t density_fused_max() { return FZ_N; }

void launch_density_fused(const FusedIOS& io, int32_t n, GridDesc g, SphConst c, hipStream_t s) {
    if (n <= 0 || n > FZ_N) return;
    const int32_t grid = (n + FZS_BLK / 64 - 1) / (FZS_BLK / 64);
    if (g.xsub == 2)
        SPH_LAUNCH(k_density_fused<2>, grid, FZS_BLK, 0, s, io, n, g, c);
    else
        SPH_LAUNCH(k_density_fused<1>, grid, FZS_BLK, 0, s, io, n, g, c);
}

void launch_density_small(const float4* pos, const uint32_t* cs, int32_t n, GridDesc g, SphConst c, float2* rp,
                          hipStream_t s) {
    if (n <= 0) return;
    if (g.xsub == 2)
        SPH_LAUNCH(k_density_small<2>, (n + 3) / 4, 256, 0, s, pos, cs, n, g, c, rp);
    else
        SPH_LAUNCH(k_density_small<1>, (n + 3) / 4, 256, 0, s, pos, cs, n, g, c, rp);
}

void launch_force_small(const float4* pos, const float4* vel, const float2* rp, const uint32_t* cs, int32_t n, GridDesc g,
                        SphConst c, float dt, float fext_x, float4* pos_o, float4* vel_o, uint32_t* keys_o, MoverSink mv,
                        hipStream_t s) {
    if (n <= 0) return;
    if (g.xsub == 2)
        SPH_LAUNCH(k_force_small<2>, (n + 3) / 4, 256, 0, s, pos, vel, rp, cs, n, g, c, pair_constants(c), dt, fext_x,
                   pos_o, vel_o, keys_o, mv);
    else
        SPH_LAUNCH(k_force_small<1>, (n + 3) / 4, 256, 0, s, pos, vel, rp, cs, n, g, c, pair_constants(c), dt, fext_x,
                   pos_o, vel_o, keys_o, mv);
}

// dr set: [ib, ie) only sizes the grid (an upper bound); the kernels read their bounds from dr
// ro.dz set: the launch also writes the slab step's ρ messages (headers by block 0, even when the grid has no
// targets: then ie <= ib must not skip it)
void launch_density_tiled(const float4* pos, const uint32_t* cs, int32_t ib, int32_t ie, GridDesc g, SphConst c,
                          float2* rp, HitMask hm, uint32_t* paths, hipStream_t s, DevRange dr, RhoOut ro, Sched sch) {
    if (ie <= ib && !ro.dz) return;
    const bool tab = sch.table && !dr.lo && ib == 0;
    const int32_t nb = tab ? sch.entries : (ie > ib ? (ie - ib + TT_BLK - 1) / TT_BLK : 1);
    const uint2* t = tab ? sch.table : nullptr;
    if (g.xsub == 2)
        SPH_LAUNCH(k_density_tiled<2>, nb, TT_BLK, 0, s, pos, cs, ib, ie, g, c, rp, dr, hm, paths, ro, t);
    else
        SPH_LAUNCH(k_density_tiled<1>, nb, TT_BLK, 0, s, pos, cs, ib, ie, g, c, rp, dr, hm, paths, ro, t);
}

// dr2 set: a second device-resident range in the same launch, ie2 slots at most (its workgroups follow
// the first range's (ie - ib) / TF_BLK)
void launch_force_tiled(const float4* pos, const float4* vel, const float2* rp, const uint32_t* cs, int32_t ib,
                        int32_t ie, GridDesc g, SphConst c, float dt, float fext_x, float4* pos_o, float4* vel_o,
                        uint32_t* keys_o, MoverSink mv, HitMask hm, uint32_t* paths, hipStream_t s, DevRange dr,
                        DevRange dr2, int32_t ie2, SendBins sb, Sched sch) {
    const int32_t nb_a = ie > ib ? (ie - ib + TF_BLK - 1) / TF_BLK : 0;
    const int32_t nb_b = dr2.lo && ie2 > 0 ? (ie2 + TF_BLK - 1) / TF_BLK : 0;
    if (nb_a + nb_b == 0) return;
    // the table's blocks hold up to 256 targets: a build with other force workgroups (make variants) keeps its mapping
    const bool tab = sch.table && TF_BLK == 256 && !dr.lo && !dr2.lo && ib == 0 && !sb.bins;
    const int32_t nb = tab ? sch.entries : nb_a + nb_b;
    const uint2* t = tab ? sch.table : nullptr;
    if (g.xsub == 2)
        SPH_LAUNCH(k_force_tiled<2>, nb, TF_BLK, 0, s, pos, vel, rp, cs, ib, ie, g, c, pair_constants(c), dt,
                   fext_x, pos_o, vel_o, keys_o, mv, hm, paths, dr, nb_b ? dr2 : DevRange{}, nb_b ? nb_a : nb_a + nb_b, sb, t);
    else
        SPH_LAUNCH(k_force_tiled<1>, nb, TF_BLK, 0, s, pos, vel, rp, cs, ib, ie, g, c, pair_constants(c), dt,
                   fext_x, pos_o, vel_o, keys_o, mv, hm, paths, dr, nb_b ? dr2 : DevRange{}, nb_b ? nb_a : nb_a + nb_b, sb, t);
}

#ifdef SPH_BTIME
extern "C" int sph_debug_block_times(uint64_t* out, int32_t count) {   // count <= 2 * BT_MAX * 2
    if (!out || count < 0 || count > 2 * BT_MAX * 2) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_btime), (size_t)count * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace sph
