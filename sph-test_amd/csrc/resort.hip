// resort.hip — incremental stable re-sort of a Model S step (SPEC_SPH.md §0 "Sort"), gfx950.
//
// After a step the particles are still in the previous step's sorted order, and the force pass
// has written each particle's new cell key. A key changes only when the particle crosses a
// sub-cell boundary (~0.5% of the particles per step on C3). The "stayers" (unchanged key) form
// a subsequence that is already sorted by (key, index), because their keys are the previous
// sorted keys. The force pass appends the "movers" (append_mover, common.h; any order). Their
// destinations, and the stayers', follow from counting alone:
//
//   stayer i : dst = (i − A(i)) + #{movers x : (k_x, x) < (k_i, i)}
//   mover  x : dst = (q − A(q)) + #{movers y : (k_y, y) < (k_x, x)},
//              q = clamp(x, cs_old[k_x], cs_old[k_x + 1])
//
// A(q) = #movers with index < q, and cs_old is the previous cell-start table. Stayers with a key
// below k_x sit exactly below cs_old[k_x]. Stayers with key k_x and a smaller index sit in
// [cs_old[k_x], q). (key, index) is the total order the stable LSD radix sort realises, so the
// permutation is bit-identical to the full sort's. All counts are order-independent (the append
// order does not matter), so every output is deterministic; the only atomics are integer adds.
// tests/test_resort_logic.py restates the formulas; tests/test_gpu_resort.py compares runs bit
// for bit with the full sort.
//
// Kernels:
//   k_mv_rank        counts per mover against every 64-mover tile (sorted in LDS, binary searches):
//                    (key, index) rank, index rank, A(q)
//   k_mv_place       movers: scatter of (pos, vel, id, key); tables by (key, index) and by index
//   k_mv_merge       stayers: scatter of (pos, vel, id, key); extra workgroups update the cell
//                    starts in place: cs[k] += #{movers: new key < k} − #{movers: old key < k}
// The scatters replace the permutation gather, and the update the cell-start rebuild, of the full path.
#include "common.h"

namespace sph {

constexpr int MV_BLK = 256;
// movers per rank tile: 64 gives ~4x the work items of 256 for a few more atomics (256 -> 64 was
// faster in every paired round, C3 re-sort ~42 -> ~39 us; 32 and 128 are within the run-to-run noise
// of 64, profiles/r01_mv_tile_ab.log)
constexpr int MV_TILE = 64;
constexpr int MV_RANK_GRID = 2048;

static __device__ __forceinline__ uint64_t comp(uint32_t key, uint32_t idx) { return (uint64_t)key << 32 | idx; }

static __device__ __forceinline__ bool asm_rec(const AsmSrc& a, int32_t x) { return x < a.nl || x >= a.nre; }

// Model R's other slot arrays (single domain: slot x is x)
static __device__ __forceinline__ void move_extra(const ResortExtra& ex, uint32_t x, uint32_t dst) {
    if (!ex.omg) return;
    ex.omg_o[dst] = ex.omg[x];
    ex.rot_o[dst] = ex.rot[x];
    ex.aux_o[dst] = ex.aux[x];
    ex.mode_o[dst] = ex.mode[x];
}

static __device__ __forceinline__ uint32_t asm_sk(const AsmSrc& a, int32_t x) {
    return asm_rec(a, x) ? a.skr[x] : a.sk[x + a.o_off];
}

static __device__ __forceinline__ uint32_t asm_key(const AsmSrc& a, int32_t x) {
    return asm_rec(a, x) ? a.keyr[x] : a.keys[x + a.o_off];
}

// a mover entry's slot in the array being re-sorted (see MV_REC)
static __device__ __forceinline__ uint32_t mv_slot(const ResortScratch& w, uint32_t mi) {
    return (mi & MV_REC) ? (mi & ~MV_REC) : mi + (uint32_t)w.mi_off;
}

// a halo record reads as the slab assemble's unpack wrote it: (x, y, z, 0), (u, v, w, 0), id
static __device__ __forceinline__ void asm_load(const AsmSrc& a, int32_t x, float4& p, float4& v, int32_t& id) {
    if (asm_rec(a, x)) {
        const float4* r = x < a.nl ? a.rl + 2 * (size_t)x : a.rr + 2 * (size_t)(x - a.nre);
        const float4 r0 = r[0], r1 = r[1];
        p = make_float4(r0.x, r0.y, r0.z, 0.f);
        v = make_float4(r1.x, r1.y, r1.z, 0.f);
        id = __float_as_int(r0.w);
    } else {
        p = a.pos[x + a.o_off];
        v = a.vel[x + a.o_off];
        id = a.id[x + a.o_off];
    }
}

// first position in sorted a[0, n) with a[pos] >= v
template <typename T>
static __device__ __forceinline__ uint32_t lower_bound(const T* __restrict__ a, uint32_t n, T v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// lower_bound by one wave: 64 probes per level, so a few dependent loads for any n (wave-uniform).
template <typename T>
static __device__ uint32_t wave_lower_bound(const T* __restrict__ a, uint32_t n, T v) {
    const uint32_t lane = lane_id();
    uint32_t base = 0, len = n;
    while (len > 64) {
        const uint32_t step = (len + 63) / 64;
        const uint32_t idx = base + lane * step;
        const bool lt = idx < base + len && a[idx] < v;
        const uint32_t k = (uint32_t)__popcll(__ballot(lt));   // probes below v form a prefix
        if (k == 0) return base;
        const uint32_t nb = base + (k - 1) * step + 1;
        const uint32_t end = k * step < len ? base + k * step : base + len;   // a[end] >= v (or end of range)
        base = nb;
        len = end - nb;
    }
    const bool lt = lane < len && a[base + lane] < v;
    return base + (uint32_t)__popcll(__ballot(lt));
}

// A(i) for the calling lane: movers with index < i (block offset + earlier waves + earlier lanes)
static __device__ __forceinline__ uint32_t movers_before(bool mv, uint32_t block_off, uint32_t* wc) {
    const uint64_t b = __ballot(mv);
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) wc[w] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t off = block_off;
    for (int k = 0; k < w; ++k) off += wc[k];
    return off + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}

// #entries below v in a sorted 64-entry LDS array (branchless; pads sort last and are never below v)
template <typename T>
static __device__ __forceinline__ uint32_t lb64(const T* __restrict__ a, T v) {
    uint32_t p = 0;
#pragma unroll
    for (uint32_t s = 32; s > 0; s >>= 1) p += a[p + s - 1] < v ? s : 0u;
    return p + (a[p] < v ? 1u : 0u);
}

// Per mover x (append order): rank[x] = #{y : (k_y, i_y) < (k_x, i_x)}, rank[cap + x] =
// #{y : i_y < i_x}, rank[2cap + x] = A(q_x) = #{y : i_y < q_x}. Work items = (MV_BLK movers) x
// (MV_TILE-mover tile); partial counts are added atomically (integers: order-independent).
// The tile is sorted twice in LDS (by (key, index) and by index: each entry's rank among the 64, counted a
// quarter per wave), and each mover counts by three 7-probe binary searches instead of 3 x 64 compares
// (~6.5 VALU per mover pair before, O(m^2) in the movers).
// Also zeroes the next step's mover counter.
// k_mv_rank's tile logic: lb64 searches exactly 64 entries, the tile is filled by threads < MV_TILE and
// counted by MV_BLK / MV_TILE parts
static_assert(MV_TILE == 64 && MV_BLK >= MV_TILE && MV_BLK % MV_TILE == 0, "k_mv_rank assumes 64-entry tiles");
__global__ __launch_bounds__(MV_BLK) void k_mv_rank(const uint32_t* __restrict__ mtotal,
                                                    uint32_t* __restrict__ next_count,
                                                    const uint32_t* __restrict__ cs_old, ResortScratch w) {
    constexpr int NPART = MV_BLK / MV_TILE;                  // waves counting one quarter of the tile each
    __shared__ uint64_t tile[MV_TILE];                       // (key, index) in append order; pads ~0
    __shared__ uint64_t sc[MV_TILE];                         // sorted by (key, index)
    __shared__ uint32_t si[MV_TILE];                         // indices, sorted
    __shared__ uint32_t part_c[NPART][MV_TILE], part_i[NPART][MV_TILE];
    if (w.dz) w.mi_off = (int32_t)w.dz->nl - (int32_t)w.dz->o0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *next_count = 0u;
    const uint32_t m = *mtotal;
    const uint64_t nr = (m + MV_BLK - 1) / MV_BLK, nt = (m + MV_TILE - 1) / MV_TILE;
    const int e = threadIdx.x % MV_TILE, part = threadIdx.x / MV_TILE;
    for (uint64_t item = blockIdx.x; item < nr * nt; item += gridDim.x) {
        const uint32_t ir = (uint32_t)(item % nr), it = (uint32_t)(item / nr);
        __syncthreads();
        if (threadIdx.x < MV_TILE) {
            const uint32_t y = it * MV_TILE + threadIdx.x;
            tile[threadIdx.x] = y < m ? comp(w.mk[y], mv_slot(w, w.mi[y])) : ~0ull;
        }
        __syncthreads();
        {   // entry e's rank among the tile, over this wave's quarter (ties, i.e. pads, by position)
            const uint64_t c = tile[e];
            const uint32_t i = (uint32_t)c;
            uint32_t rc = 0, ri = 0;
#pragma unroll 4
            for (int u = part * (MV_TILE / NPART); u < (part + 1) * (MV_TILE / NPART); ++u) {
                const uint64_t cu = tile[u];
                const uint32_t iu = (uint32_t)cu;
                rc += (cu < c || (cu == c && u < e)) ? 1u : 0u;
                ri += (iu < i || (iu == i && u < e)) ? 1u : 0u;
            }
            part_c[part][e] = rc;
            part_i[part][e] = ri;
        }
        __syncthreads();
        if (threadIdx.x < MV_TILE) {
            uint32_t rc = 0, ri = 0;
#pragma unroll
            for (int k = 0; k < NPART; ++k) {
                rc += part_c[k][threadIdx.x];
                ri += part_i[k][threadIdx.x];
            }
            const uint64_t c = tile[threadIdx.x];
            sc[rc] = c;
            si[ri] = (uint32_t)c;
        }
        __syncthreads();
        const uint32_t x = ir * MV_BLK + threadIdx.x;
        if (x < m) {
            const uint32_t ix = mv_slot(w, w.mi[x]), k = w.mk[x];
            const uint64_t cx = comp(k, ix);
            const uint32_t c0 = cs_old[k], c1 = cs_old[k + 1];
            const uint32_t q = ix < c0 ? c0 : (ix > c1 ? c1 : ix);
            const uint32_t nk = lb64(sc, cx), ni = lb64(si, ix), nq = lb64(si, q);
            if (nk) atomicAdd(&w.rank[x], nk);
            if (ni) atomicAdd(&w.rank[w.cap + x], ni);
            if (nq) atomicAdd(&w.rank[2 * w.cap + x], nq);
        }
    }
}

__global__ __launch_bounds__(MV_BLK) void k_mv_place(const uint32_t* __restrict__ mtotal,
                                                     const uint32_t* __restrict__ cs_old, ResortScratch w, AsmSrc src,
                                                     float4* __restrict__ pos_o, float4* __restrict__ vel_o,
                                                     int32_t* __restrict__ id_o, uint32_t* __restrict__ sk_o,
                                                     ResortExtra ex) {
    int32_t n_unused = 0;
    resolve_sizes(src, w, n_unused);
    const uint32_t m = *mtotal;
    for (uint32_t r = blockIdx.x * MV_BLK + threadIdx.x; r < m; r += gridDim.x * MV_BLK) {
        const uint32_t x = mv_slot(w, w.mi[r]), k = w.mk[r];
        const uint32_t c0 = cs_old[k], c1 = cs_old[k + 1];
        const uint32_t q = x < c0 ? c0 : (x > c1 ? c1 : x);
        const uint32_t rk = w.rank[r], ri = w.rank[w.cap + r], aq = w.rank[2 * w.cap + r];
        const uint32_t dst = (q - aq) + rk;
        if (dst >= w.cap || rk >= w.cap || ri >= w.cap) {   // inconsistent tables: flag, never write past them
            if (w.err) atomicOr(w.err, SZ_OVF_MOVERS);
            continue;
        }
        float4 p, v;
        int32_t pid;
        asm_load(src, (int32_t)x, p, v, pid);
        pos_o[dst] = p;
        vel_o[dst] = v;
        id_o[dst] = pid;
        sk_o[dst] = k;
        move_extra(ex, x, dst);
        w.ms[rk] = comp(k, x);
        w.mx[ri] = x;
        w.mos[ri] = w.mo[r];   // old keys by slot: ascending
    }
}

// cs[k] += #{movers: new key < k} − #{movers: old key < k}, for k in [0, ncells]; 1024 cells per
// workgroup. A workgroup whose counts agree at its start and that holds no mover key leaves its cells.
// Runs as extra workgroups of k_mv_merge (it needs only k_mv_place's tables), beside the scatter.
constexpr int MV_CS_CELLS = 4 * MV_BLK;
#ifndef SPH_MERGE_PREFETCH
#define SPH_MERGE_PREFETCH 1
#endif
// movers staged in LDS for the merge's binary searches (a workgroup's cells or slots rarely hold more)
constexpr uint32_t MV_LDS = 1024;

// Picks falling in this workgroup's cells are read back once its cells are final.
static __device__ void mv_cell_start(uint32_t* __restrict__ cs, uint32_t ncells, uint32_t m, const ResortScratch& w,
                                     uint32_t blk, uint32_t* b, const CsPick& pick, uint64_t* lms, uint32_t* lmo) {
    const uint32_t k0 = blk * MV_CS_CELLS, k1 = k0 + MV_CS_CELLS;
    const int wv = threadIdx.x >> 6;
    const uint32_t p = wv < 2 ? wave_lower_bound(w.ms, m, comp(wv == 0 ? k0 : k1, 0u))
                              : wave_lower_bound(w.mos, m, wv == 2 ? k0 : k1);
    if (lane_id() == 0) b[wv] = p;
    __syncthreads();
    const uint32_t nlo = b[0], nhi = b[1], olo = b[2], ohi = b[3];
    if (!(nlo == olo && nhi == nlo && ohi == olo)) {
        // the movers' new and old keys in this workgroup's cell range, staged in LDS (block-uniform test)
        const uint32_t nn = nhi - nlo, no = ohi - olo;
        const bool staged = nn <= MV_LDS && no <= MV_LDS;
        if (staged) {
            for (uint32_t t = threadIdx.x; t < nn; t += MV_BLK) lms[t] = w.ms[nlo + t];
            for (uint32_t t = threadIdx.x; t < no; t += MV_BLK) lmo[t] = w.mos[olo + t];
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t k = k0 + j * MV_BLK + threadIdx.x;
            if (k > ncells) break;
            const uint32_t cn = nlo + (staged ? lower_bound(lms, nn, comp(k, 0u)) : lower_bound(w.ms + nlo, nn, comp(k, 0u)));
            const uint32_t co = olo + (staged ? lower_bound(lmo, no, k) : lower_bound(w.mos + olo, no, k));
            cs[k] += cn - co;
        }
    }
    if (pick.m == 0) return;
    __syncthreads();   // this workgroup's cell updates are visible to all its lanes
    const int t = threadIdx.x;
    if (t < pick.m) {
        const uint32_t k = (uint32_t)pick.idx[t];
        if (k >= k0 && k < k1 && k <= ncells) {
            const uint32_t v = cs[k];
            pick.out[t] = v;
            if (pick.out_host) pick.out_host[t] = v;
        }
    }
}

__global__ __launch_bounds__(MV_BLK) void k_mv_merge(AsmSrc src, int32_t n,
                                                     const uint32_t* __restrict__ mtotal, ResortScratch w,
                                                     float4* __restrict__ pos_o,
                                                     float4* __restrict__ vel_o, int32_t* __restrict__ id_o,
                                                     uint32_t* __restrict__ sk_o, int32_t nb, uint32_t* __restrict__ cs,
                                                     uint32_t ncells, CsPick pick, ResortExtra ex) {
    __shared__ uint32_t wc[MV_BLK / 64];
    __shared__ uint32_t b[4];
    __shared__ uint64_t lms[MV_LDS];
    __shared__ uint32_t lmo[MV_LDS];
    if ((int32_t)blockIdx.x >= nb) {   // the cell-start workgroups
        mv_cell_start(cs, ncells, *mtotal, w, blockIdx.x - nb, b, pick, lms, lmo);
        return;
    }
    resolve_sizes(src, w, n);          // device-sized slab step: nb is an upper bound
    const int32_t i0 = xcd_block(blockIdx.x, nb) * MV_BLK;
    if (i0 >= n) return;               // whole workgroup, before any barrier
    const int32_t i = i0 + threadIdx.x;
    const int32_t ilast = min(i0 + MV_BLK, n) - 1;
    const uint32_t m = *mtotal;
    const int wv = threadIdx.x >> 6;
    // movers below this block's first slot, and the movers whose (key, index) falls inside its
    // stayers' range: ms[b1, b2)
    if (wv == 0) {
        const uint32_t p = wave_lower_bound(w.mx, m, (uint32_t)i0);
        if (lane_id() == 0) b[0] = p;
    } else if (wv < 3) {
        const uint64_t v = wv == 1 ? comp(asm_sk(src, i0), (uint32_t)i0) : comp(asm_sk(src, ilast), (uint32_t)ilast) + 1;
        const uint32_t p = wave_lower_bound(w.ms, m, v);
        if (lane_id() == 0) b[wv] = p;
    }
    const uint32_t ko = i < n ? asm_sk(src, i) : 0u;
    const bool stay = i < n && asm_key(src, i) == ko;
#if SPH_MERGE_PREFETCH
    // the slot's particle loads issue before the searches' dependent loads and the barrier (a mover's are unused)
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f), v = p;
    int32_t pid = 0;
    if (i < n) asm_load(src, i, p, v, pid);
#endif
    __syncthreads();
    const uint32_t a = movers_before(i < n && !stay, b[0], wc);
    const uint32_t lo = b[1], hi = b[2];
    const bool staged = hi - lo <= MV_LDS;   // block-uniform
    if (staged) {
        for (uint32_t t = threadIdx.x; t < hi - lo; t += MV_BLK) lms[t] = w.ms[lo + t];
        __syncthreads();
    }
    if (!stay) return;
    const uint64_t kv = comp(ko, (uint32_t)i);
    const uint32_t below = lo + (staged ? lower_bound(lms, hi - lo, kv) : lower_bound(w.ms + lo, hi - lo, kv));
    const uint32_t dst = ((uint32_t)i - a) + below;
    if (dst >= w.cap) {
        if (w.err) atomicOr(w.err, SZ_OVF_MOVERS);
        return;
    }
#if !SPH_MERGE_PREFETCH
    float4 p, v;
    int32_t pid;
    asm_load(src, i, p, v, pid);
#endif
    pos_o[dst] = p;
    vel_o[dst] = v;
    id_o[dst] = pid;
    sk_o[dst] = ko;
    move_extra(ex, (uint32_t)i, dst);
}

// The slab step's halo records: new keys (window sentinel, as k_keys) and old keys moved into this
// window, clamped into [0, ncells - 1]. The left neighbour's columns lie below this window's owned
// ones and the right neighbour's above, so clamping keeps the assembled old keys sorted. A record
// without an old key takes its side's bound (it then almost surely moves). Changed records join the
// movers the force pass appended for the own slots (mi = slot | MV_REC). A workgroup takes MV_DET
// records and reserves its entries with one atomic.
constexpr int MV_DET_PER = 4;
constexpr int MV_DET = MV_BLK * MV_DET_PER;
constexpr uint32_t REC_NO_KEY = 0xffffffffu;   // slab.hip SL_NO_KEY

// A record's old key moved into this window and clamped into [0, ncells - 1] (the clamp in 64-bit: the u32 form
// `og < base ? 0 : min(og - base, ncells - 1)` compiled to a plain subtract + min on ROCm 7.2, so keys below the
// window wrapped); a record without an old key takes its side's bound.
__device__ __forceinline__ uint32_t rec_old_key(uint32_t og, bool left, uint32_t key_base, uint32_t ncells) {
    if (og == REC_NO_KEY) return left ? 0u : ncells - 1u;
    const int64_t d = (int64_t)og - (int64_t)key_base;
    return (uint32_t)(d < 0 ? 0 : (d > (int64_t)ncells - 1 ? (int64_t)ncells - 1 : d));
}

// Workgroups [nb_rec, nb_rec + cs_old_blocks) build the old cell-start table (common.h cs_old_block) in the same
// launch, from the messages' old keys: no launch between the records and the re-sort (profiles/r04_slab_trace.log).
__global__ __launch_bounds__(MV_BLK) void k_slab_rec(AsmSrc src, int32_t n, GridDesc g, uint32_t key_base,
                                                     uint32_t* __restrict__ keyr, uint32_t* __restrict__ skr,
                                                     MoverSink sink, SizesIn in, int32_t from_headers, CsOld csp,
                                                     int32_t nb_rec) {
    __shared__ uint32_t wsum[MV_BLK / 64];
    __shared__ uint32_t base_s;
    __shared__ uint32_t samp[CS_SAMP];
    __shared__ uint32_t win[CS_WIN];
    if (from_headers) {   // device-sized slab step: every workgroup derives the layout from the headers,
        uint32_t nl, no, nr, f, hl, hr;   // the first stores it for the kernels after this one
        slab_sizes_from(src.dz, in, nl, no, nr, f, hl, hr);
        if (blockIdx.x == 0 && threadIdx.x == 0)
            slab_sizes_store(const_cast<SlabSizes*>(src.dz), nl, no, nr, f, hl, hr);
        if (csp.cs && (int32_t)blockIdx.x >= nb_rec) {   // the old cell-start table
            const float4* rl = src.rl;
            const float4* rr = src.rr;
            const uint32_t ncells = g.ncells;
            auto key = [&](int side, uint32_t t) {
                const float4* rec = side == 0 ? rl : rr;
                return rec_old_key(__float_as_uint(rec[2 * (size_t)t + 1].w), side == 0, key_base, ncells);
            };
            cs_old_block(csp, blockIdx.x - (uint32_t)nb_rec, nl, no, nr, (int32_t)nl - (int32_t)src.dz->o0, key, samp, win);
            return;
        }
        src.nl = (int32_t)nl;
        src.nre = (int32_t)(nl + no);
        n = (int32_t)(nl + no + nr);
    } else if (src.dz) {   // sizes already on the device; the launch covers the message capacities
        src.nl = (int32_t)src.dz->nl;
        src.nre = (int32_t)(src.dz->nl + src.dz->no);
        n = (int32_t)src.dz->n;
    }
    const int32_t nr = n - src.nre, nrec = src.nl + nr;
    if ((int32_t)(blockIdx.x * MV_DET) >= nrec) return;   // whole workgroup, before any barrier
    const int32_t r0 = blockIdx.x * MV_DET + threadIdx.x;
    uint32_t kn[MV_DET_PER], ko[MV_DET_PER];
    int32_t xs[MV_DET_PER];
    float4 pv[MV_DET_PER];
    uint32_t og[MV_DET_PER];
#pragma unroll
    for (int j = 0; j < MV_DET_PER; ++j) {   // loads first, unconditional
        const int32_t r = min(r0 + j * MV_BLK, nrec - 1);
        const float4* rec = r < src.nl ? src.rl + 2 * (size_t)r : src.rr + 2 * (size_t)(r - src.nl);
        pv[j] = rec[0];
        og[j] = __float_as_uint(rec[1].w);
        xs[j] = r < src.nl ? r : src.nre + (r - src.nl);
    }
    uint32_t mine = 0;   // bit j: record r0 + j * MV_BLK moved
#pragma unroll
    for (int j = 0; j < MV_DET_PER; ++j) {
        const bool left = xs[j] < src.nl;
        kn[j] = window_key(g, pv[j].x, pv[j].y, pv[j].z);
        ko[j] = rec_old_key(og[j], left, key_base, g.ncells);
        if (r0 + j * MV_BLK < nrec) {
            keyr[xs[j]] = kn[j];
            skr[xs[j]] = ko[j];
            if (kn[j] != ko[j]) mine |= 1u << j;
        }
    }
    const uint32_t c = (uint32_t)__popc(mine);
    // exclusive prefix of c over the workgroup
    uint32_t incl = c;
    const uint32_t lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)incl, o, 64);
        if (lane >= (uint32_t)o) incl += t;
    }
    const int wv = threadIdx.x >> 6;
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < MV_BLK / 64; ++k) {
        off += k < wv ? wsum[k] : 0u;
        tot += wsum[k];
    }
    if (threadIdx.x == 0) base_s = tot ? atomicAdd(sink.count, tot) : 0u;
    __syncthreads();
    uint32_t q = base_s + off + incl - c;
#pragma unroll
    for (int j = 0; j < MV_DET_PER; ++j) {
        if (!(mine >> j & 1u)) continue;
        if (q >= sink.cap) {
            if (sink.err) atomicOr(sink.err, SZ_OVF_MOVERS);
            break;
        }
        sink.mi[q] = (uint32_t)xs[j] | MV_REC;
        sink.mk[q] = kn[j];
        sink.mo[q] = ko[j];
        sink.rank[q] = 0u;
        sink.rank[sink.cap + q] = 0u;
        sink.rank[2 * sink.cap + q] = 0u;
        ++q;
    }
}

void launch_slab_rec(AsmSrc src, int32_t n, GridDesc g, uint32_t key_base, uint32_t* keyr, uint32_t* skr,
                     MoverSink sink, hipStream_t s, const SizesIn* sizes, CsOld cs) {
    const int32_t nrec = src.nl + (n - src.nre);
    const int32_t nb_rec = (nrec + MV_DET - 1) / MV_DET;
    const int32_t nb_cs = cs.cs && sizes ? cs_old_blocks(g.ncells, MV_BLK) : 0;   // the fused table: device-sized steps
    if (nb_rec + nb_cs > 0)
        k_slab_rec<<<nb_rec + nb_cs, MV_BLK, 0, s>>>(src, n, g, key_base, keyr, skr, sink, sizes ? *sizes : SizesIn{},
                                                     sizes ? 1 : 0, nb_cs ? cs : CsOld{}, nb_rec);
}

void launch_resort(AsmSrc src, uint32_t* cs, uint32_t ncells, int32_t n, const uint32_t* count,
                   uint32_t* count_other, ResortScratch w, float4* pos_o, float4* vel_o, int32_t* id_o,
                   uint32_t* sk_o, hipStream_t s, CsPick pick, ResortExtra ex) {
    if (n <= 0) return;
    const int32_t nb = (n + MV_BLK - 1) / MV_BLK;
    SPH_LAUNCH(k_mv_rank, MV_RANK_GRID, MV_BLK, 0, s, count, count_other, cs, w);
    SPH_LAUNCH(k_mv_place, std::min(nb, 1024), MV_BLK, 0, s, count, cs, w, src, pos_o, vel_o, id_o, sk_o, ex);
    // + the cell-start update, after every reader of cs_old (k_mv_rank, k_mv_place)
    const int32_t ncs = (int32_t)((ncells + MV_CS_CELLS) / MV_CS_CELLS);
    SPH_LAUNCH(k_mv_merge, nb + ncs, MV_BLK, 0, s, src, n, count, w, pos_o, vel_o, id_o, sk_o, nb, cs, ncells, pick, ex);
}

}  // namespace sph
