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
// One launch (k_mv_rank): workgroup b takes a range of old slots and the new keys they hold, and an equal share of the
// cells. Per range: the movers' ranks, insertion slots and placement, and the stayers' scatter of (pos, vel, id, key);
// per share of cells: the new cell-start table, cs_new[k] = cs[k] + #{movers: new key < k} − #{movers: old key < k},
// with the mover keys in the share staged from the same stream over the mover list. The scatters replace the
// permutation gather, and the table update the cell-start rebuild, of the full path.
#include "common.h"

namespace sph {

constexpr int MV_BLK = 256;

static __device__ __forceinline__ uint64_t comp(uint32_t key, uint32_t idx) { return (uint64_t)key << 32 | idx; }

// a workgroup-uniform value (LDS / block reductions / same-address loads) into a scalar register: the rank kernel runs
// at 64 VGPRs (two 1,024-lane workgroups per CU), and its range bounds and counts are live across every loop
static __device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

static __device__ __forceinline__ bool asm_rec(const AsmSrc& a, int32_t x) { return x < a.nl || x >= a.nre; }

// Model R's other slot arrays (single domain: slot x is x)
static __device__ __forceinline__ void move_extra(const ResortExtra& ex, uint32_t x, uint32_t dst) {
    if (!ex.omg) return;
    ex.omg_o[dst] = ex.omg[x];
    ex.rot_o[dst] = ex.rot[x];
    ex.aux_o[dst] = ex.aux[x];
    ex.mode_o[dst] = ex.mode[x];
}
struct ExtraVals { float4 omg, rot, aux; int32_t mode; };
static __device__ __forceinline__ ExtraVals load_extra(const ResortExtra& ex, uint32_t x) {
    ExtraVals e{};
    if (ex.omg) e = ExtraVals{ex.omg[x], ex.rot[x], ex.aux[x], ex.mode[x]};
    return e;
}
static __device__ __forceinline__ void store_extra(const ResortExtra& ex, const ExtraVals& e, uint32_t dst) {
    if (!ex.omg) return;
    ex.omg_o[dst] = e.omg;
    ex.rot_o[dst] = e.rot;
    ex.aux_o[dst] = e.aux;
    ex.mode_o[dst] = e.mode;
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

// Mover ranks and placement in O(m) per workgroup (replaces the all-pairs tile counts and the separate placement of
// r1-r4, whose work grew as m²: the C3 re-sort chain went from 27.7 us from rest to 41.5 us mid-collapse). Workgroup
// b of G owns the slots [x0, x1) = [b·n/G, (b+1)·n/G) of the assembled old order and the new keys
// [kd0, kd1) = [sk(x0), sk(x1)) (the old sorted keys at those slots, so every workgroup's key range holds about n/G
// particles and ~m/G movers; the ranges partition all keys, sentinels included). Its dest entries are the movers
// with a new key in its range, its source entries those with a slot in its range. One stream over the whole mover
// list (U per lane in flight) stages both in LDS and counts the movers below the ranges; then
//   rk(x) = #{y : k_y < kd0} + #{dest entries (k', y) < (k, x)}               -> ms[rk] = (k, x)
//   ri(x) = #{y : y < x}                                                      -> mx[ri] = x, mos[ri] = old key
// and for its dest entries the insertion slot q = clamp(x, cs_old[k], cs_old[k + 1]) and A(q) = #{y : y < q}. Every
// such q lies in [cs_old[kd0], x1], and cs_old[kd0] (the start of the cell holding slot x0) lies within RK_WIN below
// x0 but in cells of more than RK_WIN particles, so the stream also stages the movers with a slot in
// [xw, x1) = [x0 − RK_WIN, x1) into a presence bitmap and counts those below x0: a slot rank or A(q) is that count
// plus (or minus) the staged slots between x0 and the slot, read from the bitmap's word prefix (the slots are
// distinct, so they need no sort), with no second pass over the mover list (r5: a second stream's dependent loads
// took the kernel from ~5 to ~32 us). The dest entries are ranked by counting (LDS broadcast reads) up to RK_COUNT of
// them, by sorting beyond. The mover is placed at dst = (q − A(q)) + rk, every stayer of the slot range at
// (i − A(i)) + #{movers (k, y) < (k_i, i)} (k_i in [kd0, kd1]; at kd1 the kd1 movers staged apart), and the share of
// cells written from its staged keys.
//
// A range's key interval [kd0, kd1) can span empty cells: the last range's reaches past the fluid's last column, so
// every particle a dam-break front carries into an empty column is one of its dest entries (C5 from step ~60: more
// than MV_RK_CAP per step). Such a range runs in passes over key sub-intervals (multi-pass): a second stream over the
// mover list copies its nd dest entries to ms[below_k, below_k + nd) (the ranges' key intervals are disjoint and
// ordered, so these spans are too) and bins them by key in an LDS histogram; sub-interval p is the bins whose
// exclusive prefix lies in [p·C, (p+1)·C), C = MP_CAP − (largest bin), so each holds < MP_CAP entries. Per pass the
// sub-interval's entries are staged from the copy (nd/1024 loads per lane), sorted, placed with rank
// below_k + (entries of earlier passes) + local rank, and the stayers whose old key lies in it scattered. r5 counted
// such a range's entries against the whole mover list instead, O(slots · m): 7.75 against 4.19 ms per C5 step from
// step ~60 on. The whole-list counts remain only for states no bin layout fits (one bin of more than
// MP_CAP / 2 movers, more than RK_KD1_CAP movers into one cell, insertion slots below the staged window) and are
// counted (ResortScratch.stats, sph_read_resort_counts). Also zeroes the next step's mover counter. Per workgroup the
// kernel is a chain of memory round trips (~1.5 us each; the probe build, scripts/rank_probe.py): one before the
// stream (count, range keys and the first movers together), one for the entries' and stayers' loads, one for the
// cells.
constexpr int MV_RANK_GRID = 256;   // workgroups at least (one per CU); more above 2M slots
constexpr int RK_U = 8;             // movers per lane per streaming round
// Test-only variant (csrc/Makefile `variants`, SPH_RK_SMALLCAP): LDS caps cut so that small scenes take the
// multi-pass path; results must equal the product build's bit for bit (tests/test_gpu_path_independence.py).
#ifdef SPH_RK_SMALLCAP
constexpr int MV_RK_CAP = 32;   // (MP_CAP >= 64: lds_sort pads to 64 entries)
#else
constexpr int MV_RK_CAP = 2048;     // dest entries staged per workgroup (a power of two)
#endif
constexpr int MP_CAP = 2 * MV_RK_CAP;   // multi-pass: entries per pass (dk and ds as one array)
#ifdef SPH_RK_RANGE8K   // A/B: r5's 8,192-slot ranges
constexpr int RK_HBITS = 12;
constexpr int RK_BM_WORDS = 1024;
#else
constexpr int RK_HBITS = 11;
constexpr int RK_BM_WORDS = 2048;   // slot-presence bitmap over [xw, x1): up to 65,536 slots
#endif
constexpr int RK_HBINS = 1 << RK_HBITS; // multi-pass: key bins of a range
constexpr int RK_WIN = 2048;        // slot entries staged below x0 (covers the cell holding x0)
// Slots per range at most: the grid grows past MV_RANK_GRID workgroups for n > 8M (C5 single-context: 512 ranges).
// Every workgroup streams the whole mover list, so the grid costs ~(ranges + shares)·m of L2 reads: r5's 8,192-slot
// ranges and 16,384-cell shares made 5,627 workgroups at C5 (4.5 GB of mover reads per step, k_mv_rank 0.55 ms);
// a range's dest entries beyond LDS now take the multi-pass path, so ranges can be 4x longer.
#ifdef SPH_RK_RANGE8K
constexpr uint32_t RK_MAX_RANGE = 8192;
#else
constexpr uint32_t RK_MAX_RANGE = 32768;
#endif
static_assert(RK_MAX_RANGE + RK_WIN + 512u <= 32u * RK_BM_WORDS, "a range and its window fit the bitmap");
#ifdef SPH_RK_SMALLCAP
constexpr int RK_COUNT = 8;
#else
constexpr int RK_COUNT = 256;       // dest entries ranked by counting, more by sorting
#endif
constexpr int RK_KD1_CAP = 1024;    // movers into the cell a range ends in, staged
constexpr int RK_SU = 2;            // stayer slots per lane in flight
#ifdef SPH_RK_SMALLCAP   // (the variant: shares of several passes whose keys overflow LDS; no direct shares)
constexpr uint32_t RK_SUB = 1024;
constexpr uint32_t RK_SHARE_KEYS = 48;
constexpr uint32_t RK_DIRECT = 0;
#else
constexpr uint32_t RK_SUB = 8192;    // cells per LDS pass of a share (its difference array)
constexpr uint32_t RK_SHARE_KEYS = 16384;  // a share's mover keys staged in LDS, 16 bits each (beyond: a stream per pass)
constexpr uint32_t RK_DIRECT = 16384;      // a share of at most this many cells: one pass, the stream adding into LDS
#endif
constexpr uint32_t RK_SUBS = 8;      // passes per share at most
constexpr uint32_t RK_CELLS = RK_SUB * RK_SUBS;   // cells per share at most (k_mv_rank's cell workgroups)
constexpr int RK_POOL_U64 = 8192;   // the LDS pool (64 KB): a share's differences and keys, or a range's entries and bitmap
static_assert(4 * RK_SUB + 2 * RK_SHARE_KEYS <= 8 * RK_POOL_U64 && RK_SUB * RK_SUBS <= 65536u &&
              4 * RK_DIRECT <= 8 * RK_POOL_U64 && RK_DIRECT <= 16u * 1024u,
              "a share's LDS fits the pool; its cell offsets fit 16 bits; a direct share's prefix fits 16 cells per lane");
constexpr int RK_CU = 4;            // cells per lane in flight
constexpr int RK_CNT_U = 4;         // dest entries per counting round in flight (LDS reads)
static_assert(2 * MV_RK_CAP * 8 + 4 * (RK_KD1_CAP + 2 * (RK_BM_WORDS + 1) + RK_HBINS + 1) <= RK_POOL_U64 * 8,
              "a range's LDS fits the pool");
// ResortScratch.stats words (sph_read_resort_counts): ranges that counted against the whole mover list, lanes whose
// insertion slot lay below the staged window (a whole-list count each), multi-pass ranges, their passes, the largest
// dest-entry count of a range (recorded above MV_RK_CAP / 4), cell shares whose mover keys overflowed LDS (a stream
// of the mover list per pass instead of one)
enum { RS_WHOLE = 0, RS_WHOLE_LANES, RS_MULTI, RS_PASSES, RS_MAX_ND, RS_SHARE_RESTREAM, RS_WORDS = 8 };
// Test-only timing probe (scripts/rank_probe.py, a -DSPH_RANK_PROBE build): per workgroup the wall clock at its start,
// after the mover stream, after the sorts and at its end, with its entry counts.
#ifdef SPH_RANK_PROBE
__device__ uint64_t g_rank_probe[MV_RANK_GRID * 8];
#define RK_PROBE(slot, val)                                                                            \
    do {                                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < MV_RANK_GRID) g_rank_probe[blockIdx.x * 8 + (slot)] = (uint64_t)(val); \
    } while (0)
#else
#define RK_PROBE(slot, val) \
    do {                    \
    } while (0)
#endif

template <int BLK>
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    __syncthreads();
    if (lane_id() == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < BLK / 64; ++k) t += red[k];
    return t;
}

static __device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int j) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, j, 64), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), j, 64);
    return (uint64_t)hi << 32 | lo;
}

// The rank kernel's workgroup: 16 waves, so a crowded range's sorts and entries spread over 1024 lanes.
constexpr int RK_BLK = 1024;

// Bitonic steps (k, j) for k = k0 .. k1 and j = min(k / 2, 32) .. 1, i.e. the ones whose partners lie in the same
// 64-entry block, in registers: each wave takes whole blocks and exchanges by shuffles.
__device__ void bitonic_regs(uint64_t* a, uint32_t* b, uint32_t P, uint32_t k0, uint32_t k1) {
    const uint32_t l = lane_id();
    for (uint32_t base = (threadIdx.x >> 6) * 64; base < P; base += RK_BLK) {
        const uint32_t i = base + l;
        uint64_t v = a[i];
        uint32_t pb = b ? b[i] : 0u;
        for (uint32_t k = k0; k <= k1; k <<= 1)
            for (uint32_t j = min(k >> 1, 32u); j > 0; j >>= 1) {
                const uint64_t o = shfl_xor64(v, (int)j);
                const uint32_t ob = (uint32_t)__shfl_xor((int)pb, (int)j, 64);
                // the pair's lower entry keeps the smaller key in an ascending run, the larger in a descending one
                const bool take = ((i & j) == 0) == ((i & k) == 0) ? o < v : o > v;
                if (take) {
                    v = o;
                    pb = ob;
                }
            }
        a[i] = v;
        if (b) b[i] = pb;
    }
}

// Sorts a[0, len) ascending in LDS, the payload b (if any) moved along; the keys are distinct; the arrays hold the
// next power of two >= max(len, 64) entries. Bitonic: the steps with partners 64 or more entries apart go through LDS
// (one pair per lane, a barrier each), all shorter ones in registers (bitonic_regs), so a sort of 2048 entries takes
// 26 barriers instead of 66 (a crowded range mid-collapse holds ~1,600 entries: r5 measured 20 us for the kernel with
// the plain LDS form at 256 lanes). Every thread of the workgroup calls it; it ends on a barrier.
__device__ void lds_sort(uint64_t* a, uint32_t* b, uint32_t len) {
    if (len <= 1) {
        __syncthreads();
        return;
    }
    uint32_t P = 64;
    while (P < len) P <<= 1;
    for (uint32_t t = len + threadIdx.x; t < P; t += RK_BLK) {
        a[t] = ~0ull;
        if (b) b[t] = 0u;
    }
    __syncthreads();
    bitonic_regs(a, b, P, 2, 64);
    __syncthreads();
    for (uint32_t k = 128; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j >= 64; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < P / 2; t += RK_BLK) {
                const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), u = i | j;   // pair t: i < u = i + j
                const uint64_t x = a[i], y = a[u];
                if ((x > y) == ((i & k) == 0)) {
                    a[i] = y;
                    a[u] = x;
                    if (b) {
                        const uint32_t bi = b[i];
                        b[i] = b[u];
                        b[u] = bi;
                    }
                }
            }
            __syncthreads();
        }
        bitonic_regs(a, b, P, k, k);
        __syncthreads();
    }
}

// A share of the cells [c0, c1) of [0, ncells] (workgroups G.. of k_mv_rank): cs_new[k] = cs[k] + #{movers: new key
// < k} − #{movers: old key < k}. One stream over the movers' keys counts those below c0 and stages the others that
// change a cell of the share (key k in [c0, c1 − 1): cell k + 1 on) in LDS, as j − 1 = k − c0 in 16 bits, new keys
// from the front of the list and old keys from its back. Then per pass of RK_SUB cells: the staged keys of the pass add
// ±1 at j into a difference array, whose prefix (plus the passes before) is each cell's change. A share holds up to RK_SUBS passes, so that at C5 (58.6M cells) 895 shares
// stream the mover list instead of r5's 3,578 16,384-cell ones; a share whose keys overflow LDS streams the list once
// per pass (counted). The old table is only read (every workgroup's movers read their insertion cells from it), the new
// one written whole; the cell starts read back (picks) come from here.
// A share of up to RK_DIRECT cells (C3: 256 shares of ~14,300) in one pass, r5's form: the stream adds +1 (new key) / −1
// (old key) at key + 1 straight into an LDS difference array over the whole share. Larger shares (C5: 895 of 65,536
// cells) take the staged form below (mv_cells_staged); two functions, so that the staged form's registers do not
// reach the direct form's code (a kernel with both measured the C3 re-sort 29 → 34 µs, profiles/r06_resort_ab.log).
__device__ void mv_cells_direct(uint32_t cb, uint32_t Gc, const uint32_t* __restrict__ mtotal, const uint32_t* __restrict__ cs,
                         uint32_t* __restrict__ cs_new, uint32_t ncells, const CsPick& pick, const ResortScratch& w,
                         int32_t* diff, uint32_t* red) {
    const uint32_t c0 = (uint32_t)((uint64_t)(ncells + 1u) * cb / Gc), c1 = (uint32_t)((uint64_t)(ncells + 1u) * (cb + 1) / Gc);
    const uint32_t L = c1 - c0;   // <= RK_DIRECT (the caller's choice)
    uint32_t ks[RK_U], os[RK_U];
    auto load_round = [&](uint32_t base, uint32_t last) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < RK_U; ++u) {
            const uint32_t r = min(base + u * RK_BLK + threadIdx.x, last);
            ks[u] = w.mk[r];
            os[u] = w.mo[r];
        }
    };
    load_round(0, w.cap - 1u);
    const uint32_t m = uni(ld_vec(mtotal));
    for (uint32_t t = threadIdx.x; t < L; t += RK_BLK) diff[t] = 0;
    __syncthreads();
    uint32_t bn_c = 0, bo_c = 0;
    for (uint32_t base = 0; base < m; base += RK_BLK * RK_U) {
#pragma unroll
        for (int u = 0; u < RK_U; ++u) {
            const uint32_t r = base + u * RK_BLK + threadIdx.x;
            const bool okr = r < m;
            const uint32_t k = ks[u], o = os[u];
            bn_c += okr && k < c0 ? 1u : 0u;
            bo_c += okr && o < c0 ? 1u : 0u;
            if (okr && k >= c0 && k + 1u < c1) atomicAdd(&diff[k + 1u - c0], 1);
            if (okr && o >= c0 && o + 1u < c1) atomicAdd(&diff[o + 1u - c0], -1);
        }
        if (base + RK_BLK * RK_U < m) load_round(base + RK_BLK * RK_U, m - 1u);
    }
    bn_c = block_sum<RK_BLK>(bn_c, red);   // (its barriers also publish the differences)
    bo_c = block_sum<RK_BLK>(bo_c, red);
    // inclusive prefix of diff[0, L): RK_DIRECT / RK_BLK consecutive entries per lane
    constexpr uint32_t EPL = RK_DIRECT >= (uint32_t)RK_BLK ? RK_DIRECT / RK_BLK : 1u;
    const uint32_t e0 = EPL * threadIdx.x;
    int32_t tot = 0;
#pragma unroll
    for (uint32_t j = 0; j < EPL; ++j) tot += e0 + j < L ? diff[e0 + j] : 0;
    int32_t inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t u = __shfl_up(inc, o, 64);
        if (lane_id() >= (uint32_t)o) inc += u;
    }
    __syncthreads();   // block_sum's last reads of red
    if (lane_id() == 63) red[threadIdx.x >> 6] = (uint32_t)inc;
    __syncthreads();
    int32_t pre = (int32_t)bn_c - (int32_t)bo_c + inc - tot;
    for (uint32_t k = 0; k < (threadIdx.x >> 6); ++k) pre += (int32_t)red[k];
#pragma unroll
    for (uint32_t j = 0; j < EPL; ++j)   // now the change of cell c0 + e0 + j (each lane rewrites only its own entries)
        if (e0 + j < L) {
            pre += diff[e0 + j];
            diff[e0 + j] = pre;
        }
    __syncthreads();
    for (uint32_t base = 0; base < L; base += RK_BLK * RK_CU) {
        uint32_t cv[RK_CU];
#pragma unroll
        for (int u = 0; u < RK_CU; ++u) cv[u] = cs[c0 + min(base + u * RK_BLK + threadIdx.x, L - 1u)];
#pragma unroll
        for (int u = 0; u < RK_CU; ++u) {
            const uint32_t t = base + u * RK_BLK + threadIdx.x;
            if (t < L) cs_new[c0 + t] = (uint32_t)((int32_t)cv[u] + diff[t]);
        }
    }
    if (c1 == ncells + 1u && threadIdx.x == 0) cs_new[ncells + 1u] = cs[ncells + 1u];
    if ((int32_t)threadIdx.x < pick.m) {   // cell starts read back: the ones in this share
        const uint32_t k = (uint32_t)pick.idx[threadIdx.x];
        if (k >= c0 && k < c1) {
            const uint32_t v = (uint32_t)((int32_t)cs[k] + diff[k - c0]);
            pick.out[threadIdx.x] = v;
            if (pick.out_host) pick.out_host[threadIdx.x] = v;
        }
    }
}


__device__ void mv_cells_staged(uint32_t cb, uint32_t Gc, const uint32_t* __restrict__ mtotal, const uint32_t* __restrict__ cs,
                         uint32_t* __restrict__ cs_new, uint32_t ncells, const CsPick& pick, const ResortScratch& w,
                         int32_t* diff, uint16_t* kl, uint32_t* cnt, uint32_t* red) {
    const uint32_t c0 = (uint32_t)((uint64_t)(ncells + 1u) * cb / Gc), c1 = (uint32_t)((uint64_t)(ncells + 1u) * (cb + 1) / Gc);
    const uint32_t L = c1 - c0;   // <= RK_CELLS (the launcher's share count)
    uint32_t ks[RK_U], os[RK_U];
    auto load_round = [&](uint32_t base, uint32_t last) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < RK_U; ++u) {
            const uint32_t r = min(base + u * RK_BLK + threadIdx.x, last);
            ks[u] = w.mk[r];
            os[u] = w.mo[r];
        }
    };
    load_round(0, w.cap - 1u);
    const uint32_t m = uni(ld_vec(mtotal));
    __syncthreads();   // cnt zeroed
    // cells [c0 + a, c0 + b) of the share changed by key k: k + 1 − c0 in [a, b)
    auto in_share = [&](uint32_t k, uint32_t a, uint32_t b) { return k >= c0 && k + 1u < c1 && k + 1u - c0 >= a && k + 1u - c0 < b; };
    uint32_t bn_c = 0, bo_c = 0;
    for (uint32_t base = 0; base < m; base += RK_BLK * RK_U) {
#pragma unroll
        for (int u = 0; u < RK_U; ++u) {
            const uint32_t r = base + u * RK_BLK + threadIdx.x;
            const bool okr = r < m;
            const uint32_t k = ks[u], o = os[u];
            bn_c += okr && k < c0 ? 1u : 0u;
            bo_c += okr && o < c0 ? 1u : 0u;
            if (okr && in_share(k, 0u, L)) {
                const uint32_t p = atomicAdd(&cnt[0], 1u);
                if (p < RK_SHARE_KEYS) kl[p] = (uint16_t)(k - c0);
            }
            if (okr && in_share(o, 0u, L)) {
                const uint32_t p = atomicAdd(&cnt[1], 1u);
                if (p < RK_SHARE_KEYS) kl[RK_SHARE_KEYS - 1u - p] = (uint16_t)(o - c0);
            }
        }
        if (base + RK_BLK * RK_U < m) load_round(base + RK_BLK * RK_U, m - 1u);
    }
    bn_c = uni(block_sum<RK_BLK>(bn_c, red));   // (its barriers also publish the staged keys)
    bo_c = uni(block_sum<RK_BLK>(bo_c, red));
    const uint32_t nn = uni(cnt[0]), no = uni(cnt[1]);
    const bool staged = nn + no <= RK_SHARE_KEYS;   // block-uniform
    if (!staged && threadIdx.x == 0 && w.stats) atomicAdd(w.stats + RS_SHARE_RESTREAM, 1u);
    int32_t carry = (int32_t)uni((uint32_t)((int32_t)bn_c - (int32_t)bo_c));   // the change below the pass's first cell
    for (uint32_t s0 = 0; s0 < L; s0 += RK_SUB) {
        const uint32_t Ls = min(RK_SUB, L - s0);
        {
            __syncthreads();   // the previous pass's reads of diff and red
            for (uint32_t t = threadIdx.x; t < RK_SUB; t += RK_BLK) diff[t] = 0;
            __syncthreads();
            if (staged) {
                for (uint32_t t = threadIdx.x; t < nn + no; t += RK_BLK) {
                    const bool nw = t < nn;
                    const uint32_t j = (uint32_t)kl[nw ? t : RK_SHARE_KEYS - 1u - (t - nn)] + 1u;
                    if (j >= s0 && j < s0 + Ls) atomicAdd(&diff[j - s0], nw ? 1 : -1);
                }
            } else {   // the keys did not fit: this pass's from the whole list (rare: a plain loop, few registers)
                for (uint32_t r = threadIdx.x; r < m; r += RK_BLK) {
                    const uint32_t k = w.mk[r], o = w.mo[r];
                    if (in_share(k, s0, s0 + Ls)) atomicAdd(&diff[k + 1u - c0 - s0], 1);
                    if (in_share(o, s0, s0 + Ls)) atomicAdd(&diff[o + 1u - c0 - s0], -1);
                }
            }
            __syncthreads();
        }
        // inclusive prefix of diff[0, Ls): EPL consecutive entries per lane, from carry
        constexpr uint32_t EPL = RK_SUB / RK_BLK;
        static_assert(EPL * RK_BLK == RK_SUB, "cells per lane");
        const uint32_t e0 = EPL * threadIdx.x;
        int32_t tot = 0;
#pragma unroll
        for (uint32_t j = 0; j < EPL; ++j) tot += e0 + j < Ls ? diff[e0 + j] : 0;
        int32_t inc = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t u = __shfl_up(inc, o, 64);
            if (lane_id() >= (uint32_t)o) inc += u;
        }
        if (lane_id() == 63) red[threadIdx.x >> 6] = (uint32_t)inc;
        __syncthreads();
        int32_t pre = carry + inc - tot, all = 0;
        for (uint32_t k = 0; k < RK_BLK / 64; ++k) {
            const int32_t rk = (int32_t)red[k];
            pre += k < (threadIdx.x >> 6) ? rk : 0;
            all += rk;
        }
#pragma unroll
        for (uint32_t j = 0; j < EPL; ++j)   // now the change of cell c0 + s0 + e0 + j (each lane rewrites its own entries)
            if (e0 + j < Ls) {
                pre += diff[e0 + j];
                diff[e0 + j] = pre;
            }
        carry = (int32_t)uni((uint32_t)(carry + all));
        __syncthreads();
        const uint32_t cb0 = c0 + s0;
        for (uint32_t base = 0; base < Ls; base += RK_BLK * RK_CU) {
            uint32_t cv[RK_CU];
#pragma unroll
            for (int u = 0; u < RK_CU; ++u) cv[u] = cs[cb0 + min(base + u * RK_BLK + threadIdx.x, Ls - 1u)];
#pragma unroll
            for (int u = 0; u < RK_CU; ++u) {
                const uint32_t t = base + u * RK_BLK + threadIdx.x;
                if (t < Ls) cs_new[cb0 + t] = (uint32_t)((int32_t)cv[u] + diff[t]);
            }
        }
        if ((int32_t)threadIdx.x < pick.m) {   // cell starts read back: the ones in this pass
            const uint32_t k = (uint32_t)pick.idx[threadIdx.x];
            if (k >= cb0 && k < cb0 + Ls) {
                const uint32_t v = (uint32_t)((int32_t)cs[k] + diff[k - cb0]);
                pick.out[threadIdx.x] = v;
                if (pick.out_host) pick.out_host[threadIdx.x] = v;
            }
        }
    }
    if (c1 == ncells + 1u && threadIdx.x == 0) cs_new[ncells + 1u] = cs[ncells + 1u];
}

// STAGED: the cell shares exceed RK_DIRECT cells (mv_cells_staged), else mv_cells_direct; one form per instantiation, so
// that the C3 kernel carries only the direct form's registers (60 VGPRs, nothing spilled; both forms in one kernel
// spilled 22)
template <bool STAGED>
__global__ __launch_bounds__(RK_BLK, 8) void k_mv_rank(const uint32_t* __restrict__ mtotal, uint32_t* __restrict__ next_count,
                                                    const uint32_t* __restrict__ cs, uint32_t* __restrict__ cs_new,
                                                    uint32_t ncells, CsPick pick, uint32_t G, ResortScratch w,
                                                    AsmSrc src, int32_t n,
                                                    float4* __restrict__ pos_o, float4* __restrict__ vel_o,
                                                    int32_t* __restrict__ id_o, uint32_t* __restrict__ sk_o,
                                                    ResortExtra ex) {
    // one LDS pool, laid out per role: a range's entries and slot bitmap, or a cell share's count differences
    __shared__ uint64_t pool[RK_POOL_U64];
    __shared__ uint32_t cnt[10], red[RK_BLK / 64];
    uint64_t* dk = pool;                                    // dest entries (new key, slot); multi-pass: MP_CAP of them
    uint64_t* ds = pool + MV_RK_CAP;                        // the dest entries in (key, slot) order
    uint32_t* kx1 = (uint32_t*)(pool + 2 * MV_RK_CAP);      // slots of the movers whose new key is kd1
    uint32_t* bm = kx1 + RK_KD1_CAP;                        // movers' slots in [xw, x1): bits
    uint32_t* bpre = bm + (RK_BM_WORDS + 1);                // and the words' prefix
    uint32_t* hp = bpre + (RK_BM_WORDS + 1);                // multi-pass: key bins, then their exclusive prefix
    RK_PROBE(0, wall_clock64());
    resolve_sizes(src, w, n);
    if (threadIdx.x < 10) cnt[threadIdx.x] = 0u;
    if (blockIdx.x >= G) {   // a share of the cells: its own workgroup, beside the ranges
        if constexpr (STAGED)
            mv_cells_staged(blockIdx.x - G, gridDim.x - G, mtotal, cs, cs_new, ncells, pick, w, (int32_t*)pool,
                            (uint16_t*)((int32_t*)pool + RK_SUB), cnt, red);
        else
            mv_cells_direct(blockIdx.x - G, gridDim.x - G, mtotal, cs, cs_new, ncells, pick, w, (int32_t*)pool, red);
        return;
    }
    const uint32_t b = blockIdx.x;
    // the ranges are whole blocks of 256 slots
    const uint32_t nbk = ((uint32_t)n + 255u) / 256u;
    const uint32_t x0 = min((uint32_t)((uint64_t)nbk * b / G) * 256u, (uint32_t)n);
    const uint32_t x1 = min((uint32_t)((uint64_t)nbk * (b + 1) / G) * 256u, (uint32_t)n);
    // Everything the stream needs in one round trip (the kernel is a chain of dependent round trips of ~1.5 us each,
    // r5 probe): the mover count, both range keys (pointer selects) and the first round of movers, whose loads are
    // clamped to the lists' capacity rather than to the count they would otherwise wait for.
    auto sk_ptr = [&](uint32_t x) {
        const int32_t xi = (int32_t)min(x, (uint32_t)max(n - 1, 0));
        return asm_rec(src, xi) ? src.skr + xi : src.sk + (xi + src.o_off);
    };
    uint32_t xs[RK_U], ks[RK_U];
    auto load_round = [&](uint32_t base, uint32_t last) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < RK_U; ++u) {   // every load of the round issues before any is used
            const uint32_t r = min(base + u * RK_BLK + threadIdx.x, last);
            xs[u] = w.mi[r];
            ks[u] = w.mk[r];
        }
    };
    load_round(0, w.cap - 1u);
    // the count and the range keys through the vector path behind the movers' loads (ld_vec), all in one round trip
    // (as scalar loads, the wait for the kernel arguments also waited for them before the movers' loads could issue)
    const uint32_t z = vzero();
    const uint32_t skv0 = sk_ptr(x0)[z], skv1 = sk_ptr(x1)[z], mv = mtotal[z];
    asm volatile("" ::"v"(skv0), "v"(skv1), "v"(mv));   // issued here, not sunk into the blocks that use them
    const uint32_t m = uni(mv), sk0 = uni(skv0), sk1 = uni(skv1);
    if (b == 0 && threadIdx.x == 0) {
        *next_count = 0u;
        if (w.host_count) *w.host_count = m;   // for the host's next sort choices (no copy launch)
    }
    const uint32_t kd0 = b == 0 ? 0u : (x0 < (uint32_t)n ? sk0 : 0xffffffffu);
    const uint32_t kd1 = b == G - 1 ? 0xffffffffu : (x1 < (uint32_t)n ? sk1 : 0xffffffffu);
    // Movers' slots are staged from xw = x0 − RK_WIN: every insertion slot q of a dest entry lies in
    // [cs_old[kd0], x1], and cs_old[kd0] (the start of the cell holding slot x0) is at most RK_WIN below x0 except
    // in cells of more than RK_WIN particles; such an entry counts its A(q) against the whole list instead.
    const uint32_t xw = x0 > (uint32_t)RK_WIN ? x0 - (uint32_t)RK_WIN : 0u;
    const bool bits_ok = x1 - xw <= 32u * RK_BM_WORDS;   // block-uniform
    // the bitmap's words over [xw, x1) only (C3: 192 of 2,048)
    const uint32_t nbw = min((x1 - xw + 31u) >> 5, (uint32_t)RK_BM_WORDS);
    for (uint32_t t = threadIdx.x; t <= nbw; t += RK_BLK) bm[t] = 0u;
    __syncthreads();
    uint32_t below_k = 0, below_x0 = 0;
    for (uint32_t base = 0; base < m; base += RK_BLK * RK_U) {
#pragma unroll
        for (int u = 0; u < RK_U; ++u) {
            const uint32_t r = base + u * RK_BLK + threadIdx.x;
            const bool okr = r < m;
            const uint32_t x = mv_slot(w, xs[u]), k = ks[u];
            below_k += okr && k < kd0 ? 1u : 0u;
            below_x0 += okr && x < x0 ? 1u : 0u;
            if (okr && k >= kd0 && k < kd1) {
                const uint32_t p = atomicAdd(&cnt[0], 1u);
                if (p < MV_RK_CAP) dk[p] = comp(k, x);
            }
            if (okr && k == kd1) {
                const uint32_t p = atomicAdd(&cnt[2], 1u);
                if (p < RK_KD1_CAP) kx1[p] = x;
            }
            if (okr && bits_ok && x >= xw && x < x1) {
                atomicAdd(&cnt[1], 1u);
                atomicOr(&bm[(x - xw) >> 5], 1u << ((x - xw) & 31u));
            }
        }
        if (base + RK_BLK * RK_U < m) load_round(base + RK_BLK * RK_U, m - 1u);
    }
    below_k = uni(block_sum<RK_BLK>(below_k, red));   // (its barriers also publish the staged entries and counts)
    below_x0 = uni(block_sum<RK_BLK>(below_x0, red));
    const uint32_t nd = uni(cnt[0]), n1 = uni(cnt[2]);
    const bool dest_staged = nd <= MV_RK_CAP;   // block-uniform
    RK_PROBE(1, wall_clock64());
    RK_PROBE(4, nd);
    RK_PROBE(5, cnt[1]);
    RK_PROBE(6, m);
    if (bits_ok) {   // the bitmap's word prefix: RK_BM_WORDS / RK_BLK consecutive words per lane
        constexpr uint32_t WPL = RK_BM_WORDS / RK_BLK;
        static_assert(WPL * RK_BLK == RK_BM_WORDS, "bitmap words per lane");
        const uint32_t nw = (x1 - xw + 31u) >> 5, w0 = WPL * threadIdx.x;
        uint32_t c[WPL], inc = 0;
#pragma unroll
        for (uint32_t j = 0; j < WPL; ++j) {
            c[j] = w0 + j < nw ? (uint32_t)__popc(bm[w0 + j]) : 0u;
            inc += c[j];
        }
        const uint32_t mine = inc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)inc, o, 64);
            if (lane_id() >= (uint32_t)o) inc += u;
        }
        __syncthreads();   // block_sum's last reads of red
        if (lane_id() == 63) red[threadIdx.x >> 6] = inc;
        __syncthreads();
        uint32_t pre = 0;
        for (uint32_t k = 0; k < (threadIdx.x >> 6); ++k) pre += red[k];
        uint32_t run = pre + inc - mine;   // words before w0
#pragma unroll
        for (uint32_t j = 0; j < WPL; ++j) {
            if (w0 + j <= nw) bpre[w0 + j] = run;
            run += c[j];
        }
        if (nw == (uint32_t)RK_BM_WORDS && threadIdx.x == RK_BLK - 1) bpre[RK_BM_WORDS] = run;
    }
    // the dest entries and the old keys in order: up to RK_COUNT of them each lane counts the smaller ones (LDS
    // broadcast reads, no barrier stages), more are sorted (lds_sort)
    const bool dcount = nd <= (uint32_t)RK_COUNT;
    if (dest_staged && dcount)
        for (uint32_t e = threadIdx.x; e < nd; e += RK_BLK) {
            const uint64_t me = dk[e];
            uint32_t lr = 0, f = 0;
            // RK_CNT_U reads in flight per round (one at a time, the count waited on LDS latency per entry)
            for (; f + (uint32_t)RK_CNT_U <= nd; f += (uint32_t)RK_CNT_U) {
                uint64_t t[RK_CNT_U];
#pragma unroll
                for (int u = 0; u < RK_CNT_U; ++u) t[u] = dk[f + (uint32_t)u];
#pragma unroll
                for (int u = 0; u < RK_CNT_U; ++u) lr += t[u] < me ? 1u : 0u;
            }
            for (; f < nd; ++f) lr += dk[f] < me ? 1u : 0u;
            ds[lr] = me;
        }
    __syncthreads();
    RK_PROBE(2, wall_clock64());
    RK_PROBE(7, bits_ok ? 1 : 0);
    // ---- multi-pass (more dest entries than MV_RK_CAP; block-uniform): copy them to ms[below_k, below_k + nd) and
    // bin them by key (bin = (k − kd0) >> sh, RK_HBINS bins over the keys the range can receive; mover keys are at
    // most ncells), then the bins' exclusive prefix and the largest bin.
    uint32_t P = 1, Cg = 1, sh = 0;
    bool mp = false;
    uint32_t kb0 = kd0;   // the bins' first key
    if (!dest_staged) {
        uint64_t* const mcopy = w.ms + below_k;   // below_k + nd <= m <= cap
        // (a rare path: plain loops, little code; the kernel's instruction footprint is shared by two CUs)
        for (uint32_t r = threadIdx.x; r < m; r += RK_BLK) {
            const uint32_t k = w.mk[r];
            if (k >= kd0 && k < kd1) {
                const uint32_t j = atomicAdd(&cnt[6], 1u);
                if (j < nd) mcopy[j] = comp(k, mv_slot(w, w.mi[r]));
                atomicMax(&cnt[7], k);    // the entries' key span [kmin, kmax]
                atomicMax(&cnt[8], ~k);
            }
        }
        for (uint32_t t = threadIdx.x; t < (uint32_t)RK_HBINS; t += RK_BLK) hp[t] = 0u;
        __syncthreads();
        // bins over the entries' own key span (a front's movers fill a few columns of a range whose key interval can
        // span every empty column of the tank: bins over [kd0, kd1) put thousands in one bin at C5, r6)
        kb0 = uni(~cnt[8]);
        const uint32_t span = uni(cnt[7]) - kb0 + 1u;
        sh = span > (uint32_t)RK_HBINS ? 32u - (uint32_t)__builtin_clz((span - 1u) >> RK_HBITS) : 0u;
        for (uint32_t t = threadIdx.x; t < nd; t += RK_BLK) atomicAdd(&hp[((uint32_t)(mcopy[t] >> 32) - kb0) >> sh], 1u);
        __syncthreads();
        constexpr uint32_t HPL = RK_HBINS / RK_BLK;   // consecutive bins per lane
        static_assert(HPL * RK_BLK == RK_HBINS, "bins per lane");
        const uint32_t h0 = HPL * threadIdx.x;
        uint32_t hc[HPL], inc = 0, mx = 0;
#pragma unroll
        for (uint32_t j = 0; j < HPL; ++j) {
            hc[j] = hp[h0 + j];
            inc += hc[j];
            mx = max(mx, hc[j]);
        }
        const uint32_t mine = inc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)inc, o, 64);
            if (lane_id() >= (uint32_t)o) inc += u;
            mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
        }
        if (lane_id() == 63) red[threadIdx.x >> 6] = inc;
        if (lane_id() == 0) atomicMax(&cnt[5], mx);
        __syncthreads();
        uint32_t run = inc - mine;
        for (uint32_t k = 0; k < (threadIdx.x >> 6); ++k) run += red[k];
#pragma unroll
        for (uint32_t j = 0; j < HPL; ++j) {
            hp[h0 + j] = run;
            run += hc[j];
        }
        if (threadIdx.x == RK_BLK - 1) hp[RK_HBINS] = run;   // == nd
        __syncthreads();
        const uint32_t maxbin = uni(cnt[5]);
        mp = maxbin <= (uint32_t)(MP_CAP / 2);   // else no bin layout fits: the whole list
        if (mp) {
            Cg = (uint32_t)MP_CAP - maxbin;
            P = (nd - 1u) / Cg + 1u;
        }
    }
    const bool dest_ok = dest_staged || mp;   // block-uniform; false: every dest count takes the whole list
    // pass state: the key sub-interval [Ka, Kb), the entries of earlier passes, this pass's sorted entries
    uint32_t Ka = kd0, Kb = kd1, before = 0, ndp = nd;
    const uint64_t* sd = dcount ? ds : dk;   // sorted dest entries (dest_staged)
    // ---- counts against the whole list (a state no LDS layout fits; counted in w.stats)
    auto count_slots = [&](uint32_t y) {   // #movers with slot < y
        uint32_t c = 0;
        for (uint32_t f = 0; f < m; ++f) c += mv_slot(w, w.mi[f]) < y ? 1u : 0u;
        return c;
    };
    auto count_dest = [&](uint64_t v) {    // #movers with (new key, slot) < v
        uint32_t c = 0;
        for (uint32_t f = 0; f < m; ++f) c += comp(w.mk[f], mv_slot(w, w.mi[f])) < v ? 1u : 0u;
        return c;
    };
    // #movers with slot < y: below x0 plus (minus) the staged slots between x0 and y
    auto rank_of = [&](uint32_t y) {   // #staged slots in [xw, y), y in [xw, x1]
        const uint32_t d = min(y, x1) - xw, wd = d >> 5;
        return bpre[wd] + (uint32_t)__popc(bm[wd] & ((1u << (d & 31u)) - 1u));
    };
    const uint32_t r0 = uni(bits_ok ? rank_of(x0) : 0u);
    auto slots_below = [&](uint32_t y) {
        if (bits_ok && y >= xw) return below_x0 + rank_of(y) - r0;
        if (w.stats) atomicAdd(w.stats + RS_WHOLE_LANES, 1u);
        return count_slots(y);
    };
    // #movers with (new key, slot) < (k, i) for k in [kd0, kd1]: below the key range plus the dest entries before it;
    // at kd1 all of those plus the kd1 movers with a smaller slot
    auto dest_below = [&](uint32_t k, uint32_t i) {
        if (!dest_ok) return count_dest(comp(k, i));
        if (k < kd1) return below_k + before + lower_bound(sd, ndp, comp(k, i));
        if (n1 > (uint32_t)RK_KD1_CAP) return count_dest(comp(k, i));
        uint32_t c = below_k + nd;
        for (uint32_t f = 0; f < n1; ++f) c += kx1[f] < i ? 1u : 0u;
        return c;
    };
    // ---- the movers of this key range: rank rk = #{(k', y) < (k, x)}, insertion slot q among the stayers,
    // A(q) = #{y : y < q}; placed at (q − A(q)) + rk. Loads first.
    auto place = [&](uint64_t c) {
        const uint32_t k = (uint32_t)(c >> 32), x = (uint32_t)c;
        const uint32_t c0 = cs[k], c1 = cs[k + 1];   // not yet updated: this workgroup's cells change after a barrier
        float4 p, v;
        int32_t pid;
        asm_load(src, (int32_t)x, p, v, pid);
        const ExtraVals e = load_extra(ex, x);
        const uint32_t q = x < c0 ? c0 : (x > c1 ? c1 : x);
        const uint32_t dst = (q - slots_below(q)) + dest_below(k, x);
        if (dst >= w.cap) {   // inconsistent tables: flag, never write past them
            if (w.err) atomicOr(w.err, SZ_OVF_MOVERS);
            return;
        }
        pos_o[dst] = p;
        vel_o[dst] = v;
        id_o[dst] = pid;
        sk_o[dst] = k;
        store_extra(ex, e, dst);
    };
    for (uint32_t pass = 0; pass < P; ++pass) {
        const bool last = pass + 1u == P;
        if (mp) {   // stage the entries of bins [ba, bb) from the copy and sort them
            const uint32_t ba = pass == 0 ? 0u : lower_bound(hp, (uint32_t)RK_HBINS, pass * Cg);
            const uint32_t bb = last ? (uint32_t)RK_HBINS : lower_bound(hp, (uint32_t)RK_HBINS, (pass + 1u) * Cg);
            Ka = uni(pass == 0 ? kd0 : kb0 + (ba << sh));
            Kb = uni(last ? kd1 : kb0 + (bb << sh));
            before = uni(hp[ba]);
            ndp = uni(min(hp[bb] - before, (uint32_t)MP_CAP));
            const uint64_t* const mcopy = w.ms + below_k;
            for (uint32_t t = threadIdx.x; t < nd; t += RK_BLK) {
                const uint64_t e = mcopy[t];
                const uint32_t k = (uint32_t)(e >> 32);
                if (k >= Ka && k < Kb) {
                    const uint32_t j = atomicAdd(&cnt[3 + (pass & 1u)], 1u);
                    if (j < (uint32_t)MP_CAP) dk[j] = e;
                }
            }
            if (threadIdx.x == 0) cnt[3 + ((pass + 1u) & 1u)] = 0u;   // the next pass's counter (read before the last barrier)
            sd = dk;
        }
        // the sort of the range's entries (more than RK_COUNT) or of this pass's: one call site (its code is long)
        if (mp || (dest_staged && !dcount)) lds_sort(dk, nullptr, ndp);   // (its first barrier publishes the staged entries)
        if (dest_ok) {
            for (uint32_t t = threadIdx.x; t < ndp; t += RK_BLK) place(dk[t]);   // (multi-pass: sorted)
        } else {
            for (uint32_t r = threadIdx.x; r < m; r += RK_BLK) {
                const uint32_t k = w.mk[r];
                if (k >= kd0 && k < kd1) place(comp(k, mv_slot(w, w.mi[r])));
            }
        }
        // ---- the stayers of [x0, x1): dst = (i − A(i)) + #{movers (k, y) < (k_i, i)}, k_i in [kd0, kd1] (multi-pass:
        // those with k_i in this pass's sub-interval, kd1 in the last). Every load of a round of slots issues before
        // its stores.
        for (uint32_t base = x0; base < x1; base += RK_BLK * RK_SU) {
            uint32_t ko[RK_SU], kn[RK_SU];
            float4 p[RK_SU], v[RK_SU];
            int32_t pid[RK_SU];
#pragma unroll
            for (int u = 0; u < RK_SU; ++u) {
                const uint32_t i = min(base + u * RK_BLK + threadIdx.x, x1 - 1u);
                ko[u] = asm_sk(src, (int32_t)i);
                kn[u] = asm_key(src, (int32_t)i);
                asm_load(src, (int32_t)i, p[u], v[u], pid[u]);
            }
#pragma unroll
            for (int u = 0; u < RK_SU; ++u) {
                const uint32_t i = base + u * RK_BLK + threadIdx.x;
                if (i >= x1 || kn[u] != ko[u]) continue;
                if (mp && !((ko[u] >= Ka && ko[u] < Kb) || (last && ko[u] == kd1))) continue;
                const uint32_t dst = (i - slots_below(i)) + dest_below(ko[u], i);
                if (dst >= w.cap) {
                    if (w.err) atomicOr(w.err, SZ_OVF_MOVERS);
                    continue;
                }
                pos_o[dst] = p[u];
                vel_o[dst] = v[u];
                id_o[dst] = pid[u];
                sk_o[dst] = ko[u];
                move_extra(ex, i, dst);   // Model R's further arrays (the reference's scale: not prefetched)
            }
        }
        if (mp && !last) __syncthreads();   // this pass's entries are read until here
    }
    if (threadIdx.x == 0 && w.stats) {   // block-uniform facts: no barrier needed
        if (!dest_ok || n1 > (uint32_t)RK_KD1_CAP || !bits_ok) atomicAdd(w.stats + RS_WHOLE, 1u);
        if (mp) {
            atomicAdd(w.stats + RS_MULTI, 1u);
            atomicAdd(w.stats + RS_PASSES, P);
        }
        if (nd > (uint32_t)(MV_RK_CAP / 4)) atomicMax(w.stats + RS_MAX_ND, nd);
    }
#ifdef SPH_RANK_PROBE
    __syncthreads();
    RK_PROBE(3, wall_clock64());
#endif
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

#ifdef SPH_RANK_PROBE
extern "C" int sph_debug_rank_probe(uint64_t* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rank_probe), sizeof(g_rank_probe)) == hipSuccess ? 0 : -1;
}
#endif

uint32_t resort_ranges(int32_t n) {
    const uint32_t nbk = ((uint32_t)std::max(n, 1) + 255u) / 256u;
    const uint32_t need = ((uint32_t)std::max(n, 1) + RK_MAX_RANGE - 1u) / RK_MAX_RANGE;
    return std::min(nbk, std::max((uint32_t)MV_RANK_GRID, need + 1u));   // (+1: the ranges are whole 256-slot blocks)
}

void launch_resort(AsmSrc src, uint32_t* cs, uint32_t* cs_new, uint32_t ncells, int32_t n, const uint32_t* count,
                   uint32_t* count_other, ResortScratch w, float4* pos_o, float4* vel_o, int32_t* id_o,
                   uint32_t* sk_o, hipStream_t s, CsPick pick, ResortExtra ex) {
    if (n <= 0) return;
    // n is an upper bound of the slots on device-sized steps: the rank kernel's ranges split the device count
    const uint32_t G = resort_ranges(n);
    // the cell shares: as many workgroups as ranges, and at most RK_CELLS cells each (C3: 256 of ~14,300 cells; C5: 895)
    const uint32_t Gc = std::max(G, (ncells + RK_CELLS) / RK_CELLS);
    if ((ncells + Gc) / Gc > RK_DIRECT)   // the largest share's cells (ncells + 1 split in Gc)
        SPH_LAUNCH(k_mv_rank<true>, G + Gc, RK_BLK, 0, s, count, count_other, cs, cs_new, ncells, pick, G, w, src, n, pos_o,
                   vel_o, id_o, sk_o, ex);
    else
        SPH_LAUNCH(k_mv_rank<false>, G + Gc, RK_BLK, 0, s, count, count_other, cs, cs_new, ncells, pick, G, w, src, n,
                   pos_o, vel_o, id_o, sk_o, ex);
}

}  // namespace sph
