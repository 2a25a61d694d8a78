// fused_perm.h — the one-launch steps at the reference's scale (contact.hip k_contact_fused, wcsph_tiled.hip
// k_density_fused): every workgroup rebuilds this step's re-sort permutation in LDS from the previous step's mover list
// (resort.hip's formulas), so a pass can read the previous step's arrays in this step's sorted order and write the new
// cell-start table, without a launch (or a grid barrier) between the re-sort and the pass.
#pragma once
#include "common.h"

// test-only phase clocks (contact.hip defines it in its -DSPH_CONTACT_PROBE build)
#ifndef FZ_PROBE
#define FZ_PROBE(slot) \
    do {               \
    } while (0)
#endif

namespace sph {

constexpr int32_t FZ_N = 4096;
constexpr int FZ_WORDS = FZ_N / 32 + 1;

struct FusedMap {
    const uint32_t* cs;    // the previous step's cell-start table
    const uint64_t* ms;    // LDS: movers by (new key, old slot)
    const uint32_t* dst;   // LDS: their sorted positions, ascending
    const uint32_t* bm;    // LDS: the movers' old slots as bits, and the words' exclusive prefix
    const uint32_t* bpre;
    uint32_t m;
    __device__ __forceinline__ uint32_t A(uint32_t y) const {   // movers with an old slot < y
        const uint32_t wd = y >> 5;
        return bpre[wd] + (uint32_t)__popc(bm[wd] & ((1u << (y & 31u)) - 1u));
    }
    __device__ __forceinline__ uint32_t start(uint32_t k) const { return start_c(k, cs[k]); }   // cs_new[k]
    // the same from c = cs[k] loaded by the caller (several keys' loads in flight before any search)
    __device__ __forceinline__ uint32_t start_c(uint32_t k, uint32_t c) const {
        if (m == 0) return c;
        uint32_t lo = 0, hi = m;   // movers with new key < k
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint32_t)(ms[mid] >> 32) < k) lo = mid + 1;
            else hi = mid;
        }
        return c + lo - A(c);   // old keys follow the old slots: movers with an old key < k = A(cs[k])
    }
    // LDS: for every sorted position its previous slot (bits 0-15) and, for a mover, 1 + its index in ms (bits 16-31)
    const uint32_t* pm;
    __device__ __forceinline__ uint32_t old(uint32_t j) const { return m == 0 ? j : (pm[j] & 0xffffu); }
    // the previous order's slot of sorted position j, from the table; mv: it is a mover (its new key in key)
    __device__ __forceinline__ uint32_t old_at(uint32_t j, bool& mv, uint32_t& key) const {
        mv = false;
        if (m == 0) return j;
        const uint32_t e = pm[j];
        if (e >> 16) {
            mv = true;
            key = (uint32_t)(ms[(e >> 16) - 1u] >> 32);
        }
        return e & 0xffffu;
    }
};


// The permutation of a step with m movers (mi: old slot, mk: new key) over n <= FZ_N slots, built by every thread of a
// BLK-thread workgroup into LDS; from workgroup 0 it also zeroes `zero` and stores m into host_count (mapped host
// memory) when given. The caller writes the workgroup's share of the new cell-start table (fused_cs_share).
struct FusedLds {
    uint64_t ms[FZ_N];
    uint32_t dst[FZ_N];
    uint32_t bm[FZ_WORDS], bpre[FZ_WORDS];
    uint32_t pm[FZ_N];
};

// the bitmap's exclusive word prefix (nw <= FZ_WORDS words) by one wave, lane t: WPW consecutive words per lane and one
// DPP scan over the wave (r6: three dependent 64-word shuffle scans took ~0.4 us)
constexpr uint32_t WPW = (FZ_WORDS + 63) / 64;
__device__ __forceinline__ void word_prefix(const uint32_t* bm, uint32_t* bpre, uint32_t nw, uint32_t lane) {
    uint32_t c[WPW], mine = 0;
#pragma unroll
    for (uint32_t j = 0; j < WPW; ++j) {
        const uint32_t t = lane * WPW + j;
        c[j] = t < nw ? (uint32_t)__popc(bm[t]) : 0u;
        mine += c[j];
    }
    const uint32_t inc = wave_scan_incl(mine);
    uint32_t run = inc - mine;
#pragma unroll
    for (uint32_t j = 0; j < WPW; ++j) {
        const uint32_t t = lane * WPW + j;
        if (t < nw) bpre[t] = run;
        run += c[j];
    }
}

template <int BLK>
__device__ FusedMap fused_build(FusedLds& L, const uint32_t* __restrict__ count, const uint32_t* __restrict__ mi,
                                const uint32_t* __restrict__ mk, const uint32_t* __restrict__ cs, int32_t n, uint32_t* zero,
                                uint32_t* host_count) {
    uint64_t* ms = L.ms;
    uint32_t* dst = L.dst;
    uint32_t* bm = L.bm;
    uint32_t* bpre = L.bpre;
    uint32_t* pm = L.pm;
    // the count and the first BLK movers' entries in one round trip (the lists hold n entries: in bounds). The entries
    // are loaded first and the count after them through the vector path (ld_vec): as a scalar load, the count held the
    // entries' loads back by one round trip
    uint32_t x0 = 0u, k0 = 0u;
    if (threadIdx.x < (uint32_t)n) {
        x0 = mi[threadIdx.x];
        k0 = mk[threadIdx.x];
    }
    const uint32_t m_raw = ld_vec(count);
    const uint32_t nw = ((uint32_t)n >> 5) + 1u;
    for (uint32_t t = threadIdx.x; t < nw; t += BLK) bm[t] = 0u;
    const uint32_t m = min(m_raw, (uint32_t)n);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (zero) *zero = 0u;
        if (host_count) *host_count = m;
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < m; r += BLK) {
        const uint32_t x = r < (uint32_t)BLK ? x0 : mi[r], k = r < (uint32_t)BLK ? k0 : mk[r];
        ms[r] = (uint64_t)k << 32 | x;
        atomicOr(&bm[x >> 5], 1u << (x & 31u));
    }
    // the old cell range of a mover's new key (its position below clamps the slot into it), loaded under the sort
    uint32_t c0 = 0u, c1 = 0u;
    if (threadIdx.x < m) {
        c0 = cs[k0];
        c1 = cs[k0 + 1u];
    }
    __syncthreads();
    FZ_PROBE(4);
    // the movers in (new key, slot) order: up to BLK by counting (each entry's clamped slot q rides along in dst),
    // more by a bitonic sort
    const bool counted = m <= (uint32_t)BLK;
    // the bitmap's word prefix needs only the bitmap: the last wave takes it beside a counting sort that leaves it idle
    const bool pre_last = m <= (uint32_t)BLK - 64u;
    if (pre_last && threadIdx.x >= (uint32_t)BLK - 64u) word_prefix(bm, bpre, nw, threadIdx.x - ((uint32_t)BLK - 64u));
    if (counted) {
        uint64_t e = 0;
        uint32_t rk = 0;
        if (threadIdx.x < m) {
            e = ms[threadIdx.x];
            // eight LDS reads in flight per round: one at a time, the count waited on LDS latency (~m x 70 cycles)
            uint32_t f = 0;
            for (; f + 8u <= m; f += 8u) {
                uint64_t t[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) t[u] = ms[f + (uint32_t)u];
#pragma unroll
                for (int u = 0; u < 8; ++u) rk += t[u] < e ? 1u : 0u;
            }
            for (; f < m; ++f) rk += ms[f] < e ? 1u : 0u;
        }
        __syncthreads();
        if (threadIdx.x < m) {
            ms[rk] = e;
            dst[rk] = x0 < c0 ? c0 : (x0 > c1 ? c1 : x0);
        }
    } else {
        uint32_t P = 1;
        while (P < m) P <<= 1;
        for (uint32_t t = m + threadIdx.x; t < P; t += BLK) ms[t] = ~0ull;
        __syncthreads();
        for (uint32_t k = 2; k <= P; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t t = threadIdx.x; t < P / 2; t += BLK) {
                    const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), u = i | j;
                    const uint64_t x = ms[i], y = ms[u];
                    if ((x > y) == ((i & k) == 0)) {
                        ms[i] = y;
                        ms[u] = x;
                    }
                }
                __syncthreads();
            }
    }
    FZ_PROBE(5);
    if (!pre_last && threadIdx.x < 64) word_prefix(bm, bpre, nw, threadIdx.x);
    __syncthreads();
    FusedMap M{cs, ms, dst, bm, bpre, m, pm};
    for (uint32_t r = threadIdx.x; r < m; r += BLK) {   // the movers' sorted positions (q − A(q)) + r
        uint32_t q;
        if (counted) {
            q = dst[r];
        } else {
            const uint32_t k = (uint32_t)(ms[r] >> 32), x = (uint32_t)ms[r];
            const uint32_t a0 = cs[k], a1 = cs[k + 1];
            q = x < a0 ? a0 : (x > a1 ? a1 : x);
        }
        dst[r] = (q - M.A(q)) + r;
    }
    __syncthreads();
    FZ_PROBE(6);
    if (m) {   // the whole permutation: a lookup is one LDS read
        // movers at their positions; stayers scattered from the old order: a thread takes a run of old slots, the
        // stayer of rank s = i − A(i) lands at s + #{r : dst[r] − r <= s} (dst[r] − r, the stayers placed before
        // mover r, does not decrease): one search for the run's first stayer, then a walk
        for (uint32_t r = threadIdx.x; r < m; r += BLK) pm[dst[r]] = (uint32_t)ms[r] | ((r + 1u) << 16);
        const uint32_t per = ((uint32_t)n + BLK - 1u) / BLK;
        const uint32_t i0 = threadIdx.x * per, i1 = min(i0 + per, (uint32_t)n);
        if (i0 < i1) {
            uint32_t st = i0 - M.A(i0);
            uint32_t lo = 0, hi = m;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (dst[mid] - mid <= st) lo = mid + 1;
                else hi = mid;
            }
            for (uint32_t i = i0; i < i1; ++i) {
                if ((bm[i >> 5] >> (i & 31u)) & 1u) continue;   // a mover
                while (lo < m && dst[lo] - lo <= st) ++lo;
                pm[st + lo] = i;
                ++st;
            }
        }
        __syncthreads();
    }
    return M;
}

// This workgroup's share of the new cell-start table (ncells + 2 entries; entry ncells + 1, the slot count, unchanged),
// by threads t = 0..T-1 of it. The pass needs none of it, so a kernel runs it where its lanes would idle.
__device__ __forceinline__ void fused_cs_share(const FusedMap& M, uint32_t* __restrict__ cs_o, uint32_t ncells,
                                               uint32_t t, uint32_t T) {
    const uint32_t tot = ncells + 2u, G = gridDim.x;
    const uint32_t k0 = (uint32_t)((uint64_t)tot * blockIdx.x / G), k1 = (uint32_t)((uint64_t)tot * (blockIdx.x + 1) / G);
    for (uint32_t k = k0 + t; k < k1; k += T) cs_o[k] = k <= ncells ? M.start(k) : M.cs[k];
}

}  // namespace sph
