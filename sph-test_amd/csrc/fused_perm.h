// fused_perm.h — the one-launch steps at the reference's scale (contact.hip k_contact_fused, wcsph_tiled.hip
// k_density_fused): every workgroup rebuilds this step's re-sort permutation in LDS from the previous step's mover list
// (resort.hip's formulas), so a pass can read the previous step's arrays in this step's sorted order and write the new
// cell-start table, without a launch (or a grid barrier) between the re-sort and the pass.
#pragma once
#include "common.h"

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
    __device__ __forceinline__ uint32_t start(uint32_t k) const {   // cs_new[k]
        const uint32_t c = cs[k];
        if (m == 0) return c;
        uint32_t lo = 0, hi = m;   // movers with new key < k
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint32_t)(ms[mid] >> 32) < k) lo = mid + 1;
            else hi = mid;
        }
        return c + lo - A(c);   // old keys follow the old slots: movers with an old key < k = A(cs[k])
    }
    // the previous order's slot of sorted position j; mv: it is a mover (its new key in key)
    __device__ __forceinline__ uint32_t old_of(uint32_t j, bool& mv, uint32_t& key) const {
        mv = false;
        if (m == 0) return j;
        uint32_t lo = 0, hi = m;   // movers placed below j
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (dst[mid] < j) lo = mid + 1;
            else hi = mid;
        }
        if (lo < m && dst[lo] == j) {
            mv = true;
            key = (uint32_t)(ms[lo] >> 32);
            return (uint32_t)ms[lo];
        }
        const uint32_t s = j - lo;   // the s-th stayer: the smallest i with (i + 1) − A(i + 1) > s, i in [s, s + m]
        uint32_t a = s, b = s + m;
        while (a < b) {
            const uint32_t mid = (a + b) >> 1;
            if (mid + 1u - A(mid + 1u) > s) b = mid;
            else a = mid + 1;
        }
        return a;
    }
    const uint16_t* pm;    // LDS: old_of for every sorted position (filled once per workgroup)
    __device__ __forceinline__ uint32_t old(uint32_t j) const { return m == 0 ? j : (uint32_t)pm[j]; }
};


// The permutation of a step with m movers (mi: old slot, mk: new key) over n <= FZ_N slots, built by every thread of a
// BLK-thread workgroup into LDS; also writes the workgroup's share of the new cell-start table (cs_o, ncells + 2
// entries) and, from workgroup 0, zeroes `zero` and stores m into host_count (mapped host memory) when given.
struct FusedLds {
    uint64_t ms[FZ_N];
    uint32_t dst[FZ_N];
    uint32_t bm[FZ_WORDS], bpre[FZ_WORDS];
    uint16_t pm[FZ_N];
};

template <int BLK>
__device__ FusedMap fused_build(FusedLds& L, const uint32_t* __restrict__ count, const uint32_t* __restrict__ mi,
                                const uint32_t* __restrict__ mk, const uint32_t* __restrict__ cs, uint32_t* __restrict__ cs_o,
                                uint32_t ncells, int32_t n, uint32_t* zero, uint32_t* host_count) {
    uint64_t* ms = L.ms;
    uint32_t* dst = L.dst;
    uint32_t* bm = L.bm;
    uint32_t* bpre = L.bpre;
    uint16_t* pm = L.pm;
    const uint32_t m = min(*count, (uint32_t)n);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (zero) *zero = 0u;
        if (host_count) *host_count = m;
    }
    const uint32_t nw = ((uint32_t)n >> 5) + 1u;
    for (uint32_t t = threadIdx.x; t < nw; t += BLK) bm[t] = 0u;
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < m; r += BLK) {
        const uint32_t x = mi[r], k = mk[r];
        ms[r] = (uint64_t)k << 32 | x;
        atomicOr(&bm[x >> 5], 1u << (x & 31u));
    }
    __syncthreads();
    // the movers in (new key, slot) order: up to BLK by counting, more by a bitonic sort
    if (m <= (uint32_t)BLK) {
        uint64_t e = 0;
        uint32_t rk = 0;
        if (threadIdx.x < m) {
            e = ms[threadIdx.x];
            for (uint32_t f = 0; f < m; ++f) rk += ms[f] < e ? 1u : 0u;
        }
        __syncthreads();
        if (threadIdx.x < m) ms[rk] = e;
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
    // the bitmap's word prefix (nw <= FZ_WORDS words)
    if (threadIdx.x < 64) {
        uint32_t carry = 0;
        for (uint32_t base = 0; base < nw; base += 64) {
            const uint32_t t = base + threadIdx.x;
            const uint32_t v = t < nw ? (uint32_t)__popc(bm[t]) : 0u;
            uint32_t inc = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = (uint32_t)__shfl_up((int)inc, o, 64);
                if (lane_id() >= (uint32_t)o) inc += u;
            }
            if (t < nw) bpre[t] = carry + inc - v;
            carry += (uint32_t)__shfl((int)inc, 63, 64);
        }
    }
    __syncthreads();
    FusedMap M{cs, ms, dst, bm, bpre, m, pm};
    for (uint32_t r = threadIdx.x; r < m; r += BLK) {   // the movers' sorted positions
        const uint32_t k = (uint32_t)(ms[r] >> 32), x = (uint32_t)ms[r];
        const uint32_t c0 = cs[k], c1 = cs[k + 1];
        const uint32_t q = x < c0 ? c0 : (x > c1 ? c1 : x);
        dst[r] = (q - M.A(q)) + r;
    }
    __syncthreads();
    if (m) {   // the whole permutation: a lookup is one LDS read
        for (uint32_t j = threadIdx.x; j < (uint32_t)n; j += BLK) {
            bool mv;
            uint32_t key;
            pm[j] = (uint16_t)M.old_of(j, mv, key);
        }
        __syncthreads();
    }
    {   // this workgroup's share of the new cell-start table (entry ncells + 1: the slot count, unchanged)
        const uint32_t tot = ncells + 2u, G = gridDim.x;
        const uint32_t k0 = (uint32_t)((uint64_t)tot * blockIdx.x / G), k1 = (uint32_t)((uint64_t)tot * (blockIdx.x + 1) / G);
        for (uint32_t k = k0 + threadIdx.x; k < k1; k += BLK) cs_o[k] = k <= ncells ? M.start(k) : cs[k];
    }
    return M;
}

}  // namespace sph
