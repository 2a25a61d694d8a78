// sort.hip — stable LSD radix sort of (cell key, particle slot) pairs for gfx950.
//
// Replaces the reference's per-cell linked lists built with InterlockedExchange
// (SimulateParticles.compute:196-209): the north star asks for hash + radix sort +
// cell-start, and a stable sort gives a unique, deterministic neighbour order.
//
// One pass = 8 key bits = 3 launches:
//   rs_hist    per 2048-key tile: 256-bin digit histogram (wave64 ballot-match, one LDS
//              add per distinct digit per wave instead of one per key);
//   rs_scan    one workgroup per digit: exclusive scan of that digit's per-tile counts
//              (digit-major layout, so a row is contiguous) + the digit total;
//   rs_scatter per tile: global digit base + tile prefix + stable in-tile rank. The rank
//              comes from a 64-bit ballot match of the 8 digit bits (peers = lanes with the
//              same digit) and mbcnt-style popcounts, with wave-private running counters in
//              LDS, so ranks follow the global index order (stable) without any atomics.
#include "common.h"

namespace sph {

constexpr int RS_BLOCK = 256;
constexpr int RS_WAVES = RS_BLOCK / 64;
constexpr int RS_CHUNKS = 8;                      // 64-key chunks per wave
constexpr int RS_TILE = RS_BLOCK * RS_CHUNKS;     // 2048 keys per workgroup
constexpr int RS_WAVE_SPAN = 64 * RS_CHUNKS;      // 512 contiguous keys per wave
constexpr int RS_BINS = 256;

__device__ __forceinline__ uint64_t lanemask_lt() {
    return (1ull << lane_id()) - 1ull;
}

// Lanes (among `active`) whose 8-bit digit equals this lane's digit.
__device__ __forceinline__ uint64_t match_digit8(uint32_t d, uint64_t active) {
    uint64_t m = active;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint32_t bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        m &= bit ? bal : ~bal;
    }
    return m;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// Exclusive scan over a 256-thread block. `wsum` holds 4 words of LDS.
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (int k = 0; k < RS_WAVES; ++k) pre += (k < w) ? wsum[k] : 0u;
    const uint32_t tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    *total = tot;
    return pre + inc - v;
}

__global__ __launch_bounds__(RS_BLOCK) void rs_hist(const uint32_t* __restrict__ keys, int32_t n,
                                                    int32_t shift, uint32_t* __restrict__ hist,
                                                    int32_t ntiles) {
    __shared__ uint32_t cnt[RS_BINS];
    cnt[threadIdx.x] = 0;
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t base = (int64_t)blockIdx.x * RS_TILE + w * RS_WAVE_SPAN;
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int c = 0; c < RS_CHUNKS; ++c) {
        const int64_t i = base + c * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = valid ? (keys[i] >> shift) & 0xFFu : 0u;
        const uint64_t act = __ballot(valid);
        const uint64_t peers = match_digit8(d, act);
        if (valid && (peers & lt) == 0) atomicAdd(&cnt[d], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    hist[(int64_t)threadIdx.x * ntiles + blockIdx.x] = cnt[threadIdx.x];
}

__global__ __launch_bounds__(RS_BLOCK) void rs_scan(uint32_t* __restrict__ hist, int32_t ntiles,
                                                    uint32_t* __restrict__ bin_total) {
    __shared__ uint32_t wsum[RS_WAVES];
    uint32_t* row = hist + (int64_t)blockIdx.x * ntiles;
    uint32_t carry = 0;
    for (int32_t b = 0; b < ntiles; b += RS_BLOCK) {
        const int32_t i = b + threadIdx.x;
        const uint32_t v = i < ntiles ? row[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan256(v, wsum, &tot);
        if (i < ntiles) row[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) bin_total[blockIdx.x] = carry;
}

__global__ __launch_bounds__(RS_BLOCK) void rs_scatter(const uint32_t* __restrict__ keys_in,
                                                       const uint32_t* __restrict__ vals_in,
                                                       uint32_t* __restrict__ keys_out,
                                                       uint32_t* __restrict__ vals_out, int32_t n,
                                                       int32_t shift, const uint32_t* __restrict__ hist,
                                                       const uint32_t* __restrict__ bin_total,
                                                       int32_t ntiles) {
    __shared__ uint32_t bin_base[RS_BINS];
    __shared__ uint32_t wcnt[RS_WAVES][RS_BINS];
    __shared__ uint32_t wsum[RS_WAVES];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    {
        uint32_t tot;
        const uint32_t ex = block_excl_scan256(bin_total[tid], wsum, &tot);
        bin_base[tid] = ex + hist[(int64_t)tid * ntiles + blockIdx.x];
#pragma unroll
        for (int k = 0; k < RS_WAVES; ++k) wcnt[k][tid] = 0;
    }
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * RS_TILE + w * RS_WAVE_SPAN;
    const uint64_t lt = lanemask_lt();
    uint32_t key[RS_CHUNKS], rank[RS_CHUNKS];
#pragma unroll
    for (int c = 0; c < RS_CHUNKS; ++c) {
        const int64_t i = base + c * 64 + lane;
        const bool valid = i < n;
        const uint32_t k = valid ? keys_in[i] : 0xFFFFFFFFu;
        const uint32_t d = (k >> shift) & 0xFFu;
        const uint64_t act = __ballot(valid);
        const uint64_t peers = match_digit8(d, act);
        const uint32_t before = wcnt[w][d];
        rank[c] = before + (uint32_t)__popcll(peers & lt);
        key[c] = k;
        // the lowest lane of each digit group advances the wave-private counter; the
        // read above has completed for all lanes (same wave, in-order LDS)
        if (valid && (peers & lt) == 0) wcnt[w][d] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    {
        uint32_t s = 0;
#pragma unroll
        for (int k = 0; k < RS_WAVES; ++k) {
            const uint32_t v = wcnt[k][tid];
            wcnt[k][tid] = s;
            s += v;
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < RS_CHUNKS; ++c) {
        const int64_t i = base + c * 64 + lane;
        if (i < n) {
            const uint32_t d = (key[c] >> shift) & 0xFFu;
            const uint32_t dst = bin_base[d] + wcnt[w][d] + rank[c];
            keys_out[dst] = key[c];
            vals_out[dst] = vals_in ? vals_in[i] : (uint32_t)i;
        }
    }
}

size_t radix_hist_elems(int32_t capacity) {
    const int64_t ntiles = ((int64_t)capacity + RS_TILE - 1) / RS_TILE;
    return (size_t)(ntiles < 1 ? 1 : ntiles) * RS_BINS;
}

int radix_sort(uint32_t* keys_a, uint32_t* vals_a, uint32_t* keys_b, uint32_t* vals_b, int32_t n,
               int32_t key_bits, bool identity_vals, uint32_t* hist, uint32_t* bin_total,
               hipStream_t s) {
    if (n <= 0) return 0;
    if (identity_vals && n <= SORT_SMALL_N && key_bits <= 16) {   // one launch instead of 3 per pass
        launch_sort_small(keys_a, n, key_bits, keys_b, vals_b, s);
        return 1;
    }
    const int32_t ntiles = (n + RS_TILE - 1) / RS_TILE;
    const int passes = key_bits <= 0 ? 1 : (key_bits + 7) / 8;
    uint32_t* K[2] = {keys_a, keys_b};
    uint32_t* V[2] = {vals_a, vals_b};
    for (int p = 0; p < passes; ++p) {
        const int src = p & 1, dst = src ^ 1, shift = 8 * p;
        const uint32_t* vin = (p == 0 && identity_vals) ? nullptr : V[src];
        rs_hist<<<ntiles, RS_BLOCK, 0, s>>>(K[src], n, shift, hist, ntiles);
        rs_scan<<<RS_BINS, RS_BLOCK, 0, s>>>(hist, ntiles, bin_total);
        rs_scatter<<<ntiles, RS_BLOCK, 0, s>>>(K[src], vin, K[dst], V[dst], n, shift, hist,
                                               bin_total, ntiles);
    }
    return passes & 1;
}

}  // namespace sph
