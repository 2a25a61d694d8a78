// sort_small.hip — the stable radix sort of sort.hip in ONE workgroup, for small arrays, gfx950.
//
// At the reference's own scale (Model R, a few thousand particles, 16-bit cell keys) every pass of
// the multi-workgroup sort is three launches over almost no data: ~30 µs of fixed launch cost per
// step for two passes. Here 1,024 threads sort up to SORT_SMALL_N keys held in LDS (16-bit keys and
// slot indices, two ping-pong buffers: 128 KiB, plus 16 KiB of wave counters) in one launch.
// The algorithm is sort.hip's, so the permutation is the same stable one: per 8-bit digit, every
// wave counts its contiguous segment's digits (ballot match, one LDS add per distinct digit),
// the (digit, wave) counts are scanned digit-major, and each wave scatters its segment in order
// with wave-private running counters. No atomics, deterministic.
#include "common.h"

namespace sph {

constexpr int SS_BLOCK = 1024;
constexpr int SS_WAVES = SS_BLOCK / 64;

__device__ __forceinline__ uint64_t ss_match8(uint32_t d, uint64_t active) {
    uint64_t m = active;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint32_t bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        m &= bit ? bal : ~bal;
    }
    return m;
}

__global__ __launch_bounds__(SS_BLOCK) void k_sort_small(const uint32_t* __restrict__ keys_in, int32_t n,
                                                         int32_t passes, uint32_t* __restrict__ keys_out,
                                                         uint32_t* __restrict__ vals_out) {
    __shared__ uint16_t kbuf[2][SORT_SMALL_N];
    __shared__ uint16_t vbuf[2][SORT_SMALL_N];
    __shared__ uint32_t wcnt[SS_WAVES][256];
    __shared__ uint32_t wsum[SS_WAVES];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int32_t i = tid; i < n; i += SS_BLOCK) {
        kbuf[0][i] = (uint16_t)keys_in[i];
        vbuf[0][i] = (uint16_t)i;
    }
    // wave w owns the contiguous segment [seg0, seg1), whole 64-key chunks
    const int32_t span = ((n + SS_WAVES * 64 - 1) / (SS_WAVES * 64)) * 64;
    const int32_t seg0 = min(w * span, n), seg1 = min(seg0 + span, n);
    int src = 0;
    for (int p = 0; p < passes; ++p) {
        const int shift = 8 * p, dst = src ^ 1;
#pragma unroll
        for (int k = 0; k < 4; ++k) (&wcnt[0][0])[tid + k * SS_BLOCK] = 0u;
        __syncthreads();
        for (int32_t c = seg0; c < seg1; c += 64) {
            const int32_t i = c + lane;
            const bool valid = i < seg1;
            const uint32_t d = valid ? ((uint32_t)kbuf[src][i] >> shift) & 0xFFu : 0u;
            const uint64_t peers = ss_match8(d, __ballot(valid));
            if (valid && (peers & lt) == 0) wcnt[w][d] += (uint32_t)__popcll(peers);
        }
        __syncthreads();
        // exclusive scan of the counts in (digit, wave) order: thread t holds entries 4t..4t+3,
        // i.e. digit t/4, waves 4(t%4)..4(t%4)+3
        const int d0 = tid >> 2, w0 = (tid & 3) * 4;
        uint32_t v[4], s = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = wcnt[w0 + k][d0];
            s += v[k];
        }
        uint32_t inc = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)inc, o, 64);
            if (lane >= o) inc += t;
        }
        if (lane == 63) wsum[w] = inc;
        __syncthreads();
        uint32_t base = inc - s;
        for (int k = 0; k < w; ++k) base += wsum[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            wcnt[w0 + k][d0] = base;
            base += v[k];
        }
        __syncthreads();
        for (int32_t c = seg0; c < seg1; c += 64) {
            const int32_t i = c + lane;
            const bool valid = i < seg1;
            const uint32_t key = valid ? (uint32_t)kbuf[src][i] : 0u;
            const uint32_t d = (key >> shift) & 0xFFu;
            const uint64_t peers = ss_match8(d, __ballot(valid));
            const uint32_t before = wcnt[w][d];
            if (valid) {
                const uint32_t r = before + (uint32_t)__popcll(peers & lt);
                kbuf[dst][r] = (uint16_t)key;
                vbuf[dst][r] = vbuf[src][i];
            }
            // the lowest lane of each digit group advances the wave-private counter after every
            // lane of the wave has read it (same wave, in-order LDS)
            if (valid && (peers & lt) == 0) wcnt[w][d] = before + (uint32_t)__popcll(peers);
        }
        __syncthreads();
        src = dst;
    }
    for (int32_t i = tid; i < n; i += SS_BLOCK) {
        keys_out[i] = kbuf[src][i];
        vals_out[i] = vbuf[src][i];
    }
}

void launch_sort_small(const uint32_t* keys_in, int32_t n, int32_t key_bits, uint32_t* keys_out, uint32_t* vals_out,
                       hipStream_t s) {
    const int passes = key_bits <= 8 ? 1 : 2;
    if (n > 0) k_sort_small<<<1, SS_BLOCK, 0, s>>>(keys_in, n, passes, keys_out, vals_out);
}

}  // namespace sph
