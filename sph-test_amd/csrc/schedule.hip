// schedule.hip — the neighbour passes' workgroup -> target-range table (y-band schedule), gfx950.
//
// Each workgroup of k_density_tiled / k_force_tiled stages, per dx plane, the rows around its 256 targets; every
// particle is staged again by the workgroups of the columns on either side and of the y rows around it. Which XCD
// runs those workgroups decides whether a re-stage hits in that XCD's L2 (MI355X_MICROARCH.md: 4 MB per XCD, 8 XCDs,
// workgroups dealt to XCDs round-robin by dispatch index). Workgroups in sorted order, dealt in runs of 16
// (common.h xcd_block), send the x +- 1 and y +- 1 neighbours of a run to other XCDs.
// This table deals the targets instead by y bands: the y rows are cut into SCHED_BANDS bands of equal particle
// counts, band b goes to XCD b mod 8, and an XCD runs its bands' rows column by column, so a row and the rows
// staged around it run on one XCD within a few columns of each other (scripts/xcd_reuse_model.py: C3 staging reads
// 123 -> 51 B per particle, a C5/8 rank's 259 -> 51). Entry d (dispatch index) holds the target range [x, y) of
// workgroup d: XCD q = d mod 8 runs its segments' blocks at k = d / 8 in order; a segment (band, column) is cut into
// blocks of at most 256 targets; past an XCD's last block the entries are empty ranges.
// Any partition of the targets into ranges of at most 256 gives the same results (no result depends on the block
// partition), so the table may be rebuilt only every few steps: a stale one is still a partition while
// the slot count is unchanged. table[0] is a header: x = 1 when every XCD's blocks fit the launch's entries (a band
// that cannot be split, e.g. most particles in one y row, can give one XCD more); x = 0 makes the passes fall back
// to their own mapping for this table.
#include "common.h"

namespace sph {

constexpr int SCH_THREADS = 1024;
constexpr int SCH_MAX_GY = 4096;       // y rows the histogram holds (C5: 213)
constexpr int SCH_MAX_SEGS = 8192;     // bands x columns

__global__ __launch_bounds__(SCH_THREADS) void k_schedule(const uint32_t* __restrict__ cs, GridDesc g, int32_t n,
                                                          uint2* __restrict__ table, int32_t entries) {
    __shared__ uint32_t H[SCH_MAX_GY + 1];   // rows' particle counts, then their exclusive prefix
    __shared__ uint32_t edge[SCHED_BANDS + 1];
    __shared__ uint32_t segb[SCH_MAX_SEGS];  // blocks per segment (band-major), then per-XCD exclusive prefix
    __shared__ uint32_t kq[8];
    __shared__ uint32_t red[SCH_THREADS / 64];
    const uint32_t tid = threadIdx.x;
    const uint32_t gxs = (uint32_t)(g.gx * g.xsub), gy = (uint32_t)g.gy, gz = (uint32_t)g.gz;
    auto row_start = [&](uint32_t c, uint32_t y) { return cs[(c * gy + y) * gz]; };   // y == gy: the next column's
    for (uint32_t y = tid; y <= gy; y += SCH_THREADS) H[y] = 0u;
    __syncthreads();
    for (uint32_t t = tid; t < gxs * gy; t += SCH_THREADS) {
        const uint32_t c = t / gy, y = t % gy;
        const uint32_t len = row_start(c, y + 1) - row_start(c, y);
        if (len) atomicAdd(&H[y], len);
    }
    __syncthreads();
    if (tid == 0) {   // exclusive prefix over the rows (gy is small), band edges at equal counts
        uint32_t run = 0;
        for (uint32_t y = 0; y < gy; ++y) {
            const uint32_t v = H[y];
            H[y] = run;
            run += v;
        }
        H[gy] = run;
        uint32_t y = 0;
        edge[0] = 0;
        for (int b = 1; b < SCHED_BANDS; ++b) {
            const uint64_t target = (uint64_t)run * (uint64_t)b / SCHED_BANDS;
            while (y < gy && H[y] < target) ++y;
            edge[b] = y;
        }
        edge[SCHED_BANDS] = gy;
    }
    __syncthreads();
    const uint32_t nseg = SCHED_BANDS * gxs;
    for (uint32_t s = tid; s < nseg; s += SCH_THREADS) {
        const uint32_t b = s / gxs, c = s % gxs;
        const uint32_t len = row_start(c, edge[b + 1]) - row_start(c, edge[b]);
        segb[s] = (len + 255u) / 256u;
    }
    __syncthreads();
    // per XCD q, its segments in run order (bands q, q + 8, ..., columns ascending): exclusive prefix of the blocks
    constexpr int PER_Q = SCHED_BANDS / 8;
    for (int q = 0; q < 8; ++q) {
        const uint32_t m = PER_Q * gxs;   // segments of XCD q
        uint32_t carry = 0;
        for (uint32_t base = 0; base < m; base += SCH_THREADS) {
            const uint32_t t = base + tid;
            const uint32_t s = t < m ? (uint32_t)(q + 8 * (int)(t / gxs)) * gxs + t % gxs : 0u;
            const uint32_t v = t < m ? segb[s] : 0u;
            uint32_t inc = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = (uint32_t)__shfl_up((int)inc, o, 64);
                if ((tid & 63u) >= (uint32_t)o) inc += u;
            }
            if ((tid & 63u) == 63u) red[tid >> 6] = inc;
            __syncthreads();
            uint32_t pre = 0, tot = 0;
            for (uint32_t k = 0; k < SCH_THREADS / 64; ++k) {
                pre += k < (tid >> 6) ? red[k] : 0u;
                tot += red[k];
            }
            __syncthreads();
            if (t < m) segb[s] = carry + pre + inc - v;
            carry += tot;
        }
        if (tid == 0) kq[q] = carry;
        __syncthreads();
    }
    // the entries (table[1 + d]): every segment's blocks, then empty ranges up to the launch's grid bound
    const uint32_t kmax = (uint32_t)entries / 8u;
    const uint32_t keyed = cs[g.ncells];
    const uint32_t tail = ((uint32_t)n - min(keyed, (uint32_t)n) + 255u) / 256u;   // XCD 0's blocks of [keyed, n)
    bool fits = kq[0] + tail <= kmax;
    for (int q = 1; q < 8; ++q) fits = fits && kq[q] <= kmax;
    if (tid == 0) table[0] = make_uint2(fits ? 1u : 0u, kmax);
    if (!fits) return;
    table += 1;
    for (uint32_t s = tid; s < nseg; s += SCH_THREADS) {
        const uint32_t b = s / gxs, c = s % gxs, q = b % 8u;
        const uint32_t s0 = row_start(c, edge[b]), s1 = row_start(c, edge[b + 1]);
        uint32_t k = segb[s];
        for (uint32_t i = s0; i < s1; i += 256u, ++k) {
            const uint32_t d = k * 8u + q;
            table[d] = make_uint2(i, min(i + 256u, s1));   // k < kq[q] <= kmax: d < entries
        }
    }
    // slots past the keyed ones (a key at the sentinel ncells) and the empty tail
    for (uint32_t d = tid; d < (uint32_t)entries; d += SCH_THREADS) {
        const uint32_t q = d % 8u, k = d / 8u;
        if (k < kq[q]) continue;
        uint2 e = make_uint2(0u, 0u);
        if (q == 0) {   // XCD 0's next blocks take [keyed, n)
            const uint32_t i = keyed + (k - kq[0]) * 256u;
            if (i < (uint32_t)n) e = make_uint2(i, min(i + 256u, (uint32_t)n));
        }
        table[d] = e;
    }
}

int32_t schedule_entries(int32_t n, const GridDesc& g) {
    // every segment adds at most one partial block; each XCD's share with 25% to spare (equal-count bands split the
    // targets evenly but for whole rows); whole rows of 8
    const int64_t blocks = ((int64_t)n + 255) / 256 + (int64_t)SCHED_BANDS * g.gx * g.xsub;
    const int64_t per_xcd = (blocks + 7) / 8 * 5 / 4 + 2;
    return (int32_t)(per_xcd * 8);
}

bool schedule_fits(const GridDesc& g) {
    return g.gy <= SCH_MAX_GY && (int64_t)SCHED_BANDS * g.gx * g.xsub <= SCH_MAX_SEGS;
}

void launch_schedule(const uint32_t* cs, GridDesc g, int32_t n, uint2* table, int32_t entries, hipStream_t s) {
    SPH_LAUNCH(k_schedule, 1, SCH_THREADS, 0, s, cs, g, n, table, entries);
}

}  // namespace sph
