// slab.hip — device side of the x-slab decomposition (SPEC_SPH.md §3), gfx950.
//
// The reference is single-GPU. Here a rank owns global cell columns
// [cx_lo, cx_hi) and holds one halo column on each side. Keys are x-slowest, so every column
// is a contiguous run of sorted slots. Send lists are filtered runs, and the order of those
// runs is load-bearing: both ranks must sort a shared column into the same order.
// So every compaction here is ORDER-PRESERVING: per-block counts, one exclusive scan, then
// a scatter whose in-block ranks come from wave64 ballots + mbcnt and per-wave prefixes in
// LDS. No atomics, no dependence on block scheduling.
#include "common.h"

namespace sph {

constexpr int SL_BLK = 256;
constexpr int SL_WAVES = SL_BLK / 64;

int32_t slab_compact_blocks(int32_t b, int32_t e) { return e > b ? (e - b + SL_BLK - 1) / SL_BLK : 1; }

__device__ __forceinline__ uint32_t lane_prefix(uint64_t mask) {   // set lanes below this lane
    return (uint32_t)__popcll(mask & ((1ull << lane_id()) - 1ull));
}

// Block-wide count of a predicate -> per-wave counts in LDS; returns the block total.
__device__ __forceinline__ uint32_t block_ballot_count(bool pred, uint32_t* wcnt, uint32_t& wave_base) {
    const int w = threadIdx.x >> 6;
    const uint64_t m = __ballot(pred);
    if ((threadIdx.x & 63) == 0) wcnt[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < SL_WAVES; ++k) {
        base += k < w ? wcnt[k] : 0u;
        tot += wcnt[k];
    }
    wave_base = base;
    return tot;
}

// Send lists: each workgroup of the count / pack pair takes SL_SEND consecutive owned slots, so the
// single-workgroup scan between them sees few entries (one pass per side at C3).
constexpr int SL_PER = SPH_SL_PER;
constexpr int SL_SEND = SL_BLK * SL_PER;
static_assert(SL_SEND == SEND_SLOTS, "send blocks: common.h SEND_SLOTS");

int32_t slab_send_blocks(int32_t b, int32_t e) { return e > b ? (e - b + SL_SEND - 1) / SL_SEND : 1; }

// The own slots each side's sends are taken from (previous order). Device-sized steps: all own slots
// [o0, o1), or, in steady state (cand: the cut is older than the previous step, so its column starts are
// the picks), only the columns a send can come from: a particle moves less than a column per step, so one
// that is now in column <= lo was in lo or lo + 1 (left), >= hi - 1 in hi - 2 or hi - 1 (right). A force
// pass that moved an own particle further sets dz->jump, and the next sends scan every own slot again.
// Early sends (the next step's, packed right after this step's boundary force pass, abi_multi.cpp): the owned range is
// this step's [pick[1], pick[4]) (k_slab_lag has not run yet), and dz->jump is not consulted: the boundary pass that
// moved the candidate columns has finished, and the interior pass reports its jumps as SZ_JUMP_EARLY instead.
__device__ __forceinline__ void send_ranges(const SlabSizes* __restrict__ dz, int32_t cand, int32_t& bl, int32_t& el,
                                            int32_t& br, int32_t& er, int32_t early = 0) {
    bl = br = (int32_t)(early ? dz->pick[1] : dz->o0);
    el = er = (int32_t)(early ? dz->pick[4] : dz->o1);
    if (cand && (early || dz->jump == 0u)) {
        el = max(bl, min(el, (int32_t)dz->pick[6]));
        br = min(er, max(br, (int32_t)dz->pick[7]));
    }
}

__global__ __launch_bounds__(SL_BLK) void k_slab_count(const uint32_t* __restrict__ keys, int32_t b, int32_t e,
                                                       uint32_t gyz, int32_t col_le, int32_t col_ge,
                                                       uint32_t* __restrict__ blk, int32_t nblk,
                                                       const SlabSizes* __restrict__ dz, int32_t cand, int32_t early) {
    __shared__ uint32_t wl[SL_WAVES], wr[SL_WAVES];
    int32_t bl = b, el = e, br = b, er = e;
    if (dz) send_ranges(dz, cand, bl, el, br, er, early);   // device-sized step; nblk is an upper bound
    uint32_t cl = 0, cr = 0;
    if (bl == br && el == er) {   // one range for both sides
        const int32_t i0 = bl + blockIdx.x * SL_SEND + threadIdx.x;
#pragma unroll
        for (int j = 0; j < SL_PER && el > bl; ++j) {   // clamped index: every load issues before any is used
            const int32_t i = i0 + j * SL_BLK;
            const int32_t col = (int32_t)(keys[min(i, el - 1)] / gyz);
            cl += i < el && col <= col_le;
            cr += i < el && col >= col_ge;
        }
    } else {
        const int32_t l0 = bl + blockIdx.x * SL_SEND + threadIdx.x, r0 = br + blockIdx.x * SL_SEND + threadIdx.x;
        // clamped indices: all 2 x SL_PER loads issue before any is used (conditional loads were one round trip
        // each: 10-17 us per launch at C3 x 4, profiles/r04_slab_trace.log)
        uint32_t kl[SL_PER], kr[SL_PER];
        const bool any_l = l0 - (int32_t)threadIdx.x < el, any_r = r0 - (int32_t)threadIdx.x < er;
#pragma unroll
        for (int j = 0; j < SL_PER; ++j) {
            kl[j] = any_l ? keys[min(l0 + j * SL_BLK, el - 1)] : 0u;
            kr[j] = any_r ? keys[min(r0 + j * SL_BLK, er - 1)] : 0u;
        }
#pragma unroll
        for (int j = 0; j < SL_PER; ++j) {
            cl += l0 + j * SL_BLK < el && (int32_t)(kl[j] / gyz) <= col_le;
            cr += r0 + j * SL_BLK < er && (int32_t)(kr[j] / gyz) >= col_ge;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        cl += (uint32_t)__shfl_xor((int)cl, o, 64);
        cr += (uint32_t)__shfl_xor((int)cr, o, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { wl[w] = cl; wr[w] = cr; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tl = 0, tr = 0;
#pragma unroll
        for (int k = 0; k < SL_WAVES; ++k) { tl += wl[k]; tr += wr[k]; }
        blk[blockIdx.x] = tl;
        blk[nblk + blockIdx.x] = tr;
    }
}

// one workgroup of 1024: exclusive scan of both count rows in place, totals[2] (u32), and the
// same totals as int64 into totals64 when given (the async send counts)
constexpr int SL_SCAN = 1024;

// Message header (MSG_HDR_F4 float4s): (count, capacity, 0, 0 | 0, 0, 0, 0) as uint32 bits.
__device__ __forceinline__ void write_header(float4* msg, uint32_t count, uint32_t cap) {
    msg[0] = make_float4(__uint_as_float(count), __uint_as_float(cap), 0.f, 0.f);
    msg[1] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// inplace 0: the totals only (the device-sized step's k_slab_pack2 takes the raw per-block counts)
__global__ __launch_bounds__(SL_SCAN) void k_slab_scan(uint32_t* __restrict__ blk, int32_t nblk,
                                                       uint32_t* __restrict__ totals, int64_t* __restrict__ totals64,
                                                       float4* __restrict__ hdr_l, float4* __restrict__ hdr_r,
                                                       int32_t cap_l, int32_t cap_r, int32_t inplace = 1) {
    __shared__ uint32_t ws[SL_SCAN / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int side = 0; side < 2; ++side) {
        uint32_t* row = blk + side * nblk;
        uint32_t carry = 0;
        for (int32_t base = 0; base < nblk; base += SL_SCAN) {
            const int32_t i = base + threadIdx.x;
            const uint32_t v = i < nblk ? row[i] : 0u;
            uint32_t inc = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(inc, o, 64);
                if (lane >= o) inc += t;
            }
            if (lane == 63) ws[w] = inc;
            __syncthreads();
            uint32_t pre = 0, tot = 0;
#pragma unroll
            for (int k = 0; k < SL_SCAN / 64; ++k) {
                pre += k < w ? ws[k] : 0u;
                tot += ws[k];
            }
            __syncthreads();
            if (i < nblk && inplace) row[i] = carry + pre + inc - v;
            carry += tot;
        }
        if (threadIdx.x == 0) {
            totals[side] = carry;
            if (totals64) totals64[side] = (int64_t)carry;
            float4* h = side == 0 ? hdr_l : hdr_r;
            if (h) write_header(h, carry, (uint32_t)(side == 0 ? cap_l : cap_r));
        }
    }
}

// A record is (x, y, z, id) (u, v, w, old key): the old key is the particle's sorted key before this
// step's drift, as a GLOBAL key (sender's local key + its window's first key), or SL_NO_KEY when
// the sender holds no valid sorted keys. The receiver's incremental re-sort uses it.
constexpr uint32_t SL_NO_KEY = 0xffffffffu;

// The compaction of one workgroup's SL_SEND slots [i0, ...) of [b, e) into records from `run` on (the side's
// exclusive prefix of the per-block counts). The sent slots are listed in LDS in record order first, and then every
// thread copies list entries: the record loads of all entries issue together (one round trip) instead of one
// dependent load-and-store round per sub-chunk (~20 us per pack launch at C3 x 4, profiles/r04_slab_trace.log).
__device__ __forceinline__ void pack_block(const uint32_t* __restrict__ keys, const float4* __restrict__ pos,
                                           const float4* __restrict__ vel, const int32_t* __restrict__ id,
                                           const uint32_t* __restrict__ sk, uint32_t key_base, int32_t b, int32_t e,
                                           uint32_t gyz, int32_t side, int32_t col_le, int32_t col_ge, uint32_t run,
                                           float4* __restrict__ out, uint32_t cap, uint32_t (*wc)[SL_WAVES],
                                           int32_t* list) {
    const int w = threadIdx.x >> 6;
    const int32_t i0 = b + blockIdx.x * SL_SEND + threadIdx.x;
    // every key load issues before any is used; then one barrier for all sub-chunks' wave counts
    uint32_t col[SL_PER];
#pragma unroll
    for (int j = 0; j < SL_PER; ++j) col[j] = keys[min(i0 + j * SL_BLK, e - 1)] / gyz;
    uint32_t mine = 0;   // bit j: the slot of sub-chunk j is sent
#pragma unroll
    for (int j = 0; j < SL_PER; ++j) {
        const bool pred = i0 + j * SL_BLK < e && (side == 0 ? (int32_t)col[j] <= col_le : (int32_t)col[j] >= col_ge);
        const uint64_t m = __ballot(pred);
        if ((threadIdx.x & 63) == 0) wc[j][w] = (uint32_t)__popcll(m);
        mine |= (uint32_t)pred << j;
    }
    __syncthreads();
    // sub-chunks in slot order, waves in order within a sub-chunk: the list keeps slot order
    uint32_t loc = 0;
#pragma unroll
    for (int j = 0; j < SL_PER; ++j) {
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < SL_WAVES; ++k) {
            before += k < w ? wc[j][k] : 0u;
            tot += wc[j][k];
        }
        const bool pred = (mine >> j) & 1u;
        const uint64_t m = __ballot(pred);
        if (pred) list[loc + before + lane_prefix(m)] = i0 + j * SL_BLK;
        loc += tot;
    }
    __syncthreads();
    // loc: the block's record count. Records past the message capacity are dropped; the header's count tells the
    // receiver.
    const uint32_t lim = run < cap ? min(loc, cap - run) : 0u;
    constexpr int U = 4;
    for (uint32_t t0 = threadIdx.x; t0 < lim; t0 += U * SL_BLK) {
        float4 p[U], v[U];
        int32_t q[U];
        uint32_t ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = t0 + u * SL_BLK;
            const int32_t i = list[min(t, lim - 1)];
            p[u] = pos[i];
            v[u] = vel[i];
            q[u] = id[i];
            ok[u] = sk ? sk[i] + key_base : SL_NO_KEY;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = t0 + u * SL_BLK;
            if (t < lim) {
                out[2 * (size_t)(run + t)] = make_float4(p[u].x, p[u].y, p[u].z, __int_as_float(q[u]));
                out[2 * (size_t)(run + t) + 1] = make_float4(v[u].x, v[u].y, v[u].z, __uint_as_float(ok[u]));
            }
        }
    }
}

__global__ __launch_bounds__(SL_BLK) void k_slab_pack(const uint32_t* __restrict__ keys,
                                                      const float4* __restrict__ pos,
                                                      const float4* __restrict__ vel,
                                                      const int32_t* __restrict__ id,
                                                      const uint32_t* __restrict__ sk, uint32_t key_base,
                                                      int32_t b, int32_t e, uint32_t gyz, int32_t side,
                                                      int32_t col_le, int32_t col_ge,
                                                      const uint32_t* __restrict__ blk, int32_t nblk,
                                                      float4* __restrict__ out, uint32_t cap) {
    __shared__ uint32_t wc[SL_PER][SL_WAVES];
    __shared__ int32_t list[SL_SEND];
    if (b + (int32_t)blockIdx.x * SL_SEND >= e) return;   // whole workgroup, before the barrier
    pack_block(keys, pos, vel, id, sk, key_base, b, e, gyz, side, col_le, col_ge, blk[side * nblk + blockIdx.x], out,
               cap, wc, list);
}

// The device-sized step's pack: both sides in one launch (blockIdx.y = side), straight from k_slab_count's
// per-block counts: each workgroup sums the counts of the blocks before it (at most a few hundred), and
// workgroup 0 of a side writes the side's total into the message header and into totals[side] (for
// k_slab_lag). No scan launch between count and pack.
struct PackOut {
    float4* msg[2];          // header + records; null: no neighbour on that side
    uint32_t cap[2];
    uint32_t* totals;
};
__global__ __launch_bounds__(SL_BLK) void k_slab_pack2(const uint32_t* __restrict__ keys, const float4* __restrict__ pos,
                                                       const float4* __restrict__ vel, const int32_t* __restrict__ id,
                                                       const uint32_t* __restrict__ sk, uint32_t key_base, uint32_t gyz,
                                                       int32_t col_le, int32_t col_ge, const uint32_t* __restrict__ blk,
                                                       int32_t nblk, const SlabSizes* __restrict__ dz, PackOut po,
                                                       int32_t cand, int32_t early) {
    __shared__ uint32_t wc[SL_PER][SL_WAVES];
    __shared__ uint32_t red[SL_WAVES][2];
    __shared__ int32_t list[SL_SEND];
    const int32_t side = (int32_t)blockIdx.y;
    float4* msg = po.msg[side];
    if (!msg) return;
    int32_t bl, el, br, er;
    send_ranges(dz, cand, bl, el, br, er, early);
    const int32_t b = side == 0 ? bl : br, e = side == 0 ? el : er;
    const bool work = b + (int32_t)blockIdx.x * SL_SEND < e;
    if (!work && blockIdx.x != 0) return;   // whole workgroup, before any barrier
    // this block's exclusive prefix (blocks < blockIdx.x) and, for block 0, the side's total
    const uint32_t* row = blk + side * nblk;
    uint32_t pre = 0, tot = 0;
    for (int32_t k = threadIdx.x; k < nblk; k += SL_BLK) {
        const uint32_t v = row[k];
        pre += k < (int32_t)blockIdx.x ? v : 0u;
        tot += v;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        pre += (uint32_t)__shfl_xor((int)pre, o, 64);
        tot += (uint32_t)__shfl_xor((int)tot, o, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[w][0] = pre; red[w][1] = tot; }
    __syncthreads();
    uint32_t run = 0, total = 0;
#pragma unroll
    for (int k = 0; k < SL_WAVES; ++k) { run += red[k][0]; total += red[k][1]; }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        write_header(msg, total, po.cap[side]);
        po.totals[side] = total;
    }
    if (!work) return;   // block 0 of an empty side: header only (the barrier above is behind it)
    pack_block(keys, pos, vel, id, sk, key_base, b, e, gyz, side, col_le, col_ge, run, msg + MSG_HDR_F4, po.cap[side],
               wc, list);
}

__global__ __launch_bounds__(SL_BLK) void k_slab_unpack(const float4* __restrict__ rec, int32_t n,
                                                        float4* __restrict__ pos, float4* __restrict__ vel,
                                                        int32_t* __restrict__ id) {
    const int32_t i = blockIdx.x * SL_BLK + threadIdx.x;
    if (i >= n) return;
    const float4 a = rec[2 * (size_t)i], v = rec[2 * (size_t)i + 1];
    pos[i] = make_float4(a.x, a.y, a.z, 0.f);
    vel[i] = make_float4(v.x, v.y, v.z, 0.f);
    id[i] = __float_as_int(a.w);
}

// The per-phase path's old cell-start table (common.h cs_old_block; the in-library step runs the same body inside
// k_slab_rec, reading the old keys from the messages).
__global__ __launch_bounds__(SL_BLK) void k_slab_cs_old(CsOld p, int32_t shift, const uint32_t* __restrict__ sk,
                                                        int32_t nl, int32_t no, int32_t nr,
                                                        const SlabSizes* __restrict__ dz) {
    __shared__ uint32_t samp[CS_SAMP];
    __shared__ uint32_t win[CS_WIN];
    if (dz) {
        nl = (int32_t)dz->nl;
        no = (int32_t)dz->no;
        nr = (int32_t)dz->nr;
        shift = nl - (int32_t)dz->o0;
    }
    const uint32_t rbase = (uint32_t)(nl + no);
    auto key = [&](int side, uint32_t t) { return sk[(side == 0 ? 0u : rbase) + t]; };
    cs_old_block(p, blockIdx.x, (uint32_t)nl, (uint32_t)no, (uint32_t)nr, shift, key, samp, win);
}

// ---- init-time selection of owned columns (global grid in `g`)
__global__ __launch_bounds__(SL_BLK) void k_sel_count(const float4* __restrict__ pos, int32_t n, GridDesc g,
                                                      int32_t lo, int32_t hi, uint32_t* __restrict__ blk) {
    __shared__ uint32_t wc[SL_WAVES];
    const int32_t i = blockIdx.x * SL_BLK + threadIdx.x;
    bool pred = false;
    if (i < n) {
        const int32_t c = cell_cx(g, pos[i].x);
        pred = c >= lo && c < hi;
    }
    uint32_t wb;
    const uint32_t t = block_ballot_count(pred, wc, wb);
    if (threadIdx.x == 0) blk[blockIdx.x] = t;
}

__global__ __launch_bounds__(SL_BLK) void k_sel_scatter(const float4* __restrict__ pos,
                                                        const float4* __restrict__ vel,
                                                        const int32_t* __restrict__ id, int32_t n, GridDesc g,
                                                        int32_t lo, int32_t hi, const uint32_t* __restrict__ blk,
                                                        float4* __restrict__ pos_o, float4* __restrict__ vel_o,
                                                        int32_t* __restrict__ id_o) {
    __shared__ uint32_t wc[SL_WAVES];
    const int32_t i = blockIdx.x * SL_BLK + threadIdx.x;
    bool pred = false;
    if (i < n) {
        const int32_t c = cell_cx(g, pos[i].x);
        pred = c >= lo && c < hi;
    }
    uint32_t wb;
    block_ballot_count(pred, wc, wb);
    if (!pred) return;
    const uint32_t r = blk[blockIdx.x] + wb + lane_prefix(__ballot(pred));
    pos_o[r] = pos[i];
    vel_o[r] = vel[i];
    id_o[r] = id[i];
}

struct Pick10 {
    int32_t idx[10];
};

// out: device copy (kernels read it); out_host (optional): mapped pinned host memory, written
// directly so no copy-back is queued (the host waits on an event after this kernel)
__global__ void k_pick(const uint32_t* __restrict__ cs, Pick10 p, int32_t m, uint32_t* __restrict__ out,
                       uint32_t* __restrict__ out_host) {
    const int t = threadIdx.x;
    if (t < m) {
        const uint32_t v = cs[p.idx[t]];
        out[t] = v;
        if (out_host) out_host[t] = v;
    }
}

__global__ __launch_bounds__(SL_BLK) void k_pack_owned(const float4* __restrict__ pos, const float4* __restrict__ vel,
                                                       const int32_t* __restrict__ id,
                                                       const float2* __restrict__ rp, int32_t o0, int32_t n,
                                                       float* __restrict__ out) {
    const int32_t i = blockIdx.x * SL_BLK + threadIdx.x;
    if (i >= n) return;
    const float4 p = pos[o0 + i], v = vel[o0 + i];
    float* q = out + 8 * (size_t)i;
    q[0] = p.x; q[1] = p.y; q[2] = p.z; q[3] = v.x; q[4] = v.y; q[5] = v.z;
    q[6] = __int_as_float(id[o0 + i]);
    q[7] = rp ? rp[o0 + i].x : 0.f;
}

// out[t] = cs at the start of local column c0 + t, t in [0, m)
__global__ __launch_bounds__(SL_BLK) void k_column_starts(const uint32_t* __restrict__ cs, uint32_t gyz, int32_t c0,
                                                          int32_t m, uint32_t* __restrict__ out) {
    const int32_t t = blockIdx.x * SL_BLK + threadIdx.x;
    if (t < m) out[t] = cs[(size_t)(c0 + t) * gyz];
}

void launch_column_starts(const uint32_t* cs, uint32_t gyz, int32_t c0, int32_t m, uint32_t* out, hipStream_t s) {
    if (m > 0) k_column_starts<<<(m + SL_BLK - 1) / SL_BLK, SL_BLK, 0, s>>>(cs, gyz, c0, m, out);
}

void launch_pick(const uint32_t* cs, const int32_t* idx, int32_t m, uint32_t* out, hipStream_t s,
                 uint32_t* out_host) {
    Pick10 p{};
    for (int k = 0; k < m && k < 10; ++k) p.idx[k] = idx[k];
    k_pick<<<1, 64, 0, s>>>(cs, p, m, out, out_host);
}

void launch_pack_owned(const float4* pos, const float4* vel, const int32_t* id, const float2* rp, int32_t o0,
                       int32_t n, float* out, hipStream_t s) {
    if (n > 0) k_pack_owned<<<(n + SL_BLK - 1) / SL_BLK, SL_BLK, 0, s>>>(pos, vel, id, rp, o0, n, out);
}

void launch_slab_count(const uint32_t* keys, int32_t b, int32_t e, uint32_t gyz, int32_t col_le, int32_t col_ge,
                       uint32_t* blk, uint32_t* totals, hipStream_t s, int64_t* totals64) {
    const int32_t nb = slab_send_blocks(b, e);
    k_slab_count<<<nb, SL_BLK, 0, s>>>(keys, b, e, gyz, col_le, col_ge, blk, nb, nullptr, 0, 0);
    k_slab_scan<<<1, SL_SCAN, 0, s>>>(blk, nb, totals, totals64, nullptr, nullptr, 0, 0);
}

void launch_slab_pack(const uint32_t* keys, const float4* pos, const float4* vel, const int32_t* id,
                      const uint32_t* sk, uint32_t key_base, int32_t b, int32_t e, uint32_t gyz, int32_t side,
                      int32_t col_le, int32_t col_ge, const uint32_t* blk, float4* out, hipStream_t s) {
    const int32_t nb = slab_send_blocks(b, e);
    if (e > b)
        k_slab_pack<<<nb, SL_BLK, 0, s>>>(keys, pos, vel, id, sk, key_base, b, e, gyz, side, col_le, col_ge, blk, nb,
                                          out, 0xffffffffu);
}

// exact: the host reads the totals before packing (k_slab_scan, totals only); steady steps need no scan
void launch_slab_count_dev(const uint32_t* keys, const SlabSizes* dz, int32_t nb_ub, uint32_t gyz, int32_t col_le,
                           int32_t col_ge, uint32_t* blk, uint32_t* totals, hipStream_t s, bool cand, bool exact,
                           bool early) {
    k_slab_count<<<nb_ub, SL_BLK, 0, s>>>(keys, 0, 0, gyz, col_le, col_ge, blk, nb_ub, dz, cand ? 1 : 0, early ? 1 : 0);
    if (exact) k_slab_scan<<<1, SL_SCAN, 0, s>>>(blk, nb_ub, totals, nullptr, nullptr, nullptr, 0, 0, 0);
}

void launch_slab_pack2_dev(const uint32_t* keys, const float4* pos, const float4* vel, const int32_t* id,
                           const uint32_t* sk, uint32_t key_base, const SlabSizes* dz, int32_t nb_ub, uint32_t gyz,
                           int32_t col_le, int32_t col_ge, const uint32_t* blk, float4* msg_l, int32_t cap_l,
                           float4* msg_r, int32_t cap_r, uint32_t* totals, hipStream_t s, bool cand, bool early) {
    if (!msg_l && !msg_r) return;
    const PackOut po{{msg_l, msg_r}, {(uint32_t)cap_l, (uint32_t)cap_r}, totals};
    k_slab_pack2<<<dim3(nb_ub, 2), SL_BLK, 0, s>>>(keys, pos, vel, id, sk, key_base, gyz, col_le, col_ge, blk, nb_ub, dz,
                                                   po, cand ? 1 : 0, early ? 1 : 0);
}

// The assembled layout from the message headers and the owned range of the previous order (a
// host-sized step; device-sized steps compute it in k_slab_rec).
__global__ void k_slab_sizes(SlabSizes* __restrict__ dz, SizesIn in) {
    if (threadIdx.x != 0) return;
    uint32_t nl, no, nr, f, hl, hr;
    slab_sizes_from(dz, in, nl, no, nr, f, hl, hr);
    slab_sizes_store(dz, nl, no, nr, f, hl, hr);
}

void launch_slab_sizes(SlabSizes* dz, const float4* msg_l, const float4* msg_r, int32_t cap_l, int32_t cap_r,
                       int32_t capacity, hipStream_t s) {
    SPH_LAUNCH(k_slab_sizes, 1, 64, 0, s, dz, SizesIn{msg_l, msg_r, cap_l, cap_r, capacity});
}

// ρ messages (common.h RHO_HDR): the per-phase ABI packs them here; the in-library step's density pass
// writes them itself (RhoOut)
// both sides in one launch (blockIdx.y = side; a side without a message has no workgroups' work)
__global__ __launch_bounds__(SL_BLK) void k_slab_pack_rho2(const float2* __restrict__ rp, const SlabSizes* __restrict__ dz,
                                                           float2* __restrict__ msg_l, int32_t cap_l,
                                                           float2* __restrict__ msg_r, int32_t cap_r) {
    const int32_t side = (int32_t)blockIdx.y;
    float2* msg = side == 0 ? msg_l : msg_r;
    const int32_t cap = side == 0 ? cap_l : cap_r;
    if (!msg || (int32_t)(blockIdx.x * SL_BLK) > cap) return;
    const uint32_t b = dz->pick[1 + 2 * side], e = dz->pick[2 + 2 * side];
    const uint32_t cnt = e - b;
    const uint32_t t = blockIdx.x * SL_BLK + threadIdx.x;
    if (t == 0) {
        msg[0] = make_float2(__uint_as_float(cnt), __uint_as_float((uint32_t)cap));
        msg[1] = msg[2] = msg[3] = make_float2(0.f, 0.f);
    }
    if (t < cnt && t < (uint32_t)cap) msg[RHO_HDR + t] = rp[b + t];
}

__global__ __launch_bounds__(SL_BLK) void k_slab_unpack_rho2(float2* __restrict__ rp, SlabSizes* __restrict__ dz,
                                                             const float2* __restrict__ msg_l, int32_t cap_l,
                                                             const float2* __restrict__ msg_r, int32_t cap_r) {
    const int32_t side = (int32_t)blockIdx.y;
    const float2* msg = side == 0 ? msg_l : msg_r;
    const int32_t cap = side == 0 ? cap_l : cap_r;
    if (!msg || (int32_t)(blockIdx.x * SL_BLK) > cap) return;
    const uint32_t b = dz->pick[4 * side], e = dz->pick[4 * side + 1];
    const uint32_t cnt = __float_as_uint(msg[0].x);
    const uint32_t m = min(min(cnt, (uint32_t)cap), e - b);
    const uint32_t t = blockIdx.x * SL_BLK + threadIdx.x;
    if (t == 0 && (cnt != e - b || cnt > (uint32_t)cap)) atomicOr(&dz->flags, SZ_RHO_MISMATCH);
    if (t < m) rp[b + t] = msg[RHO_HDR + t];
}

void launch_slab_pack_rho2(const float2* rp, SlabSizes* dz, float2* msg_l, int32_t cap_l, float2* msg_r, int32_t cap_r,
                           hipStream_t s) {
    if (!msg_l && !msg_r) return;
    const int32_t cl = msg_l ? cap_l : 0, cr = msg_r ? cap_r : 0, cap = cl > cr ? cl : cr;
    k_slab_pack_rho2<<<dim3(cap / SL_BLK + 1, 2), SL_BLK, 0, s>>>(rp, dz, msg_l, cap_l, msg_r, cap_r);
}

void launch_slab_unpack_rho2(float2* rp, SlabSizes* dz, const float2* msg_l, int32_t cap_l, const float2* msg_r,
                             int32_t cap_r, hipStream_t s) {
    if (!msg_l && !msg_r) return;
    const int32_t cl = msg_l ? cap_l : 0, cr = msg_r ? cap_r : 0, cap = cl > cr ? cl : cr;
    k_slab_unpack_rho2<<<dim3(cap / SL_BLK + 1, 2), SL_BLK, 0, s>>>(rp, dz, msg_l, cap_l, msg_r, cap_r);
}

// End of a device-sized step: the slot ranges of the new order from the picked column starts (the
// kernels of this step read the picks themselves; these copies are for the host and the next step),
// the next step's owned range, the sizes of a rank without neighbours (no message will set them), and
// this step's counts for the capacities two steps on (mapped pinned memory).
// out[2], out[3]: the header counts of this step's received messages as the record kernel saw them (the message
// buffers may hold the next step's early messages by now); out[10], out[11]: the two columns at each side (the early
// boundary pass's ranges), for the next grids.
__global__ void k_slab_lag(SlabSizes* __restrict__ dz, int32_t has_left, int32_t has_right,
                           const uint32_t* __restrict__ totals, const float2* __restrict__ rho_in_l,
                           const float2* __restrict__ rho_in_r, const uint32_t* __restrict__ gflags,
                           uint32_t* __restrict__ out, uint32_t* __restrict__ zero, int32_t nzero) {
    for (int32_t t = (int32_t)threadIdx.x; t < nzero; t += (int32_t)blockDim.x) zero[t] = 0u;
    if (threadIdx.x != 0) return;
    const uint32_t* v = dz->pick;
    const uint32_t rg[10] = {v[0], v[1], v[1], v[4], v[4], v[5], v[1], v[2], v[3], v[4]};
    for (int k = 0; k < 10; ++k) dz->rg[k] = rg[k];
    const uint32_t ib = has_left ? v[2] : v[1], ie = has_right ? v[3] : v[4];
    dz->fr[0] = ib;
    dz->fr[1] = ie > ib ? ie : ib;
    if (ie < ib) {   // one-column slab: both boundary columns are the owned column
        dz->fr[2] = v[1]; dz->fr[3] = v[4]; dz->fr[4] = 0u; dz->fr[5] = 0u;
    } else {
        dz->fr[2] = v[1]; dz->fr[3] = ib; dz->fr[4] = ie; dz->fr[5] = v[4];
    }
    dz->dropped = dz->n - v[5];
    dz->o0 = v[1];
    dz->o1 = v[4];
    const uint32_t f = dz->flags;
    if (!has_left && !has_right) {   // the next step's layout: the owned slots alone
        dz->nl = dz->nr = 0u;
        dz->no = v[4] - v[1];
        dz->n = v[4] - v[1];
    } else {
        dz->n = v[5];
    }
    out[0] = totals[0];
    out[1] = totals[1];
    out[2] = has_left ? dz->hl_raw : 0u;
    out[3] = has_right ? dz->hr_raw : 0u;
    out[4] = v[2] - v[1];
    out[5] = v[4] - v[3];
    out[6] = rho_in_l ? __float_as_uint(rho_in_l[0].x) : 0u;
    out[7] = rho_in_r ? __float_as_uint(rho_in_r[0].x) : 0u;
    out[8] = v[5];
    uint32_t gf = f;
    if (gflags) {   // RCCL: one word per flag bit, max-reduced over the ranks: the OR (the same on all ranks)
        gf = 0u;
        for (int k = 0; k < SZ_BITS; ++k) gf |= (gflags[k] != 0u ? 1u : 0u) << k;
    }
    out[9] = gf;
    out[10] = v[6] - v[1];
    out[11] = v[4] - v[7];
}

void launch_slab_lag(SlabSizes* dz, int32_t has_left, int32_t has_right, const uint32_t* totals,
                     const float2* rho_in_l, const float2* rho_in_r, const uint32_t* gflags, uint32_t* out,
                     hipStream_t s, uint32_t* zero, int32_t nzero) {
    k_slab_lag<<<1, 256, 0, s>>>(dz, has_left, has_right, totals, rho_in_l, rho_in_r, gflags, out, zero,
                                 zero ? nzero : 0);
}

void launch_slab_unpack(const float4* rec, int32_t n, float4* pos, float4* vel, int32_t* id, hipStream_t s) {
    if (n > 0) k_slab_unpack<<<(n + SL_BLK - 1) / SL_BLK, SL_BLK, 0, s>>>(rec, n, pos, vel, id);
}

void launch_slab_cs_old(uint32_t* cs, uint32_t ncells, uint32_t gyz, uint32_t gx, bool has_left, bool has_right,
                        int32_t shift, const uint32_t* sk, int32_t nl, int32_t no, int32_t nr, hipStream_t s,
                        const SlabSizes* dz) {
    CsOld p;
    p.cs = cs;
    p.ncells = ncells;
    p.gyz = gyz;
    p.gx = gx;
    p.has_left = has_left ? 1 : 0;
    p.has_right = has_right ? 1 : 0;
    SPH_LAUNCH(k_slab_cs_old, cs_old_blocks(ncells, SL_BLK), SL_BLK, 0, s, p, shift, sk, nl, no, nr, dz);
}

void launch_slab_select_columns(const float4* pos, const float4* vel, const int32_t* id, int32_t n, GridDesc g,
                                int32_t lo, int32_t hi, uint32_t* blk, uint32_t* total, float4* pos_o,
                                float4* vel_o, int32_t* id_o, hipStream_t s) {
    const int32_t nb = slab_compact_blocks(0, n);
    k_sel_count<<<nb, SL_BLK, 0, s>>>(pos, n, g, lo, hi, blk);
    // reuse the two-row scan: row 1 is a dummy of zeros
    (void)hipMemsetAsync(blk + nb, 0, sizeof(uint32_t) * nb, s);
    k_slab_scan<<<1, SL_SCAN, 0, s>>>(blk, nb, total, nullptr, nullptr, nullptr, 0, 0);
    if (n > 0 && pos_o != nullptr) k_sel_scatter<<<nb, SL_BLK, 0, s>>>(pos, vel, id, n, g, lo, hi, blk, pos_o, vel_o, id_o);
}

}  // namespace sph
