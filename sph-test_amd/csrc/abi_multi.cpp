// abi_multi.cpp — the decomposed Model S step inside the library (SPEC_SPH.md §3).
//
// The reference has one GPU and one host thread (ParticleSystemController.cs:244-351, InitializeBuffers
// :373-451). Here one sph_step drives an x-slab decomposition over several GPUs, in two forms:
//   * sph_config.ndev > 1: one context in one process owns a slab context per GPU (a "local group");
//     the halos move by device-to-device copies (hipMemcpyPeerAsync: xGMI between GPUs, a plain copy
//     when two slabs share a device, as on a one-GPU test box);
//   * sph_comm_init: one context per process (one process per GPU, as torchrun launches), the halos
//     move over RCCL (ncclSend / ncclRecv in one group per exchange, so both neighbours at once).
// Both run the same per-rank phases (the kernels of the per-phase ABI in abi_slab.cpp), phase-major
// over the ranks this process drives:
//   A  send counts + packing of migrants / x,v halo into capacity-sized messages (header = count)
//   X1 exchange 1
//   B  sizes from the headers → incremental re-sort over [left | own | right] (device sizes), or the
//      full radix sort (after a re-cut: a host-sized step) → ranges → density → ρ of the boundary columns
//   X2 exchange 2 on the comm stream, in flight while the interior columns' force pass runs
//   C  ghost densities in → boundary columns' force pass → finish
// No host read happens in a steady-state step. Message capacities come from the counts of two steps
// before (a kernel writes them to mapped pinned memory; both neighbours read the same numbers, so they
// agree on every message size), with a margin far above what particles moving < 0.1 h per step can add.
// A larger count is caught on the device (SZ_* flags) and the next sph_step fails with SPH_ERR_CAPACITY.
// The first three steps after the initial cut and after every re-cut size the messages exactly (a count
// exchange and one host read per exchange): the lagged counts would describe the old cut's columns, or
// the one-off migration exchange of the first step after the re-cut.
#include "host.h"

#include <rccl/rccl.h>

#include <chrono>
#include <cmath>

namespace sph {

constexpr int LAG_SLOTS = 4;
constexpr int LAG_WORDS = 16;
constexpr int SDEV_TOTALS = 10;   // sdev[10..13]: send counts, two slots by step parity (sdev[0..7] picks, [8..9] gaps)
// The send counts of step `step` (the early sends of step s + 1 are packed while step s's bookkeeping still reads
// step s's counts, so the two live in different slots).
uint32_t* totals_slot(sph_ctx* c, int64_t step) { return c->sdev + SDEV_TOTALS + 2 * (int)(step & 1); }

struct RankState {
    sph_ctx* c = nullptr;
    int rank = 0, world = 1, left = -1, right = -1;
    hipStream_t comm = nullptr;                       // exchange 2 (overlaps the interior force pass)
    hipEvent_t ev_packed = nullptr, ev_in = nullptr;  // exchange 1: messages packed / received
    hipEvent_t ev_rho_packed = nullptr, ev_rho_recv = nullptr;
    hipEvent_t ev_bdone = nullptr;   // the boundary force pass (comm stream) is done: the step's end waits on it
    hipEvent_t ev_sent = nullptr;    // early sends: the next step's messages have arrived (comm stream)
    hipEvent_t ev_fdone = nullptr;   // early sends without the jump guard: the interior force pass is done
    int32_t e_c1o[2] = {0, 0}, e_c1i[2] = {0, 0};   // the next step's message capacities (early sends)
    bool comm_borrowed = false;      // SPH_DEBUG_SERIAL_GROUP: slab 0's comm stream
    bool sent_pending = false;       // ev_sent closes comm-stream work the main stream has not waited for yet
    uint32_t* ebins = nullptr;       // early sends: the boundary pass's send counts (SendBins), 2 x ebin_cap words
    int32_t ebin_cap = 0;
    bool ebins_used = false;         // this step's boundary pass counted into ebins (k_slab_lag clears them)
    uint32_t* cs_alt = nullptr;      // pre-issued records: the next step's old cell-start table, built beside ctx->cs
    uint32_t cs_alt_cap = 0;
    bool pre_rec = false;            // the next step's k_slab_rec ran at the end of this step (comm stream)
    int32_t g2[2] = {0, 0};          // grid bounds of the two-column boundary ranges (early sends), 0: n_ub
    SlabSizes* dz = nullptr;
    float4* msg_out[2] = {nullptr, nullptr};
    float4* msg_in[2] = {nullptr, nullptr};
    int32_t mcap_out[2] = {0, 0}, mcap_in[2] = {0, 0};   // allocated records
    float2* rho_out[2] = {nullptr, nullptr};
    float2* rho_in[2] = {nullptr, nullptr};
    int32_t rcap_out[2] = {0, 0}, rcap_in[2] = {0, 0};
    int32_t c1o[2] = {0, 0}, c1i[2] = {0, 0}, c2o[2] = {0, 0}, c2i[2] = {0, 0};   // this step's capacities
    uint32_t* cnt_dev = nullptr;   // [12] received counts [0, 2) (exact-size steps over RCCL); [4, 9): one word per
                                   // SZ_* bit, written by the density pass and max-reduced over the ranks (an OR);
                                   // SZ_* flags, max-reduced over the communicator each step (RCCL, world > 1)
    uint32_t* lag = nullptr;       // pinned, mapped: LAG_SLOTS x LAG_WORDS (launch_slab_lag)
    hipEvent_t lag_ev[LAG_SLOTS] = {};
    int64_t cin_hist[LAG_SLOTS] = {};   // Σ records received per step (slot bound bookkeeping)
    int64_t since_cut = 0;              // steps since the initial cut or the last re-cut
    bool jump_guard = false;            // the last force pass ran the column-jump guard (it needs the sorted old
                                        // keys: incremental re-sort on); without it the sends scan every own slot
    int64_t n_prev_ub = 0;              // upper bound of the previous step's assembled slots
    int64_t n_ub = 0;                   // this step's
    int32_t nb_send = 1;                // count / pack blocks of this step
};

struct Multi {
    int mode = 0;                    // 1: local group (ndev), 2: RCCL
    std::vector<sph_ctx*> kids;      // local group: one slab context per GPU (owned)
    std::vector<RankState> ranks;    // the ranks this process drives
    int world = 1;
    ncclComm_t comm = nullptr;
    int64_t* hist_dev = nullptr;     // RCCL: the re-balancing histogram
    int32_t hist_cap = 0;
    int rebalance_every = 50;
    int rebalances = 0;
    std::vector<sph_slab> cuts;      // every rank's owned columns
    int64_t n_total = 0;
    bool ready = false;
    int64_t steps = 0;
    bool early = false;              // this step's messages were packed and exchanged during the previous step
    int hold_early = 0;              // steps to run without early sends (after a host-side state change)
    // switches every rank must agree on (they decide the exchange sequence and the message sizes): read from the
    // environment once per scenario and, over RCCL, max-reduced over the ranks (agree_switches)
    bool no_early = false;           // SPH_NO_EARLY_SENDS
    int32_t msg_cap = 0;             // SPH_DEBUG_MSG_CAP (tests): > 0 caps every lag-sized message
};

namespace {

#define NCCLCHK(call)                                                                                  \
    do {                                                                                               \
        ncclResult_t r_ = (call);                                                                      \
        if (r_ != ncclSuccess) return fail(ctx, SPH_ERR_HIP, "%s: %s", #call, ncclGetErrorString(r_)); \
    } while (0)

int32_t cap_of(const Multi& M, uint32_t cnt) {
    // the count two or three steps ago + 25% + 512 (a one-column halo changes by far less in three steps), whole 256s
    const int64_t c = (int64_t)cnt + cnt / 4 + 512;
    // SPH_DEBUG_MSG_CAP (tests only): cap every lag-sized message, to force the overflow path
    if (M.msg_cap > 0) return M.msg_cap;
    return (int32_t)std::min<int64_t>((c + 255) / 256 * 256, INT32_MAX / 4);
}

// Neighbouring slabs of a local group on different GPUs copy halos device to device: enable peer
// access both ways so the copies go GPU to GPU over xGMI. A pair without a peer path still works
// (hipMemcpyPeerAsync stages such a copy through host memory) but slowly: it is reported on stderr once
// per pair, not made an error (supported configurations).
int enable_peers(sph_ctx* ctx, int da, int db) {
    if (da == db) return SPH_OK;
    for (int k = 0; k < 2; ++k) {
        const int from = k ? db : da, to = k ? da : db;
        int can = 0;
        HIPCHK(hipDeviceCanAccessPeer(&can, from, to));
        if (!can) {
            std::fprintf(stderr, "sphhip: device %d cannot access device %d: the slab halo copies between them are "
                                 "staged through host memory (slow)\n", from, to);
            continue;
        }
        HIPCHK(hipSetDevice(from));
        const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
            return fail(ctx, SPH_ERR_HIP, "hipDeviceEnablePeerAccess(%d -> %d): %s", from, to, hipGetErrorString(e));
        (void)hipGetLastError();   // clear an "already enabled"
    }
    HIPCHK(hipSetDevice(ctx->device));
    return SPH_OK;
}

int global_columns(const sph_params& p) {
    const float cell = 2.0f * p.h;
    return (int)floorf(p.box[0] / cell) + 1;
}

// Lattice x-indices per global column of a scenario (jitter ignored; slab.py balanced_cuts). Times
// ny·nz: the initial particles per column.
std::vector<int64_t> lattice_columns(const sph_scenario& sc, const sph_params& p) {
    const float cell = 2.0f * p.h, inv = 1.0f / cell;
    const int G = global_columns(p);
    std::vector<int64_t> per(G, 0);
    for (int i = 0; i < sc.nx; ++i) {
        const float x = ((float)i + 0.5f) * sc.dx;
        int c = (int)floorf(x * inv);
        c = std::min(std::max(c, 0), G - 1);
        per[c] += 1;
    }
    return per;
}

// Equal-count cuts (slab.py balanced_cuts): cut r at the first column whose cumulative count reaches r/world.
std::vector<sph_slab> balanced_cuts(const std::vector<int64_t>& per, int world) {
    const int G = (int)per.size();
    std::vector<double> cum(G);
    double t = 0;
    for (int c = 0; c < G; ++c) cum[c] = (t += (double)per[c]);
    std::vector<int> b{0};
    for (int r = 1; r < world; ++r) {
        const double target = t * r / world;
        int c = (int)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin()) + 1;
        c = std::max(c, b.back() + 1);
        c = std::min(c, G - (world - r));
        b.push_back(c);
    }
    b.push_back(G);
    std::vector<sph_slab> out(world);
    for (int r = 0; r < world; ++r) out[r] = sph_slab{b[r], b[r + 1]};
    return out;
}

// slab.py rebalance_cuts: every inner cut moves at most one column toward equal counts; moves that
// would leave a slab narrower than two columns are dropped. A pure function: every rank agrees.
std::vector<sph_slab> rebalance_cuts(const std::vector<sph_slab>& cuts, const std::vector<int64_t>& hist) {
    const int world = (int)cuts.size();
    std::vector<int> b, nb;
    for (auto& c : cuts) b.push_back(c.cx_lo);
    b.push_back(cuts.back().cx_hi);
    nb = b;
    std::vector<double> cum(hist.size());
    double t = 0;
    for (size_t c = 0; c < hist.size(); ++c) cum[c] = (t += (double)hist[c]);
    if (t > 0)
        for (int r = 1; r < world; ++r) {
            const int ideal = (int)(std::lower_bound(cum.begin(), cum.end(), t * r / world) - cum.begin()) + 1;
            nb[r] = b[r] + std::max(-1, std::min(1, ideal - b[r]));
        }
    for (bool changed = true; changed;) {
        changed = false;
        for (int r = 1; r < world; ++r)
            if (nb[r] != b[r] && (nb[r] - nb[r - 1] < 2 || nb[r + 1] - nb[r] < 2)) {
                nb[r] = b[r];
                changed = true;
            }
    }
    std::vector<sph_slab> out(world);
    for (int r = 0; r < world; ++r) out[r] = sph_slab{nb[r], nb[r + 1]};
    return out;
}

// Every stream of the ranks this process drives: a message buffer is about to be reallocated and a
// neighbour's copy may still read it (rare: capacities only grow).
int sync_all(Multi& M, sph_ctx* ctx) {
    for (auto& R : M.ranks) {
        if (!R.c) continue;
        HIPCHK(hipSetDevice(R.c->device));
        HIPCHK(hipStreamSynchronize(R.c->stream));
        if (R.comm) HIPCHK(hipStreamSynchronize(R.comm));
    }
    HIPCHK(hipSetDevice(ctx->device));
    return SPH_OK;
}

template <class T>
int ensure_buf(Multi& M, sph_ctx* ctx, T** p, int32_t* cap, int32_t need) {
    if (need <= *cap && *p) return SPH_OK;
    int r = sync_all(M, ctx);
    if (r != SPH_OK) return r;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    const int32_t n = std::max(need + need / 2, 4096);
    HIPCHK(hipMalloc((void**)p, (size_t)n * sizeof(T)));
    *cap = n;
    return SPH_OK;
}

// a switch in the environment: set and not "0"
bool env_on(const char* name) {
    const char* v = std::getenv(name);
    return v && *v && std::atoi(v) != 0;
}

// the early sends' count bins (SendBins): both sides' send blocks, zeroed; allocated once per slot capacity
int ensure_ebins(Multi& M, RankState& R, int32_t nb) {
    if (nb <= R.ebin_cap && R.ebins) return SPH_OK;
    sph_ctx* ctx = R.c;
    int r = sync_all(M, ctx);
    if (r != SPH_OK) return r;
    dfree(R.ebins);
    const int32_t cap = std::max(nb, slab_send_blocks(0, std::max(ctx->capacity, 1)));
    HIPCHK(hipMalloc((void**)&R.ebins, 2 * (size_t)cap * sizeof(uint32_t)));
    HIPCHK(hipMemset(R.ebins, 0, 2 * (size_t)cap * sizeof(uint32_t)));
    HIPCHK(hipDeviceSynchronize());
    R.ebin_cap = cap;
    return SPH_OK;
}

int rank_init(RankState& R) {
    sph_ctx* ctx = R.c;
    HIPCHK(hipSetDevice(ctx->device));
    // the comm stream's work (ρ halo, boundary force pass, the next step's sends) must end under the interior
    // pass: at the device's highest stream priority its workgroups dispatch ahead of the interior pass's pending
    // ones. Serialised C3 x 2 / x 4 (profiles/r04_comm_priority_ab.log): the comm work's slack under the interior
    // passes 43 -> 55 / 39 -> 84 us. SPH_COMM_PRIORITY=0: normal priority
    int prio_least = 0, prio_greatest = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
    const char* pe = std::getenv("SPH_COMM_PRIORITY");
    if (pe && std::atoi(pe) == 0)
        HIPCHK(hipStreamCreateWithFlags(&R.comm, hipStreamNonBlocking));
    else
        HIPCHK(hipStreamCreateWithPriority(&R.comm, hipStreamNonBlocking, prio_greatest));
    for (hipEvent_t* e : {&R.ev_packed, &R.ev_in, &R.ev_rho_packed, &R.ev_rho_recv, &R.ev_bdone, &R.ev_sent, &R.ev_fdone})
        HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    for (auto& e : R.lag_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipMalloc((void**)&R.dz, sizeof(SlabSizes)));
    HIPCHK(hipMemset(R.dz, 0, sizeof(SlabSizes)));
    R.c->dz = R.dz;
    HIPCHK(hipMalloc((void**)&R.cnt_dev, 12 * sizeof(uint32_t)));
    HIPCHK(hipMemset(R.cnt_dev, 0, 12 * sizeof(uint32_t)));
    HIPCHK(hipMemset(R.c->sdev + SDEV_TOTALS, 0, 4 * sizeof(uint32_t)));
    HIPCHK(hipHostMalloc((void**)&R.lag, LAG_SLOTS * LAG_WORDS * sizeof(uint32_t), hipHostMallocMapped));
    std::memset(R.lag, 0, LAG_SLOTS * LAG_WORDS * sizeof(uint32_t));
    return SPH_OK;
}

void rank_free(RankState& R) {
    if (!R.c) return;
    (void)hipSetDevice(R.c->device);
    if (R.comm) (void)hipStreamSynchronize(R.comm);
    for (hipEvent_t e : {R.ev_packed, R.ev_in, R.ev_rho_packed, R.ev_rho_recv, R.ev_bdone, R.ev_sent, R.ev_fdone})
        if (e) (void)hipEventDestroy(e);
    for (auto e : R.lag_ev)
        if (e) (void)hipEventDestroy(e);
    for (int s = 0; s < 2; ++s) {
        dfree(R.msg_out[s]); dfree(R.msg_in[s]); dfree(R.rho_out[s]); dfree(R.rho_in[s]);
    }
    R.c->dz = nullptr;
    R.c->dz_ahead = false;
    dfree(R.dz);
    dfree(R.cnt_dev);
    dfree(R.ebins);
    dfree(R.cs_alt);
    if (R.lag) (void)hipHostFree(R.lag);
    if (R.comm && !R.comm_borrowed) (void)hipStreamDestroy(R.comm);
    R = RankState{};
}

// The host copies of the slab ranges from the device sizes (after device-sized steps), with one wait.
int sync_dz(RankState& R) {
    sph_ctx* ctx = R.c;
    ctx->dz_ahead = true;
    int r = slab_sync_ranges(ctx);
    if (r != SPH_OK) return r;
    R.n_prev_ub = ctx->n;
    return SPH_OK;
}

// device sizes from the host's (after init or a host-sized step's bookkeeping)
int put_dz(RankState& R) {
    sph_ctx* ctx = R.c;
    SlabSizes h{};
    HIPCHK(hipMemcpy(&h, R.dz, sizeof h, hipMemcpyDeviceToHost));
    h.o0 = (uint32_t)ctx->o0;
    h.o1 = (uint32_t)ctx->o1;
    h.no = h.o1 - h.o0;
    h.n = (uint32_t)ctx->n;
    HIPCHK(hipMemcpy(R.dz, &h, sizeof h, hipMemcpyHostToDevice));
    R.n_prev_ub = ctx->n;
    return SPH_OK;
}

int col_le(const sph_ctx* c) { return c->has_left ? c->sl.cx_lo - c->grid.cx0 : -1; }
int col_ge(const sph_ctx* c) { return c->has_right ? c->sl.cx_hi - 1 - c->grid.cx0 : 0x7fffffff; }
uint32_t gyz(const sph_ctx* c) { return col_keys(c->grid); }

// SPH_HOST_TIMING=1 (measurement): host time per step in multi_one_step and the part of it spent blocked on lag
// events, printed when the context is destroyed (the issue rate a rank's host sustains against its GPU)
struct HostTiming {
    bool on = std::getenv("SPH_HOST_TIMING") != nullptr;
    double total = 0.0, wait = 0.0;
    int64_t steps = 0;
};
HostTiming g_ht;
double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

const uint32_t* lag_slot(RankState& R, int64_t step, sph_ctx* ctx, int* rc) {
    const int k = (int)(step % LAG_SLOTS);
    const double t0 = g_ht.on ? now_s() : 0.0;
    // waits for the step's comm work: at a step's start for the step two back (done unless the host runs more than a
    // step ahead), in an early-send boundary phase for the previous step
    const hipError_t e = hipEventSynchronize(R.lag_ev[k]);
    if (g_ht.on) g_ht.wait += now_s() - t0;
    if (e != hipSuccess) *rc = fail(ctx, SPH_ERR_HIP, "lag event: %s", hipGetErrorString(e));
    return R.lag + k * LAG_WORDS;
}

// SPH_FLAG_VALIDATE: wait for the rank's streams after a launch group and name it in the error
int checkpoint(RankState& R, const char* what) {
    sph_ctx* ctx = R.c;
    if (!(ctx->cfg.flags & SPH_FLAG_VALIDATE)) return SPH_OK;
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess && R.comm) e = hipStreamSynchronize(R.comm);
    if (e != hipSuccess) return fail(ctx, SPH_ERR_HIP, "rank %d, %s: %s", R.rank, what, hipGetErrorString(e));
    return SPH_OK;
}
#define CKPT(R, what) \
    do { if (int rc_ = checkpoint(R, what)) return rc_; } while (0)

// SPH_FLAG_VALIDATE, before the incremental re-sort: the mover lists and the old cell starts it reads
int validate_movers(RankState& R, int used) {
    sph_ctx* ctx = R.c;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    SlabSizes h;
    HIPCHK(hipMemcpy(&h, R.dz, sizeof h, hipMemcpyDeviceToHost));
    uint32_t m = 0;
    HIPCHK(hipMemcpy(&m, ctx->mv_count + used, 4, hipMemcpyDeviceToHost));
    const uint32_t cap = (uint32_t)ctx->capacity, ncells = ctx->grid.ncells;
    if (m > cap) return fail(ctx, SPH_ERR_STATE, "validate(movers) rank %d: %u movers > cap %u", R.rank, m, cap);
    std::vector<uint32_t> mi(m), mk(m), mo(m), cs(ncells + 2);
    if (m) {
        HIPCHK(hipMemcpy(mi.data(), ctx->mv_mi, m * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(mk.data(), ctx->mv_mk, m * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(mo.data(), ctx->mv_mo, m * 4, hipMemcpyDeviceToHost));
    }
    HIPCHK(hipMemcpy(cs.data(), ctx->cs, cs.size() * 4, hipMemcpyDeviceToHost));
    const int64_t mi_off = (int64_t)h.nl - (int64_t)h.o0;
    struct Ent { uint32_t slot, mo, r; bool operator<(const Ent& o) const { return slot < o.slot; } };
    std::vector<Ent> by_slot;
    for (uint32_t r = 0; r < m; ++r) {
        const int64_t x = (mi[r] & MV_REC) ? (int64_t)(mi[r] & ~MV_REC) : (int64_t)mi[r] + mi_off;
        const bool rec = (mi[r] & MV_REC) != 0;
        const bool slot_ok = x >= 0 && x < (int64_t)h.n && (rec ? (x < h.nl || x >= h.nl + h.no) : (x >= h.nl && x < h.nl + h.no));
        if (!slot_ok || mk[r] > ncells || mo[r] > ncells)
            return fail(ctx, SPH_ERR_STATE,
                        "validate(movers) rank %d step %lld: entry %u of %u: mi %#x (slot %lld) mk %u mo %u; nl %u no %u nr %u "
                        "n %u o0 %u o1 %u ncells %u",
                        R.rank, (long long)ctx->steps, r, m, mi[r], (long long)x, mk[r], mo[r], h.nl, h.no, h.nr, h.n, h.o0,
                        h.o1, ncells);
        by_slot.push_back(Ent{(uint32_t)x, mo[r], r});
    }
    if (g_ht.on) {   // measurement (SPH_HOST_TIMING with SPH_FLAG_VALIDATE): the movers by origin and column move
        const uint32_t gyz = col_keys(ctx->grid);
        uint32_t own = 0, rec = 0, rec_clamped = 0, rec_col0 = 0, rec_col1 = 0, rec_colx = 0, own_col0 = 0;
        for (uint32_t r = 0; r < m; ++r) {
            const bool isr = (mi[r] & MV_REC) != 0;
            const int32_t dc = (int32_t)(mk[r] / gyz) - (int32_t)(mo[r] / gyz);
            if (isr) {
                ++rec;
                if (mo[r] == 0u || mo[r] == ncells - 1u) ++rec_clamped;
                if (dc == 0) ++rec_col0; else if (dc == 1 || dc == -1) ++rec_col1; else ++rec_colx;
            } else {
                ++own;
                if (dc == 0) ++own_col0;
            }
        }
        std::fprintf(stderr, "[movers] rank %d step %lld: own %u (same column %u), records %u (clamped old key %u; same column "
                     "%u, one column %u, more %u) of nl %u nr %u\n", R.rank, (long long)ctx->steps, own, own_col0, rec,
                     rec_clamped, rec_col0, rec_col1, rec_colx, h.nl, h.nr);
    }
    // the assembled old keys (records: keys2, own: sk_cur) and new keys (records: vals, own: keys)
    const uint32_t n = h.n;
    std::vector<uint32_t> skr(n), keyr(n), sko(h.no), keyo(h.no);
    if (n) {
        HIPCHK(hipMemcpy(skr.data(), ctx->keys2, n * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(keyr.data(), ctx->vals, n * 4, hipMemcpyDeviceToHost));
    }
    if (h.no) {
        HIPCHK(hipMemcpy(sko.data(), ctx->sk_cur + h.o0, h.no * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(keyo.data(), ctx->keys + h.o0, h.no * 4, hipMemcpyDeviceToHost));
    }
    std::sort(by_slot.begin(), by_slot.end());
    uint32_t nrec = 0;
    for (uint32_t r = 0; r < m; ++r) nrec += (mi[r] & MV_REC) != 0;
    for (size_t k = 1; k < by_slot.size(); ++k)
        if (by_slot[k].slot == by_slot[k - 1].slot || by_slot[k].mo < by_slot[k - 1].mo) {
            const Ent& a = by_slot[k - 1];
            const Ent& b = by_slot[k];
            float4 rec[4] = {};
            if (R.left >= 0) HIPCHK(hipMemcpy(rec, R.msg_in[0], sizeof rec, hipMemcpyDeviceToHost));
            uint32_t u[16];
            std::memcpy(u, rec, sizeof u);
            return fail(ctx, SPH_ERR_STATE,
                        "validate(movers) rank %d step %lld: slot %u (entry %u: mi %#x mk %u mo %u) before slot %u (entry %u: "
                        "mi %#x mk %u mo %u); %u movers (%u records); nl %u no %u nr %u n %u o0 %u o1 %u ncells %u; "
                        "left hdr %u %u rec0 pos %g %g %g id %d og %u; c1i %d %d c1o %d %d mcap_in %d; skr0 %u keyr0 %u "
                        "cx0 %d gyz %u",
                        R.rank, (long long)ctx->steps, a.slot, a.r, mi[a.r], mk[a.r], mo[a.r], b.slot, b.r, mi[b.r], mk[b.r],
                        mo[b.r], m, nrec, h.nl, h.no, h.nr, h.n, h.o0, h.o1, ncells, u[0], u[1], rec[2].x, rec[2].y, rec[2].z,
                        (int)u[11], u[15], R.c1i[0], R.c1i[1], R.c1o[0], R.c1o[1], R.mcap_in[0], n ? skr[0] : 0u,
                        n ? keyr[0] : 0u, ctx->grid.cx0, gyz(ctx));
        }
    for (uint32_t k = 0; k <= ncells; ++k)
        if (cs[k] > cs[k + 1] || (k == ncells && cs[k] != h.n))
            return fail(ctx, SPH_ERR_STATE, "validate(movers) rank %d: old cell starts broken at %u (%u %u, n %u)", R.rank,
                        k, cs[k], cs[k + 1], h.n);
    auto ask = [&](uint32_t x) { return (x < h.nl || x >= h.nl + h.no) ? skr[x] : sko[x - h.nl]; };
    auto akey = [&](uint32_t x) { return (x < h.nl || x >= h.nl + h.no) ? keyr[x] : keyo[x - h.nl]; };
    uint32_t moved = 0;
    for (uint32_t x = 0; x < n; ++x) {
        const uint32_t k = ask(x);
        if (k >= ncells || (x && ask(x - 1) > k) || x < cs[k] || x >= cs[k + 1])
            return fail(ctx, SPH_ERR_STATE, "validate(movers) rank %d: old key %u of slot %u (prev %u) vs cs %u %u; nl %u no %u n %u",
                        R.rank, k, x, x ? ask(x - 1) : 0u, k < ncells ? cs[k] : 0u, k < ncells ? cs[k + 1] : 0u, h.nl, h.no, n);
        moved += akey(x) != k;
    }
    if (moved != m)
        return fail(ctx, SPH_ERR_STATE, "validate(movers) rank %d: %u slots changed key, %u movers listed", R.rank, moved, m);
    for (uint32_t r = 0; r < m; ++r) {
        const uint32_t x = by_slot[r].slot;
        if (ask(x) != by_slot[r].mo)
            return fail(ctx, SPH_ERR_STATE, "validate(movers) rank %d: mover slot %u old key %u, slot holds %u", R.rank, x,
                        by_slot[r].mo, ask(x));
    }
    return SPH_OK;
}

// ---------------------------------------------------------------- phase A: counts and messages
// Sends from the four boundary columns only (slab.hip send_ranges): the cut is older than three steps and the
// last force pass checked that no own particle moved more than one column (SlabSizes.jump). That check reads
// the previous slot order's keys (MoverSink.sk), which exist only with the incremental re-sort; after a
// full-sort step (SPH_RESORT=0, or a step past the mover limit) every own slot is scanned.
bool steady_sends(const RankState& R) { return R.since_cut >= 3 && R.jump_guard; }

int phase_count(RankState& R, bool exact, int64_t step) {
    sph_ctx* ctx = R.c;
    HIPCHK(hipSetDevice(ctx->device));
    if (!ctx->keys_valid) {   // after init or a re-cut: keys of the owned slots in the (new) window
        const int32_t no = ctx->o1 - ctx->o0;
        if (no > 0) {
            KTimer t(ctx, "keys", 20.0 * no);
            launch_keys(ctx->pos + ctx->o0, no, nullptr, 0, ctx->grid, ctx->keys + ctx->o0, ctx->stream);
        }
        ctx->keys_valid = true;
    }
    if (R.left < 0 && R.right < 0) return SPH_OK;
    // the count blocks over the owned slots of the previous order (within its slot bound); the pack
    // reads the per-block counts with this same block count
    R.nb_send = slab_send_blocks(0, (int32_t)std::max<int64_t>(R.n_prev_ub, 1));
    KTimer t(ctx, "slab_count", 4.0 * R.n_prev_ub);
    launch_slab_count_dev(ctx->keys, R.dz, R.nb_send, gyz(ctx), col_le(ctx), col_ge(ctx), ctx->sblk,
                          totals_slot(ctx, step), ctx->stream, steady_sends(R), exact);
    CKPT(R, "count");
    return SPH_OK;
}

int phase_pack(RankState& R, Multi& M, int64_t step) {
    sph_ctx* ctx = R.c;
    HIPCHK(hipSetDevice(ctx->device));
    for (int s = 0; s < 2; ++s) {
        const int peer = s == 0 ? R.left : R.right;
        if (peer < 0) continue;
        int r = ensure_buf(M, ctx, &R.msg_out[s], &R.mcap_out[s], MSG_HDR_F4 + 2 * R.c1o[s]);
        if (r != SPH_OK) return r;
        r = ensure_buf(M, ctx, &R.msg_in[s], &R.mcap_in[s], MSG_HDR_F4 + 2 * R.c1i[s]);
        if (r != SPH_OK) return r;
        // the neighbour's copy of last step's message must be done before it is overwritten
        if (M.mode == 1) HIPCHK(hipStreamWaitEvent(ctx->stream, M.ranks[peer - M.ranks[0].rank].ev_in, 0));
    }
    {
        KTimer t(ctx, "slab_pack", 36.0 * (R.c1o[0] + R.c1o[1]));
        launch_slab_pack2_dev(ctx->keys, ctx->pos, ctx->vel, ctx->id, ctx->sk_valid ? ctx->sk_cur : nullptr,
                              (uint32_t)ctx->grid.cx0 * gyz(ctx), R.dz, R.nb_send, gyz(ctx), col_le(ctx), col_ge(ctx),
                              ctx->sblk, R.left >= 0 ? R.msg_out[0] : nullptr, R.c1o[0],
                              R.right >= 0 ? R.msg_out[1] : nullptr, R.c1o[1], totals_slot(ctx, step), ctx->stream,
                              steady_sends(R));
    }
    HIPCHK(hipGetLastError());
    // the peer copies of a local group wait for it (RCCL orders its sends on this stream itself); a
    // marker costs the stream a few microseconds, so none without a neighbour
    if (M.mode == 1 && (R.left >= 0 || R.right >= 0)) HIPCHK(hipEventRecord(R.ev_packed, ctx->stream));
    CKPT(R, "pack");
    return SPH_OK;
}

// ---------------------------------------------------------------- exchanges
int exchange_counts(Multi& M, sph_ctx* pctx, int64_t step) {
    // exact-size steps: the host reads every local rank's send counts, then learns the neighbours'
    for (auto& R : M.ranks) {
        sph_ctx* ctx = R.c;
        HIPCHK(hipSetDevice(ctx->device));
        uint32_t t[2] = {0, 0};
        if (R.left >= 0 || R.right >= 0) {
            HIPCHK(hipMemcpyAsync(t, totals_slot(ctx, step), 8, hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(hipStreamSynchronize(ctx->stream));
        }
        R.c1o[0] = R.left >= 0 ? (int32_t)t[0] : 0;
        R.c1o[1] = R.right >= 0 ? (int32_t)t[1] : 0;
    }
    if (M.mode == 1) {
        const int r0 = M.ranks[0].rank;
        for (auto& R : M.ranks) {
            R.c1i[0] = R.left >= 0 ? M.ranks[R.left - r0].c1o[1] : 0;
            R.c1i[1] = R.right >= 0 ? M.ranks[R.right - r0].c1o[0] : 0;
        }
        return SPH_OK;
    }
    RankState& R = M.ranks[0];
    sph_ctx* ctx = R.c;
    (void)pctx;
    NCCLCHK(ncclGroupStart());
    if (R.left >= 0) {
        NCCLCHK(ncclSend(totals_slot(ctx, step), 1, ncclUint32, R.left, M.comm, ctx->stream));
        NCCLCHK(ncclRecv(R.cnt_dev + 0, 1, ncclUint32, R.left, M.comm, ctx->stream));
    }
    if (R.right >= 0) {
        NCCLCHK(ncclSend(totals_slot(ctx, step) + 1, 1, ncclUint32, R.right, M.comm, ctx->stream));
        NCCLCHK(ncclRecv(R.cnt_dev + 1, 1, ncclUint32, R.right, M.comm, ctx->stream));
    }
    NCCLCHK(ncclGroupEnd());
    uint32_t in[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(in, R.cnt_dev, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    R.c1i[0] = R.left >= 0 ? (int32_t)in[0] : 0;
    R.c1i[1] = R.right >= 0 ? (int32_t)in[1] : 0;
    return SPH_OK;
}

int exchange1(Multi& M) {
    if (M.mode == 1) {
        const int r0 = M.ranks[0].rank;
        for (auto& R : M.ranks) {
            sph_ctx* ctx = R.c;
            HIPCHK(hipSetDevice(ctx->device));
            for (int s = 0; s < 2; ++s) {
                const int peer = s == 0 ? R.left : R.right;
                if (peer < 0) continue;
                RankState& S = M.ranks[peer - r0];
                const size_t bytes = (size_t)(MSG_HDR_F4 + 2 * R.c1i[s]) * sizeof(float4);
                HIPCHK(hipStreamWaitEvent(ctx->stream, S.ev_packed, 0));
                HIPCHK(hipMemcpyPeerAsync(R.msg_in[s], ctx->device, S.msg_out[1 - s], S.c->device, bytes, ctx->stream));
            }
            if (R.left >= 0 || R.right >= 0) HIPCHK(hipEventRecord(R.ev_in, ctx->stream));
        }
        return SPH_OK;
    }
    RankState& R = M.ranks[0];
    sph_ctx* ctx = R.c;
    NCCLCHK(ncclGroupStart());
    for (int s = 0; s < 2; ++s) {
        const int peer = s == 0 ? R.left : R.right;
        if (peer < 0) continue;
        NCCLCHK(ncclSend(R.msg_out[s], (size_t)(MSG_HDR_F4 + 2 * R.c1o[s]) * sizeof(float4), ncclUint8, peer, M.comm,
                         ctx->stream));
        NCCLCHK(ncclRecv(R.msg_in[s], (size_t)(MSG_HDR_F4 + 2 * R.c1i[s]) * sizeof(float4), ncclUint8, peer, M.comm,
                         ctx->stream));
    }
    NCCLCHK(ncclGroupEnd());
    return SPH_OK;
}

int exchange2_start(Multi& M) {
    if (M.mode == 1) {
        const int r0 = M.ranks[0].rank;
        for (auto& R : M.ranks) {
            sph_ctx* ctx = R.c;
            HIPCHK(hipSetDevice(ctx->device));
            for (int s = 0; s < 2; ++s) {
                const int peer = s == 0 ? R.left : R.right;
                if (peer < 0) continue;
                RankState& S = M.ranks[peer - r0];
                if (s == 0 || R.left < 0)   // once: the boundary force pass on this stream reads this rank's density
                    HIPCHK(hipStreamWaitEvent(R.comm, R.ev_rho_packed, 0));
                HIPCHK(hipStreamWaitEvent(R.comm, S.ev_rho_packed, 0));
                HIPCHK(hipMemcpyPeerAsync(R.rho_in[s], ctx->device, S.rho_out[1 - s], S.c->device,
                                          (size_t)(RHO_HDR + R.c2i[s]) * sizeof(float2), R.comm));
            }
            HIPCHK(hipEventRecord(R.ev_rho_recv, R.comm));
        }
        return SPH_OK;
    }
    RankState& R = M.ranks[0];
    sph_ctx* ctx = R.c;
    HIPCHK(hipStreamWaitEvent(R.comm, R.ev_rho_packed, 0));
    NCCLCHK(ncclGroupStart());
    for (int s = 0; s < 2; ++s) {
        const int peer = s == 0 ? R.left : R.right;
        if (peer < 0) continue;
        NCCLCHK(ncclSend(R.rho_out[s], (size_t)(RHO_HDR + R.c2o[s]) * sizeof(float2), ncclUint8, peer, M.comm, R.comm));
        NCCLCHK(ncclRecv(R.rho_in[s], (size_t)(RHO_HDR + R.c2i[s]) * sizeof(float2), ncclUint8, peer, M.comm, R.comm));
    }
    NCCLCHK(ncclGroupEnd());
    HIPCHK(hipEventRecord(R.ev_rho_recv, R.comm));
    return SPH_OK;
}

// ---------------------------------------------------------------- phase B: assemble, density, ρ out
int phase_assemble(RankState& R, bool exact) {
    sph_ctx* ctx = R.c;
    ctx->hm_valid = false;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    // the layout [left | own | right] from the message headers: in k_slab_rec on device-sized steps
    // (a rank without neighbours has it from the previous step's k_slab_lag), k_slab_sizes otherwise
    const SizesIn sizes{R.left >= 0 ? R.msg_in[0] : nullptr, R.right >= 0 ? R.msg_in[1] : nullptr, R.c1i[0], R.c1i[1],
                        ctx->capacity};
    R.n_ub = std::min<int64_t>(R.c1i[0] + R.n_prev_ub + R.c1i[1], ctx->capacity);
    const bool pre = R.pre_rec;   // the record kernel ran at the end of the last step (issue_next_rec)
    R.pre_rec = false;
    ctx->dz_next = false;
    const bool many = !pre && ctx->resort_mode == 1 && *(volatile uint32_t*)ctx->mv_host > resort_limit((int32_t)R.n_ub);
    if (pre || (ctx->resort_mode != 0 && !many && ctx->sk_valid && R.n_ub > 0)) {
        // incremental re-sort over [left records | own slots | right records], sizes on the device
        const int32_t nl_ub = R.c1i[0], nr_ub = R.c1i[1], n_ub = (int32_t)R.n_ub;
        const AsmSrc src{ctx->pos, ctx->vel, ctx->id, ctx->sk_cur, ctx->keys, 0,
                         R.left >= 0 ? (const float4*)(R.msg_in[0] + MSG_HDR_F4) : nullptr,
                         R.right >= 0 ? (const float4*)(R.msg_in[1] + MSG_HDR_F4) : nullptr,
                         ctx->keys2, ctx->vals, nl_ub, n_ub - nr_ub, R.dz};
        const int used = ctx->mv_par;
        const MoverSink mv{ctx->keys2, ctx->mv_count + used, ctx->mv_mi, ctx->mv_mk, ctx->mv_mo,
                           (uint32_t)std::max(ctx->capacity, 1), &R.dz->flags};
        const uint32_t key_base = (uint32_t)ctx->grid.cx0 * gyz(ctx);
        CKPT(R, "exchange 1");
        KTimer t(ctx, "resort", (double)R.n_ub * (2 * 4 + 2 * 36), true);
        if (pre) {   // its old cell-start table becomes the table of this step
            std::swap(ctx->cs, R.cs_alt);
            std::swap(ctx->cs_cap, R.cs_alt_cap);
        } else if (nl_ub + nr_ub > 0) {   // every rank with a neighbour (capacities are >= 512)
            // the records' keys and movers, the sizes, and the old cell-start table in one launch (without
            // neighbours the own block keeps its cell starts)
            CsOld csp;
            csp.cs = ctx->cs;
            csp.ncells = ctx->grid.ncells;
            csp.gyz = gyz(ctx);
            csp.gx = (uint32_t)ctx->grid.gx;
            csp.has_left = ctx->has_left ? 1 : 0;
            csp.has_right = ctx->has_right ? 1 : 0;
            launch_slab_rec(src, n_ub, ctx->grid, key_base, ctx->vals, ctx->keys2, mv, s, &sizes, csp);  // grid: nl_ub + nr_ub
        }
        CKPT(R, "sizes + slab_rec + cs_old");
        if (ctx->cfg.flags & SPH_FLAG_VALIDATE) {
            int r = validate_movers(R, used);
            if (r != SPH_OK) return r;
        }
        const int32_t lc_lo = ctx->sl.cx_lo - ctx->grid.cx0, lc_hi = ctx->sl.cx_hi - ctx->grid.cx0;
        CsPick pick{{col_start(ctx, 0), col_start(ctx, lc_lo), col_start(ctx, lc_lo + 1), col_start(ctx, lc_hi - 1),
                     col_start(ctx, lc_hi), col_start(ctx, ctx->grid.gx), col_start(ctx, std::min(lc_lo + 2, lc_hi)),
                     col_start(ctx, std::max(lc_hi - 2, lc_lo))},
                    8, R.dz->pick, nullptr};
        ResortScratch w = resort_scratch(ctx);
        w.dz = R.dz;
        w.err = &R.dz->flags;
        launch_resort(src, ctx->cs, ctx->cs2, ctx->grid.ncells, n_ub, ctx->mv_count + used, ctx->mv_count + (1 - used),
                      w, ctx->pos2, ctx->vel2, ctx->id2, ctx->sk_next, s, pick);
        swap_cs(ctx);
        CKPT(R, "resort");   // (k_mv_rank stored the mover count for the host)
        ctx->mv_par = 1 - used;
        swap_sv(ctx);
        std::swap(ctx->id, ctx->id2);
        std::swap(ctx->sk_cur, ctx->sk_next);
        ctx->keys_valid = false;
        ctx->sk_valid = true;
        ctx->n = n_ub;
    } else {
        // the full radix sort: host-sized (after a re-cut, or while many particles move)
        launch_slab_sizes(R.dz, sizes.hl, sizes.hr, sizes.cap_l, sizes.cap_r, sizes.capacity, s);
        HIPCHK(hipStreamSynchronize(s));
        SlabSizes h;
        HIPCHK(hipMemcpy(&h, R.dz, sizeof h, hipMemcpyDeviceToHost));
        // an overflow here is not returned on this rank alone (its neighbours would wait in the next
        // exchange): the sizes are clamped (nl = nr = 0 past the capacity), the step completes, and the
        // sticky flag stops every rank together two steps on (multi_one_step)
        ctx->dz_ahead = false;
        ctx->o0 = (int32_t)h.o0;
        ctx->o1 = (int32_t)h.o1;
        int r = slab_assemble(ctx, R.left >= 0 ? (const void*)(R.msg_in[0] + MSG_HDR_F4) : nullptr, (int32_t)h.nl,
                              R.right >= 0 ? (const void*)(R.msg_in[1] + MSG_HDR_F4) : nullptr, (int32_t)h.nr, true);
        if (r != SPH_OK) return r;
        ctx->rng_pending = false;
        // the picked column starts (sdev[0..7]) and the slot count into the device sizes
        HIPCHK(hipMemcpyAsync(R.dz->pick, ctx->sdev, 8 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
        const uint32_t nn = (uint32_t)ctx->n;
        HIPCHK(hipMemcpyAsync(&R.dz->n, &nn, sizeof nn, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));   // nn lives on this stack frame
        R.n_ub = ctx->n;
    }
    if (exact && (R.left >= 0 || R.right >= 0)) {   // exact ρ message sizes: this rank's own columns
        HIPCHK(hipStreamSynchronize(s));
        SlabSizes h;
        HIPCHK(hipMemcpy(&h, R.dz, sizeof h, hipMemcpyDeviceToHost));
        R.c2o[0] = R.left >= 0 ? (int32_t)(h.pick[2] - h.pick[1]) : 0;
        R.c2o[1] = R.right >= 0 ? (int32_t)(h.pick[4] - h.pick[3]) : 0;
        R.c2i[0] = R.left >= 0 ? (int32_t)(h.pick[1] - h.pick[0]) : 0;
        R.c2i[1] = R.right >= 0 ? (int32_t)(h.pick[5] - h.pick[4]) : 0;
    }
    return SPH_OK;
}

// The density pass over the owned slots of the new order (the column starts the re-sort picked; k_slab_lag
// copies the ranges for the host at the end of the step). It also writes both ρ halo messages: the own
// boundary columns' (ρ, P/ρ²) in slot order (RhoOut), so no packing launch follows it.
int phase_density(RankState& R, Multi& M) {
    sph_ctx* ctx = R.c;
    HIPCHK(hipSetDevice(ctx->device));
    RhoOut ro;
    for (int sd = 0; sd < 2; ++sd) {
        const int peer = sd == 0 ? R.left : R.right;
        if (peer < 0) continue;
        int r = ensure_buf(M, ctx, &R.rho_out[sd], &R.rcap_out[sd], RHO_HDR + R.c2o[sd]);
        if (r != SPH_OK) return r;
        r = ensure_buf(M, ctx, &R.rho_in[sd], &R.rcap_in[sd], RHO_HDR + R.c2i[sd]);
        if (r != SPH_OK) return r;
        // the neighbour's copy of last step's message must be done before the density pass overwrites it
        if (M.mode == 1) HIPCHK(hipStreamWaitEvent(ctx->stream, M.ranks[peer - M.ranks[0].rank].ev_rho_recv, 0));
        ro.msg[sd] = R.rho_out[sd];
        ro.cap[sd] = R.c2o[sd];
    }
    if (ro.msg[0] || ro.msg[1]) ro.dz = R.dz;
    if (M.mode == 2 && M.world > 1) ro.fbits = R.cnt_dev + 4;   // this rank's flags, one word per bit, for the OR
    {
        KTimer t(ctx, "density", 24.0 * (double)R.n_ub, true);
        launch_density_tiled(ctx->pos, ctx->cs, 0, (int32_t)R.n_ub, ctx->grid, ctx->sc, ctx->rp, hit_mask_write(ctx),
                             path_ctr(ctx), ctx->stream, DevRange{&R.dz->pick[1], &R.dz->pick[4]}, ro);
    }
    HIPCHK(hipGetLastError());
    if (R.left >= 0 || R.right >= 0) HIPCHK(hipEventRecord(R.ev_rho_packed, ctx->stream));
    CKPT(R, "density + rho pack");
    return SPH_OK;
}

// ---------------------------------------------------------------- phase C: force passes, finish
// Returns whether the pass ran the column-jump guard (steady_sends). A second range [lo2, hi2) (at most
// grid_ub2 slots) runs in the same launch: the two boundary columns are one launch.
bool force_dev(sph_ctx* ctx, const uint32_t* lo, const uint32_t* hi, int64_t grid_ub, float dt,
               const uint32_t* lo2 = nullptr, const uint32_t* hi2 = nullptr, int64_t grid_ub2 = 0,
               hipStream_t st = nullptr, bool jump_err = false, SendBins sb = SendBins{}) {
    MoverSink mv = mover_sink(ctx);
    if (grid_ub <= 0 && grid_ub2 <= 0) return mv.sk != nullptr;
    KTimer t(ctx, "force_integrate", 76.0 * (double)(std::max<int64_t>(grid_ub, 0) + grid_ub2), true);
    mv.err = &ctx->dz->flags;
    mv.jump = &ctx->dz->jump;
    mv.jump_err = jump_err ? 1 : 0;
    launch_force_tiled(ctx->pos, ctx->vel, ctx->rp, ctx->cs, 0, (int32_t)std::max<int64_t>(grid_ub, 0), ctx->grid, ctx->sc,
                       dt, forcing(ctx), ctx->pos2, ctx->vel2, ctx->keys, mv, hit_mask_read(ctx), path_ctr(ctx),
                       st ? st : ctx->stream, DevRange{lo, hi}, DevRange{lo2, hi2}, (int32_t)grid_ub2, sb);
    return mv.sk != nullptr;
}

// early: the next step's messages are packed right after the boundary pass, so that pass takes the two columns at
// each side a send can come from (lo, lo + 1 | hi − 2, hi − 1; slab.hip send_ranges) and the interior pass the
// rest; an interior particle that moves two or more columns could then be missed by the sends, so the interior pass
// reports it (SZ_JUMP_EARLY stops every rank) instead of asking for a full scan.
int phase_interior(RankState& R, float dt, bool early) {
    sph_ctx* ctx = R.c;
    HIPCHK(hipSetDevice(ctx->device));
    // interior columns: [pick[2] or pick[1], pick[3] or pick[4]) (empty when a one-column slab has both
    // neighbours: then the bound is below the start and every workgroup exits); early: [pick[6], pick[7])
    const uint32_t* pk = R.dz->pick;
    if (early)
        R.jump_guard = force_dev(ctx, ctx->has_left ? &pk[6] : &pk[1], ctx->has_right ? &pk[7] : &pk[4], R.n_ub, dt,
                                 nullptr, nullptr, 0, nullptr, true);
    else
        R.jump_guard = force_dev(ctx, ctx->has_left ? &pk[2] : &pk[1], ctx->has_right ? &pk[3] : &pk[4], R.n_ub, dt);
    if (early && !R.jump_guard) HIPCHK(hipEventRecord(R.ev_fdone, ctx->stream));   // the early sends scan all slots
    CKPT(R, "interior force");
    return SPH_OK;
}

// The ghost ρ and the boundary columns' force pass run on the comm stream, behind the ρ receive (which is ordered
// after this rank's density pass, exchange2_start), so the boundary workgroups run alongside the interior pass and
// fill its tail instead of making a small launch of their own after it. early: the two columns at each side, then
// the next step's counts and messages on the same stream (phase_interior).
int phase_boundary(RankState& R, Multi& M, float dt, bool early) {
    sph_ctx* ctx = R.c;
    HIPCHK(hipSetDevice(ctx->device));
    const bool halo = R.left >= 0 || R.right >= 0;
    hipStream_t b = halo ? R.comm : ctx->stream;
    launch_slab_unpack_rho2(ctx->rp, R.dz, R.left >= 0 ? R.rho_in[0] : nullptr, R.c2i[0],
                            R.right >= 0 ? R.rho_in[1] : nullptr, R.c2i[1], b);
    CKPT(R, "rho unpack");
    const bool one_col = ctx->sl.cx_hi - ctx->sl.cx_lo == 1;
    const uint32_t* pk = R.dz->pick;
    R.ebins_used = false;
    if (early) {   // lo, lo + 1 | hi − 2, hi − 1 (every slab has at least four columns)
        const int64_t gl = R.g2[0] > 0 ? std::min<int64_t>(R.g2[0], R.n_ub) : R.n_ub;
        const int64_t gr = R.g2[1] > 0 ? std::min<int64_t>(R.g2[1], R.n_ub) : R.n_ub;
        // with the jump guard the next step's sends come from exactly these columns, so this pass counts them per
        // send block (SendBins: no count launch); without it they come from every own slot (phase_boundary below)
        SendBins sb;
        R.nb_send = slab_send_blocks(0, (int32_t)std::max<int64_t>(R.n_ub, 1));
        if (halo && R.jump_guard && !env_on("SPH_NO_FOLDED_COUNT")) {
            int r = ensure_ebins(M, R, R.nb_send);
            if (r != SPH_OK) return r;
            sb.bins = R.ebins;
            sb.nblk = R.nb_send;
            sb.col_le = col_le(ctx);
            sb.col_ge = col_ge(ctx);
            sb.side[0] = ctx->has_left ? 0 : 1;
            sb.side[1] = ctx->has_left && ctx->has_right ? 1 : -1;
            R.ebins_used = true;
        }
        // a boundary particle that moves two columns can leave the candidate columns of the other side too
        if (ctx->has_left && ctx->has_right)
            force_dev(ctx, &pk[1], &pk[6], gl, dt, &pk[7], &pk[4], gr, b, true, sb);
        else if (ctx->has_left)
            force_dev(ctx, &pk[1], &pk[6], gl, dt, nullptr, nullptr, 0, b, true, sb);
        else if (ctx->has_right)
            force_dev(ctx, &pk[7], &pk[4], gr, dt, nullptr, nullptr, 0, b, true, sb);
    } else if (one_col && (ctx->has_left || ctx->has_right)) {   // the owned column is both boundary columns
        force_dev(ctx, &pk[1], &pk[4], R.n_ub, dt, nullptr, nullptr, 0, b);
    } else if (ctx->has_left && ctx->has_right) {   // both boundary columns in one launch
        force_dev(ctx, &pk[1], &pk[2], std::min<int64_t>(R.c2o[0], R.n_ub), dt, &pk[3], &pk[4],
                  std::min<int64_t>(R.c2o[1], R.n_ub), b);
    } else {
        if (ctx->has_left) force_dev(ctx, &pk[1], &pk[2], std::min<int64_t>(R.c2o[0], R.n_ub), dt, nullptr, nullptr, 0, b);
        if (ctx->has_right) force_dev(ctx, &pk[3], &pk[4], std::min<int64_t>(R.c2o[1], R.n_ub), dt, nullptr, nullptr, 0, b);
    }
    if (halo) HIPCHK(hipEventRecord(R.ev_bdone, b));
    CKPT(R, "boundary force");
    if (!early || !halo) return SPH_OK;
    // An error below leaves the counts the boundary pass added into ebins (only k_slab_lag clears them): cleared
    // here on the comm stream, so that a later early step cannot add to stale counts.
    auto bail = [&](int rc) {
        if (R.ebins_used) (void)hipMemsetAsync(R.ebins, 0, 2 * (size_t)R.nb_send * sizeof(uint32_t), b);
        R.ebins_used = false;
        return rc;
    };
    // the next step's sends, from this step's order and new positions: capacities from the counts two steps before
    // the next step (as multi_one_step derives them), one count launch and one pack launch. Both neighbours derive
    // them from the same record. The host waits here for the previous step's comm work, so it runs at most one step
    // ahead of the GPU. (Three steps before, from the record already waited for at this step's start, overflowed a
    // message after a re-cut: the record of the first step after a cut holds the migration, not the new halo.)
    int r = SPH_OK;
    const uint32_t* L = lag_slot(R, M.steps - 1, ctx, &r);
    if (r != SPH_OK) return bail(r);
    R.e_c1o[0] = R.left >= 0 ? cap_of(M, L[0]) : 0;
    R.e_c1o[1] = R.right >= 0 ? cap_of(M, L[1]) : 0;
    R.e_c1i[0] = R.left >= 0 ? cap_of(M, L[2]) : 0;
    R.e_c1i[1] = R.right >= 0 ? cap_of(M, L[3]) : 0;
    for (int sd = 0; sd < 2; ++sd) {
        const int peer = sd == 0 ? R.left : R.right;
        if (peer < 0) continue;
        if ((r = ensure_buf(M, ctx, &R.msg_out[sd], &R.mcap_out[sd], MSG_HDR_F4 + 2 * R.e_c1o[sd])) != SPH_OK) return bail(r);
        if ((r = ensure_buf(M, ctx, &R.msg_in[sd], &R.mcap_in[sd], MSG_HDR_F4 + 2 * R.e_c1i[sd])) != SPH_OK) return bail(r);
        // the neighbour's copy of this step's message must be done before it is overwritten
        if (M.mode == 1) HIPCHK(hipStreamWaitEvent(b, M.ranks[peer - M.ranks[0].rank].ev_in, 0));
    }
    // without the jump guard (a full-sort step) the sends scan every own slot, after the interior pass
    const bool cand = R.jump_guard;
    if (!cand && hipStreamWaitEvent(b, R.ev_fdone, 0) != hipSuccess) return bail(fail(ctx, SPH_ERR_HIP, "wait ev_fdone"));
    if (!R.ebins_used) {
        KTimer t(ctx, "slab_count", 4.0 * R.n_ub, false, b);
        launch_slab_count_dev(ctx->keys, R.dz, R.nb_send, gyz(ctx), col_le(ctx), col_ge(ctx), ctx->sblk,
                              totals_slot(ctx, M.steps + 1), b, cand, false, true);
    }
    {
        KTimer t(ctx, "slab_pack", 36.0 * (R.e_c1o[0] + R.e_c1o[1]), false, b);
        launch_slab_pack2_dev(ctx->keys, ctx->pos2, ctx->vel2, ctx->id, ctx->sk_valid ? ctx->sk_cur : nullptr,
                              (uint32_t)ctx->grid.cx0 * gyz(ctx), R.dz, R.nb_send, gyz(ctx), col_le(ctx), col_ge(ctx),
                              R.ebins_used ? R.ebins : ctx->sblk, R.left >= 0 ? R.msg_out[0] : nullptr, R.e_c1o[0],
                              R.right >= 0 ? R.msg_out[1] : nullptr, R.e_c1o[1], totals_slot(ctx, M.steps + 1), b, cand,
                              true);
    }
    HIPCHK(hipGetLastError());
    if (M.mode == 1) HIPCHK(hipEventRecord(R.ev_packed, b));
    CKPT(R, "early pack");
    return SPH_OK;
}

// The next step's halo messages, on the comm streams (early sends): peer copies in a local group, one RCCL group
// per rank otherwise. The step's bookkeeping follows them there (phase_finish), and the next step's first launch
// waits for ev_sent.
int exchange1_early(Multi& M) {
    if (M.mode == 1) {
        const int r0 = M.ranks[0].rank;
        for (auto& R : M.ranks) {
            sph_ctx* ctx = R.c;
            HIPCHK(hipSetDevice(ctx->device));
            for (int s = 0; s < 2; ++s) {
                const int peer = s == 0 ? R.left : R.right;
                if (peer < 0) continue;
                RankState& S = M.ranks[peer - r0];
                const size_t bytes = (size_t)(MSG_HDR_F4 + 2 * R.e_c1i[s]) * sizeof(float4);
                HIPCHK(hipStreamWaitEvent(R.comm, S.ev_packed, 0));
                HIPCHK(hipMemcpyPeerAsync(R.msg_in[s], ctx->device, S.msg_out[1 - s], S.c->device, bytes, R.comm));
            }
            if (R.left >= 0 || R.right >= 0) HIPCHK(hipEventRecord(R.ev_in, R.comm));
        }
        return SPH_OK;
    }
    RankState& R = M.ranks[0];
    if (R.left < 0 && R.right < 0) return SPH_OK;
    sph_ctx* ctx = R.c;
    NCCLCHK(ncclGroupStart());
    for (int s = 0; s < 2; ++s) {
        const int peer = s == 0 ? R.left : R.right;
        if (peer < 0) continue;
        NCCLCHK(ncclSend(R.msg_out[s], (size_t)(MSG_HDR_F4 + 2 * R.e_c1o[s]) * sizeof(float4), ncclUint8, peer, M.comm,
                         R.comm));
        NCCLCHK(ncclRecv(R.msg_in[s], (size_t)(MSG_HDR_F4 + 2 * R.e_c1i[s]) * sizeof(float4), ncclUint8, peer, M.comm,
                         R.comm));
    }
    NCCLCHK(ncclGroupEnd());
    return SPH_OK;
}

// early (the next step's messages went out on the comm stream): the bookkeeping kernel follows them there, so the
// main stream runs from this step's interior pass into the next step's assemble behind one wait (ev_sent,
// multi_join) instead of a wait for the boundary pass plus a launch of its own. Its flags word then holds what the
// interior pass of this step flagged only if that pass has finished; the flags are sticky, so the next step's record
// carries them (an RCCL rank's flags are the all-reduced ones of the density pass either way).
// The next step's record kernel, issued at the end of this one (early sends: the messages it reads have arrived on
// the comm stream): the records' keys and movers, the assembled sizes and the old cell-start table leave the compute
// stream's critical path (~12 µs per step at C3) for the comm stream, which runs under the interior force pass. The
// table is built into a second buffer (the interior pass still reads ctx->cs), swapped in by the next assemble. The
// records' movers join the force passes' in the same counter (the re-sort does not depend on the list order), and
// its size store clears SlabSizes.jump, which this step's passes do not set (early sends report jumps as
// SZ_JUMP_EARLY). A host-side change between the steps (sph_debug_kick) keeps it valid: the messages the next step
// re-packs hold the same particles at the same positions.
int issue_next_rec(Multi& M, RankState& R) {
    sph_ctx* ctx = R.c;
    if (env_on("SPH_NO_PRE_REC") || ctx->resort_mode == 0 || !ctx->sk_valid) return SPH_OK;
    const int32_t nl_ub = R.e_c1i[0], nr_ub = R.e_c1i[1];
    if (nl_ub + nr_ub <= 0) return SPH_OK;
    const int64_t n_ub = std::min<int64_t>(nl_ub + R.n_ub + nr_ub, ctx->capacity);   // a bound: sizes come from headers
    if (ctx->resort_mode == 1 && *(volatile uint32_t*)ctx->mv_host > resort_limit((int32_t)n_ub)) return SPH_OK;
    const uint32_t need = ctx->grid.ncells + 2;
    if (need > R.cs_alt_cap || !R.cs_alt) {
        int r = sync_all(M, ctx);
        if (r != SPH_OK) return r;
        dfree(R.cs_alt);
        HIPCHK(hipMalloc((void**)&R.cs_alt, (size_t)need * sizeof(uint32_t)));
        R.cs_alt_cap = need;
    }
    const SizesIn sizes{R.left >= 0 ? R.msg_in[0] : nullptr, R.right >= 0 ? R.msg_in[1] : nullptr, nl_ub, nr_ub,
                        ctx->capacity};
    const AsmSrc src{ctx->pos, ctx->vel, ctx->id, ctx->sk_cur, ctx->keys, 0,
                     R.left >= 0 ? (const float4*)(R.msg_in[0] + MSG_HDR_F4) : nullptr,
                     R.right >= 0 ? (const float4*)(R.msg_in[1] + MSG_HDR_F4) : nullptr,
                     ctx->keys2, ctx->vals, nl_ub, (int32_t)n_ub - nr_ub, R.dz};
    const MoverSink mv{ctx->keys2, ctx->mv_count + ctx->mv_par, ctx->mv_mi, ctx->mv_mk, ctx->mv_mo,
                       (uint32_t)std::max(ctx->capacity, 1), &R.dz->flags};
    CsOld csp;
    csp.cs = R.cs_alt;
    csp.src = ctx->cs;
    csp.ncells = ctx->grid.ncells;
    csp.gyz = gyz(ctx);
    csp.gx = (uint32_t)ctx->grid.gx;
    csp.has_left = ctx->has_left ? 1 : 0;
    csp.has_right = ctx->has_right ? 1 : 0;
    launch_slab_rec(src, (int32_t)n_ub, ctx->grid, (uint32_t)ctx->grid.cx0 * gyz(ctx), ctx->vals, ctx->keys2, mv, R.comm,
                    &sizes, csp);
    HIPCHK(hipGetLastError());
    R.pre_rec = true;
    ctx->dz_next = true;
    return SPH_OK;
}

int phase_finish(Multi& M, RankState& R, float dt, int64_t step, bool early) {
    sph_ctx* ctx = R.c;
    HIPCHK(hipSetDevice(ctx->device));
    const bool halo = R.left >= 0 || R.right >= 0;
    const bool on_comm = early && halo;
    hipStream_t s = on_comm ? R.comm : ctx->stream;
    if (halo && !on_comm) HIPCHK(hipStreamWaitEvent(s, R.ev_bdone, 0));
    swap_sv(ctx);
    ctx->keys_valid = true;
    ctx->steps++;
    ctx->sim_time += (double)dt;
    const int k = (int)(step % LAG_SLOTS);
    // the count bins the boundary pass filled and the pack read (on this same stream) are cleared for the next use
    const bool clear = on_comm && R.ebins_used;
    // flags: a local group's host ORs its ranks' own. RCCL ranks: every rank's sticky SZ_* flags as of its density
    // pass, one word per bit, max-reduced, i.e. each bit is the OR over the ranks (the failure message names every
    // rank's cause); the step's lag record carries them, so every rank stops two steps on, at the same step. The
    // all-reduce runs behind this step's exchanges (early sends: at the end of the comm stream's work), where no pass
    // of the step waits on it; it sat between the ρ halo and the boundary force pass before. It stays per step: with
    // a reduction only every few steps, ranks ran on for up to that many steps on a state whose sizes had overflowed,
    // and a two-rank overflow run did not finish (tests/test_gpu_rccl.py).
    const bool gflags = M.mode == 2 && M.world > 1;
    if (gflags) NCCLCHK(ncclAllReduce(R.cnt_dev + 4, R.cnt_dev + 4, SZ_BITS, ncclUint32, ncclMax, M.comm, s));
    launch_slab_lag(R.dz, ctx->has_left ? 1 : 0, ctx->has_right ? 1 : 0, totals_slot(ctx, step),
                    R.left >= 0 ? R.rho_in[0] : nullptr, R.right >= 0 ? R.rho_in[1] : nullptr,
                    gflags ? R.cnt_dev + 4 : nullptr, R.lag + k * LAG_WORDS, s, clear ? R.ebins : nullptr,
                    clear ? 2 * R.nb_send : 0);
    R.ebins_used = false;
    if (halo) HIPCHK(hipEventRecord(R.lag_ev[k], s));   // read two steps on
    if (on_comm) {
        int r = issue_next_rec(M, R);
        if (r != SPH_OK) return r;
        HIPCHK(hipEventRecord(R.ev_sent, s));
        R.sent_pending = true;
    }
    R.cin_hist[k] = R.c1i[0] + R.c1i[1];
    R.n_prev_ub = R.n_ub;
    R.since_cut++;
    ctx->dz_ahead = true;   // o0 / o1 / n / rng on the host are last step's until slab_sync_ranges
    HIPCHK(hipGetLastError());
    return SPH_OK;
}

// The main streams wait for the comm-stream work of the last step (its boundary pass, early sends and bookkeeping):
// at the next step's start, at the end of every sph_step call (so reads, kicks and re-cuts see the whole step), and
// before a host-side state change.
int multi_join(Multi& M) {
    for (auto& R : M.ranks) {
        if (!R.sent_pending) continue;
        sph_ctx* ctx = R.c;
        HIPCHK(hipSetDevice(ctx->device));
        HIPCHK(hipStreamWaitEvent(ctx->stream, R.ev_sent, 0));
        R.sent_pending = false;
    }
    return SPH_OK;
}

// Early sends for the next step: every rank decides alike from state all ranks share (the cut age, the re-balancing
// schedule, the cuts, the re-sort mode), so the exchanges issued early are matched on every rank.
bool early_next(const Multi& M) {
    if (M.world < 2 || M.ranks.empty()) return false;
    if (M.hold_early > 0 || M.no_early) return false;
    const RankState& R0 = M.ranks[0];
    if (R0.since_cut + 1 < 3) return false;   // the next step sizes its messages exactly
    if (M.rebalance_every > 0 && (M.steps + 1) % M.rebalance_every == 0) return false;   // it may re-cut
    if (R0.c->resort_mode == 0) return false;   // no jump guard anywhere
    for (const sph_slab& c : M.cuts)
        if (c.cx_hi - c.cx_lo < 4) return false;
    return true;
}

// ---------------------------------------------------------------- re-balancing
int rebalance(Multi& M, sph_ctx* pctx) {
    sph_ctx* ctx = pctx;
    const int G = global_columns(M.ranks[0].c->prm);
    // hist[G]: ranks that failed to read their counts (a flagged step): over RCCL every rank still joins
    // the all-reduce, so all of them learn of the failure together and none waits in a collective alone
    std::vector<int64_t> hist(G + 1, 0), part(G);
    int local_rc = SPH_OK;
    std::string local_err;
    for (auto& R : M.ranks) {
        int r = sync_dz(R);
        if (r == SPH_OK) r = sph_slab_column_counts(R.c, part.data(), G);
        if (r != SPH_OK) {
            if (M.mode != 2) return fail(ctx, r, "%s", R.c->err.c_str());
            local_rc = r;
            local_err = R.c->err;
            hist[G] += 1;
            break;
        }
        for (int c = 0; c < G; ++c) hist[c] += part[c];
    }
    if (M.mode == 2 && M.world > 1) {
        sph_ctx* rc = M.ranks[0].c;
        HIPCHK(hipSetDevice(rc->device));
        if (M.hist_cap < G + 1) {
            dfree(M.hist_dev);
            HIPCHK(hipMalloc((void**)&M.hist_dev, (size_t)(G + 1) * sizeof(int64_t)));
            M.hist_cap = G + 1;
        }
        HIPCHK(hipMemcpyAsync(M.hist_dev, hist.data(), (size_t)(G + 1) * 8, hipMemcpyHostToDevice, rc->stream));
        NCCLCHK(ncclAllReduce(M.hist_dev, M.hist_dev, (size_t)(G + 1), ncclInt64, ncclSum, M.comm, rc->stream));
        HIPCHK(hipMemcpyAsync(hist.data(), M.hist_dev, (size_t)(G + 1) * 8, hipMemcpyDeviceToHost, rc->stream));
        HIPCHK(hipStreamSynchronize(rc->stream));
    }
    if (local_rc != SPH_OK) return fail(ctx, local_rc, "%s", local_err.c_str());
    if (hist[G] > 0)
        return fail(ctx, SPH_ERR_CAPACITY, "re-balancing at step %lld: %lld rank(s) reported a flagged slab step",
                    (long long)M.steps, (long long)hist[G]);
    hist.resize(G);
    const std::vector<sph_slab> nc = rebalance_cuts(M.cuts, hist);
    bool changed = false;
    for (int r = 0; r < M.world; ++r) changed |= nc[r].cx_lo != M.cuts[r].cx_lo || nc[r].cx_hi != M.cuts[r].cx_hi;
    if (!changed) return SPH_OK;
    M.cuts = nc;
    M.rebalances++;
    M.early = false;
    for (auto& R : M.ranks) R.pre_rec = R.c->dz_next = false;
    for (auto& R : M.ranks) {
        int r = sph_slab_recut(R.c, &M.cuts[R.rank]);
        if (r != SPH_OK) return r;
        R.since_cut = 0;
    }
    return SPH_OK;
}

// SPH_FLAG_VALIDATE, after the assemble: the sizes the density and force passes will use
int validate_mid(Multi& M, sph_ctx* pctx) {
    for (auto& R : M.ranks) {
        sph_ctx* ctx = R.c;
        HIPCHK(hipSetDevice(ctx->device));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        SlabSizes h;
        HIPCHK(hipMemcpy(&h, R.dz, sizeof h, hipMemcpyDeviceToHost));
        const uint32_t* v = h.pick;   // the column starts every kernel of the rest of the step reads
        bool ok = h.flags == 0 && h.n <= (uint32_t)ctx->capacity && (int64_t)h.n <= R.n_ub && h.nl <= (uint32_t)R.c1i[0] &&
                  h.nr <= (uint32_t)R.c1i[1] && v[5] <= h.n &&
                  v[2] - v[1] <= (uint32_t)std::max(R.c2o[0], 0) + (R.left < 0 ? h.n : 0) &&
                  v[4] - v[3] <= (uint32_t)std::max(R.c2o[1], 0) + (R.right < 0 ? h.n : 0);
        for (int k = 0; k < 5; ++k) ok = ok && v[k] <= v[k + 1];
        // the cell-start table the neighbour passes will walk: monotone, within the assembled slots
        std::vector<uint32_t> cs(ctx->grid.ncells + 2);
        HIPCHK(hipMemcpy(cs.data(), ctx->cs, cs.size() * 4, hipMemcpyDeviceToHost));
        int64_t bad_at = -1;
        for (size_t k = 0; k + 1 < cs.size() && bad_at < 0; ++k)
            if (cs[k] > cs[k + 1] || cs[k + 1] > h.n) bad_at = (int64_t)k;   // h.n: the assembled slots
        // cs[ncells]: the slots kept (the dropped ones, which left the window, sort after it)
        if (cs[0] != 0 || cs[ctx->grid.ncells] != v[5]) bad_at = bad_at < 0 ? (int64_t)ctx->grid.ncells : bad_at;
        if (bad_at >= 0)
            return fail(pctx, SPH_ERR_STATE, "validate(mid) rank %d step %lld: cell starts broken at %lld (%u %u, n %u, ncells %u)",
                        R.rank, (long long)M.steps, (long long)bad_at, cs[bad_at], cs[bad_at + 1], h.n, ctx->grid.ncells);
        if (!ok)
            return fail(pctx, SPH_ERR_STATE,
                        "validate(mid) rank %d step %lld: flags %u n %u (ub %lld) picks %u %u %u %u %u %u "
                        "nl %u nr %u no %u c1i %d %d c2o %d %d",
                        R.rank, (long long)M.steps, h.flags, h.n, (long long)R.n_ub, v[0], v[1], v[2], v[3], v[4], v[5],
                        h.nl, h.nr, h.no, R.c1i[0], R.c1i[1], R.c2o[0], R.c2o[1]);
    }
    return SPH_OK;
}

int multi_one_step(Multi& M, sph_ctx* pctx, float dt) {
    int r = multi_join(M);
    if (r != SPH_OK) return r;
    if (M.rebalance_every > 0 && M.world > 1 && M.steps > 0 && M.steps % M.rebalance_every == 0) {
        r = rebalance(M, pctx);
        if (r != SPH_OK) return r;
    }
    // exact sizes for three steps after a cut: the lagged counts of step s come from step s - 2, and the
    // first step after a re-cut carries the migration to the new cut, not the new steady halo
    const bool exact = M.ranks[0].since_cut < 3;   // the same on every rank
    // early: this step's messages were packed and exchanged during the previous step (never on an exact step)
    const bool early = M.early && !exact;
    M.early = false;
    if (!early)
        for (auto& R : M.ranks)
            if ((r = phase_count(R, exact, M.steps)) != SPH_OK) return r;
    if (exact) {
        if ((r = exchange_counts(M, pctx, M.steps)) != SPH_OK) return r;
        for (auto& R : M.ranks) R.g2[0] = R.g2[1] = 0;   // no lagged column counts of the new cut yet: grids of n_ub
    } else {
        // an overflow flagged two steps ago (or earlier; flags are sticky) stops every rank at this same
        // step, before any exchange: over RCCL the lag record holds the flags OR-reduced over all ranks
        // (phase_finish), in a local group the host ORs its ranks' own
        uint32_t flags = 0;
        for (auto& R : M.ranks) {
            if (R.left < 0 && R.right < 0) continue;
            const uint32_t* L = lag_slot(R, M.steps - 2, R.c, &r);
            if (r != SPH_OK) return r;
            flags |= L[9];
        }
        if (flags)
            return fail(pctx, SPH_ERR_CAPACITY, "slab step %lld: a rank flagged%s%s%s%s%s%s (flags %#x, seen two steps on)",
                        (long long)M.steps, (flags & SZ_OVF_MSG) ? " a halo message overflow" : "",
                        (flags & SZ_OVF_CAP) ? " slots over capacity" : "",
                        (flags & SZ_RHO_MISMATCH) ? " a ghost density count mismatch" : "",
                        (flags & SZ_OVF_MOVERS) ? " a mover list / re-sort destination out of range" : "",
                        (flags & SZ_JUMP) ? " a particle that left the held columns in one step" : "",
                        (flags & SZ_JUMP_EARLY) ? " a particle that moved two or more columns in one step" : "", flags);
        for (auto& R : M.ranks) {
            if (R.left < 0 && R.right < 0) continue;   // no messages: nothing to size
            // the counts of two steps before: both neighbours read the same numbers
            const uint32_t* L = lag_slot(R, M.steps - 2, R.c, &r);
            if (r != SPH_OK) return r;
            R.c1o[0] = R.left >= 0 ? cap_of(M, L[0]) : 0;
            R.c1o[1] = R.right >= 0 ? cap_of(M, L[1]) : 0;
            R.c1i[0] = R.left >= 0 ? cap_of(M, L[2]) : 0;
            R.c1i[1] = R.right >= 0 ? cap_of(M, L[3]) : 0;
            R.c2o[0] = R.left >= 0 ? cap_of(M, L[4]) : 0;
            R.c2o[1] = R.right >= 0 ? cap_of(M, L[5]) : 0;
            R.c2i[0] = R.left >= 0 ? cap_of(M, L[6]) : 0;
            R.c2i[1] = R.right >= 0 ? cap_of(M, L[7]) : 0;
            R.g2[0] = R.left >= 0 ? cap_of(M, L[10]) : 0;
            R.g2[1] = R.right >= 0 ? cap_of(M, L[11]) : 0;
            // slot bound: the assembled count two steps ago plus every record received since
            const int64_t km1 = (M.steps - 1) % LAG_SLOTS;
            R.n_prev_ub = std::min<int64_t>(R.n_prev_ub, (int64_t)L[8] + R.cin_hist[km1]);
        }
    }
    if (early) {   // the messages the previous step sent (multi_join waited for them): their capacities
        for (auto& R : M.ranks) {
            if (R.left < 0 && R.right < 0) continue;
            for (int sd = 0; sd < 2; ++sd) {
                R.c1o[sd] = R.e_c1o[sd];
                R.c1i[sd] = R.e_c1i[sd];
            }
        }
    } else {
        for (auto& R : M.ranks)
            if ((r = phase_pack(R, M, M.steps)) != SPH_OK) return r;
        if ((r = exchange1(M)) != SPH_OK) return r;
    }
    for (auto& R : M.ranks)
        if ((r = phase_assemble(R, exact)) != SPH_OK) return r;
    if ((pctx->cfg.flags & SPH_FLAG_VALIDATE) && (r = validate_mid(M, pctx)) != SPH_OK) return r;
    for (auto& R : M.ranks)
        if ((r = phase_density(R, M)) != SPH_OK) return r;
    if (M.world > 1 && (r = exchange2_start(M)) != SPH_OK) return r;
    const bool nxt = early_next(M);   // decided before the force passes, whose ranges depend on it
    for (auto& R : M.ranks)
        if ((r = phase_interior(R, dt, nxt)) != SPH_OK) return r;
    for (auto& R : M.ranks)
        if ((r = phase_boundary(R, M, dt, nxt)) != SPH_OK) return r;
    if (nxt && (r = exchange1_early(M)) != SPH_OK) return r;
    for (auto& R : M.ranks)
        if ((r = phase_finish(M, R, dt, M.steps, nxt)) != SPH_OK) return r;
    M.early = nxt;
    if (M.hold_early > 0) M.hold_early--;
    M.steps++;
    return SPH_OK;
}

int rank_setup(Multi& M, RankState& R, sph_ctx* c, int rank) {
    R.c = c;
    R.rank = rank;
    R.world = M.world;
    R.left = rank > 0 ? rank - 1 : -1;
    R.right = rank + 1 < M.world ? rank + 1 : -1;
    return rank_init(R);
}

}  // namespace

void multi_free(sph_ctx* ctx) {
    Multi* M = ctx->mg;
    if (!M) return;
    if (g_ht.on && g_ht.steps > 0)
        std::fprintf(stderr, "[host] world %d ranks here %zu: %lld steps, %.1f us/step on the host, %.1f us/step of it blocked on "
                     "lag events\n", M->world, M->ranks.size(), (long long)g_ht.steps, 1e6 * g_ht.total / (double)g_ht.steps,
                     1e6 * g_ht.wait / (double)g_ht.steps);
    for (auto& R : M->ranks) rank_free(R);
    if (M->hist_dev) (void)hipFree(M->hist_dev);
    if (M->comm) (void)ncclCommDestroy(M->comm);
    // in reverse: under SPH_DEBUG_SERIAL_GROUP the later slabs borrow slab 0's stream
    for (auto k = M->kids.rbegin(); k != M->kids.rend(); ++k) sph_destroy(*k);
    delete M;
    ctx->mg = nullptr;
}

bool is_group(const sph_ctx* ctx) { return ctx->mg && ctx->mg->mode == 1; }
// The next step packs and exchanges its messages itself: the ones sent during the last step hold the state
// before the change (over RCCL every rank must make the same change between the same steps: the exchanges pair up).
// The step after the change runs without early sends too, so its force passes keep the graceful column-jump guard
// (an external velocity change is what can move a particle two columns in one step).
int multi_state_changed(sph_ctx* ctx) {
    if (!ctx || !ctx->mg) return SPH_OK;
    ctx->mg->early = false;
    ctx->mg->hold_early = 1;
    return multi_join(*ctx->mg);
}

int multi_params_changing(sph_ctx* ctx, const sph_params& next) {
    if (!ctx || !ctx->mg || !ctx->mg->ready) return SPH_OK;
    const sph_params& o = ctx->prm;
    // the grid (cell size 2h, the box) sizes every slab's window, cell-start tables and message columns
    if (next.h != o.h || next.box[0] != o.box[0] || next.box[1] != o.box[1] || next.box[2] != o.box[2])
        return fail(ctx, SPH_ERR_STATE, "multi-GPU context: h and the box are fixed once the scenario is initialised "
                    "(sph_init_scenario again)");
    // the messages sent during the last step and the pre-issued record kernel stay valid (same particles, same
    // grid); the next step's force passes keep the graceful column-jump guard
    return multi_state_changed(ctx);
}

std::vector<sph_ctx*> multi_kids(const sph_ctx* ctx) { return ctx->mg ? ctx->mg->kids : std::vector<sph_ctx*>{}; }

int multi_create_group(sph_ctx* ctx) {
    Multi* M = new Multi();
    M->mode = 1;
    M->world = ctx->cfg.ndev;
    ctx->mg = M;
    return SPH_OK;
}

// Switches that decide the exchange sequence, the message sizes or the cuts, read from the environment once per
// scenario. Over RCCL every rank must hold the same values: a rank alone with SPH_NO_EARLY_SENDS would issue its
// exchanges at other points of the step than its neighbours, and both would wait in mismatched send / receive
// sequences until the watchdog fired. So they are compared with one all-reduce (max of v and of -v) and a mismatch
// fails every rank's init alike. Returns SPH_DEBUG_CUT_SKEW.
int read_switches(Multi& M, sph_ctx* ctx, int* skew) {
    M.no_early = env_on("SPH_NO_EARLY_SENDS");
    const char* mc = std::getenv("SPH_DEBUG_MSG_CAP");
    M.msg_cap = mc ? std::max(0, std::atoi(mc)) : 0;
    const char* sk = std::getenv("SPH_DEBUG_CUT_SKEW");
    *skew = sk ? std::atoi(sk) : 0;
    if (M.mode != 2 || M.world < 2) return SPH_OK;
    int32_t v[6] = {M.no_early ? 1 : 0, M.msg_cap, *skew, M.no_early ? -1 : 0, -M.msg_cap, -*skew};
    // The context's small scratch (sdev[0..6): the step's column-start picks, rewritten by the first sort), not an
    // allocation: a rank whose allocation failed would return before the all-reduce its peers then wait in. Every
    // rank enters the all-reduce, a failed copy included, and fails after it.
    int32_t* d = (int32_t*)ctx->sdev;
    hipError_t he = hipMemcpy(d, v, sizeof v, hipMemcpyHostToDevice);
    const ncclResult_t nr = ncclAllReduce(d, d, 6, ncclInt32, ncclMax, M.comm, ctx->stream);
    if (nr == ncclSuccess) {
        const hipError_t h2 = hipMemcpyAsync(v, d, sizeof v, hipMemcpyDeviceToHost, ctx->stream);
        const hipError_t h3 = hipStreamSynchronize(ctx->stream);
        if (he == hipSuccess) he = h2 != hipSuccess ? h2 : h3;
    }
    if (nr != ncclSuccess) return fail(ctx, SPH_ERR_HIP, "switch agreement: %s", ncclGetErrorString(nr));
    if (he != hipSuccess) return fail(ctx, SPH_ERR_HIP, "switch agreement: %s", hipGetErrorString(he));
    for (int k = 0; k < 3; ++k)
        if (v[k] != -v[k + 3])
            return fail(ctx, SPH_ERR_INVALID, "ranks disagree on SPH_NO_EARLY_SENDS / SPH_DEBUG_MSG_CAP / "
                        "SPH_DEBUG_CUT_SKEW (max %d %d %d, min %d %d %d)", v[0], v[1], v[2], -v[3], -v[4], -v[5]);
    return SPH_OK;
}

// Test knob (tests/test_gpu_multi.py): SPH_DEBUG_CUT_SKEW=k moves every inner cut k columns right of the equal-count
// position (every slab keeps at least one column), so the first re-balancing re-cuts the slabs of a full-size run.
void skew_cuts(std::vector<sph_slab>& cuts, int k) {
    if (k == 0) return;
    for (size_t r = 0; r + 1 < cuts.size(); ++r) {
        const int c = std::max(cuts[r].cx_lo + 1, std::min(cuts[r].cx_hi + k, cuts[r + 1].cx_hi - 1));
        cuts[r].cx_hi = c;
        cuts[r + 1].cx_lo = c;
    }
}

// Distribute a scenario over a local group: equal-count cuts, one slab context per GPU.
int multi_init_scenario(sph_ctx* ctx, const sph_scenario* sc) {
    Multi& M = *ctx->mg;
    if (sc->dim != ctx->cfg.dim) return fail(ctx, SPH_ERR_INVALID, "scenario dim %d != context dim %d", sc->dim, ctx->cfg.dim);
    if (!ctx->params_set) return fail(ctx, SPH_ERR_STATE, "sph_set_params first");
    const sph_params& p = ctx->prm;
    const int G = global_columns(p);
    if (G < 2 * M.world) return fail(ctx, SPH_ERR_INVALID, "%d columns cannot be cut into %d slabs", G, M.world);
    const std::vector<int64_t> per = lattice_columns(*sc, p);
    int skew = 0;
    if (int r = read_switches(M, ctx, &skew)) return r;
    M.cuts = balanced_cuts(per, M.world);
    skew_cuts(M.cuts, skew);
    M.n_total = (int64_t)sc->nx * sc->ny * (sc->dim == 3 ? sc->nz : 1);
    const int64_t per_x = (int64_t)sc->ny * (sc->dim == 3 ? sc->nz : 1);
    int64_t maxcol = 0;
    for (int64_t v : per) maxcol = std::max(maxcol, v * per_x);
    auto need_cap = [&](int r) {   // an even share or this rank's initial share, plus a halo column per side, x1.5
        int64_t own = 0;
        for (int c = M.cuts[r].cx_lo; c < M.cuts[r].cx_hi; ++c) own += per[c] * per_x;
        const double share = std::max((double)M.n_total / M.world, (double)own);
        return (int64_t)((share + 2.0 * (double)maxcol) * 1.5) + 4096;
    };
    for (auto& R : M.ranks) rank_free(R);
    M.ranks.clear();
    {
        for (auto k = M.kids.rbegin(); k != M.kids.rend(); ++k) sph_destroy(*k);
        M.kids.clear();
        int nvis = 0;
        HIPCHK(hipGetDeviceCount(&nvis));
        for (int r = 0; r < M.world; ++r) {
            const int64_t cap = std::max<int64_t>(need_cap(r), ctx->cfg.capacity);
            if (cap > INT32_MAX) return fail(ctx, SPH_ERR_CAPACITY, "slab %d needs %lld slots", r, (long long)cap);
            sph_config kc = ctx->cfg;
            kc.ndev = 1;
            kc.capacity = (int32_t)cap;
            sph_ctx* k = nullptr;
            int rc = sph_create(&kc, (ctx->device + r) % nvis, &k);
            if (rc != SPH_OK) return fail(ctx, rc, "slab context %d on device %d", r, (ctx->device + r) % nvis);
            M.kids.push_back(k);
        }
        // measurement knob (scripts/slab_overhead.py --serial): every slab of a one-device group launches on
        // slab 0's stream, so the slabs run one after another and the group's step time is the sum of the
        // per-slab step costs instead of an overlapped bound. 1: every slab's comm work on slab 0's comm stream as
        // well (two streams in all); 2: each slab keeps its own comm stream, as on the GPUs of a real group (run
        // with GPU_MAX_HW_QUEUES >= slabs + 2, or streams share hardware queues and order unrelated work)
        const char* ser = std::getenv("SPH_DEBUG_SERIAL_GROUP");
        const int ser_mode = ser ? std::atoi(ser) : 0;
        if (ser_mode != 0) {
            for (int r = 1; r < M.world; ++r) {
                if (M.kids[r]->device != M.kids[0]->device)
                    return fail(ctx, SPH_ERR_INVALID, "SPH_DEBUG_SERIAL_GROUP needs every slab on one device");
                const int rc = sph_set_stream(M.kids[r], M.kids[0]->stream);
                if (rc != SPH_OK) return fail(ctx, rc, "serial group: slab %d stream", r);
            }
        }
        for (int r = 0; r + 1 < M.world; ++r) {   // halo neighbours r, r + 1
            const int rc = enable_peers(ctx, M.kids[r]->device, M.kids[r + 1]->device);
            if (rc != SPH_OK) return rc;
        }
        M.ranks.resize(M.world);
        for (int r = 0; r < M.world; ++r) {
            sph_ctx* k = M.kids[r];
            int rc = sph_set_params(k, &p);
            if (rc == SPH_OK) rc = sph_slab_set(k, &M.cuts[r]);
            if (rc == SPH_OK) rc = sph_slab_init_scenario(k, sc);
            if (rc == SPH_OK) rc = rank_setup(M, M.ranks[r], k, r);
            if (rc == SPH_OK) rc = put_dz(M.ranks[r]);
            if (rc != SPH_OK) return fail(ctx, rc, "slab %d: %s", r, sph_last_error(k));
        }
        // ... and every slab's halo work on slab 0's comm stream: two streams in all, as on each GPU of a real
        // group (more streams than the device's hardware queues would share queues and order unrelated work)
        if (ser_mode == 1) {
            HIPCHK(hipDeviceSynchronize());
            for (int r = 1; r < M.world; ++r) {
                RankState& R = M.ranks[r];
                HIPCHK(hipStreamDestroy(R.comm));
                R.comm = M.ranks[0].comm;
                R.comm_borrowed = true;
            }
        }
    }
    M.steps = 0;
    M.ready = true;
    return SPH_OK;
}

// SPH_FLAG_VALIDATE: after every step, one wait and a check of every rank's device sizes
int validate(Multi& M, sph_ctx* pctx) {
    for (auto& R : M.ranks) {
        sph_ctx* ctx = R.c;
        HIPCHK(hipSetDevice(ctx->device));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        HIPCHK(hipStreamSynchronize(R.comm));
        SlabSizes h;
        HIPCHK(hipMemcpy(&h, R.dz, sizeof h, hipMemcpyDeviceToHost));
        const uint32_t cap = (uint32_t)ctx->capacity;
        // the slots of the last step's order; SlabSizes.n already holds the next layout's when its record kernel ran
        const uint32_t n = R.pre_rec ? h.rg[5] : h.n;
        bool ok = h.flags == 0 && h.n <= cap && n <= cap && h.o0 <= h.o1 && h.o1 <= n && h.rg[0] <= h.rg[1] &&
                  h.rg[1] <= h.rg[3] && h.rg[3] <= h.rg[5] && h.rg[5] <= n && (int64_t)n <= R.n_ub;
        for (int k = 0; k < 6; k += 2) ok = ok && h.fr[k] <= h.fr[k + 1] && h.fr[k + 1] <= n;
        if (!ok)
            return fail(pctx, SPH_ERR_STATE,
                        "validate rank %d step %lld: flags %u n %u (ub %lld, cap %u) o %u..%u rg %u %u %u %u %u %u "
                        "fr %u %u %u %u %u %u nl %u nr %u no %u c1i %d %d c2i %d %d",
                        R.rank, (long long)M.steps, h.flags, h.n, (long long)R.n_ub, cap, h.o0, h.o1, h.rg[0], h.rg[1],
                        h.rg[2], h.rg[3], h.rg[4], h.rg[5], h.fr[0], h.fr[1], h.fr[2], h.fr[3], h.fr[4], h.fr[5], h.nl,
                        h.nr, h.no, R.c1i[0], R.c1i[1], R.c2i[0], R.c2i[1]);
    }
    return SPH_OK;
}

int multi_step(sph_ctx* ctx, float dt, int32_t nsteps) {
    Multi& M = *ctx->mg;
    if (!M.ready) return fail(ctx, SPH_ERR_STATE, "multi-GPU context: sph_init_scenario first");
    for (int32_t k = 0; k < nsteps; ++k) {
        if ((ctx->cfg.flags & SPH_FLAG_VALIDATE) && M.steps > 0) {
            int r = validate(M, ctx);
            if (r != SPH_OK) return r;
        }
        const double t0 = g_ht.on ? now_s() : 0.0;
        int r = multi_one_step(M, ctx, dt);
        if (g_ht.on) {
            g_ht.total += now_s() - t0;
            g_ht.steps++;
        }
        static const bool trace = std::getenv("SPH_TRACE_LAG") != nullptr;
        if (r == SPH_OK && trace && (ctx->cfg.flags & SPH_FLAG_VALIDATE))
            for (auto& R : M.ranks) {
                (void)hipStreamSynchronize(R.c->stream);
                const uint32_t* L = R.lag + ((M.steps - 1) % LAG_SLOTS) * LAG_WORDS;
                std::fprintf(stderr, "[lag] step %lld rank %d: sent %u %u recv %u %u rho sent %u %u recv %u %u n %u flags %u | "
                             "c1o %d %d c1i %d %d n_ub %lld since_cut %lld\n", (long long)(M.steps - 1), R.rank, L[0], L[1],
                             L[2], L[3], L[4], L[5], L[6], L[7], L[8], L[9], R.c1o[0], R.c1o[1], R.c1i[0], R.c1i[1],
                             (long long)R.n_ub, (long long)R.since_cut);
            }
        if (r != SPH_OK) {
            (void)multi_join(M);
            if (M.mode == 1)   // a slab context's message on the group
                for (auto& R : M.ranks)
                    if (R.c && !R.c->err.empty()) ctx->err = R.c->err;
            return r;
        }
    }
    int r = multi_join(M);
    if (r != SPH_OK) return r;
    if (M.mode == 1) {
        ctx->steps = M.ranks[0].c->steps;
        ctx->sim_time = M.ranks[0].c->sim_time;
    }
    return SPH_OK;
}

// owned particles of every local rank -> index-order host arrays (comps of the 8-float record)
int multi_read(sph_ctx* ctx, int field, float* dst, int32_t count) {
    Multi& M = *ctx->mg;
    if (!M.ready) return fail(ctx, SPH_ERR_STATE, "no scenario");
    if (count < M.n_total) return fail(ctx, SPH_ERR_INVALID, "count %d < particles %lld", count, (long long)M.n_total);
    std::vector<float> rec;
    int64_t seen = 0;
    for (auto& R : M.ranks) {
        int r = sync_dz(R);
        if (r != SPH_OK) return fail(ctx, r, "%s", R.c->err.c_str());
        const int32_t no = R.c->o1 - R.c->o0;
        rec.resize((size_t)std::max(no, 1) * 8);
        int32_t got = 0;
        r = sph_slab_read_owned(R.c, rec.data(), no, &got);
        if (r != SPH_OK) return fail(ctx, r, "%s", R.c->err.c_str());
        for (int32_t i = 0; i < got; ++i) {
            const float* q = rec.data() + 8 * (size_t)i;
            int32_t id;
            std::memcpy(&id, q + 6, 4);
            if (id < 0 || id >= count) return fail(ctx, SPH_ERR_STATE, "particle id %d out of range", id);
            if (field == 0) { dst[3 * (size_t)id] = q[0]; dst[3 * (size_t)id + 1] = q[1]; dst[3 * (size_t)id + 2] = q[2]; }
            if (field == 1) { dst[3 * (size_t)id] = q[3]; dst[3 * (size_t)id + 1] = q[4]; dst[3 * (size_t)id + 2] = q[5]; }
            if (field == 2) dst[id] = q[7];
        }
        seen += got;
    }
    if (seen != M.n_total) return fail(ctx, SPH_ERR_STATE, "ranks own %lld particles, expected %lld", (long long)seen, (long long)M.n_total);
    return SPH_OK;
}

}  // namespace sph

using namespace sph;

extern "C" {

int sph_comm_unique_id(sph_comm_id* out) {
    if (!out) return SPH_ERR_INVALID;
    static_assert(sizeof(sph_comm_id) == sizeof(ncclUniqueId), "sph_comm_id is an ncclUniqueId");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return SPH_ERR_HIP;
    std::memcpy(out, &id, sizeof id);
    return SPH_OK;
}

int sph_comm_init(sph_ctx* ctx, const sph_comm_id* id, int32_t nranks, int32_t rank) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return SPH_ERR_INVALID;
    if (is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "the multi-GPU step is Model S only");
    if (ctx->mg) return fail(ctx, SPH_ERR_STATE, "context already multi-GPU");
    HIPCHK(hipSetDevice(ctx->device));
    Multi* M = new Multi();
    M->mode = 2;
    M->world = nranks;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    const ncclResult_t r = ncclCommInitRank(&M->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete M;
        return fail(ctx, SPH_ERR_HIP, "ncclCommInitRank(%d of %d): %s", rank, nranks, ncclGetErrorString(r));
    }
    M->ranks.resize(1);
    M->ranks[0].rank = rank;
    ctx->mg = M;
    return SPH_OK;
}

int sph_set_rebalance(sph_ctx* ctx, int32_t every) {
    if (!ctx || every < 0) return SPH_ERR_INVALID;
    if (!ctx->mg) return fail(ctx, SPH_ERR_STATE, "not a multi-GPU context");
    ctx->mg->rebalance_every = every;
    return SPH_OK;
}

int sph_get_decomposition(sph_ctx* ctx, sph_decomp* out) {
    if (!ctx || !out) return SPH_ERR_INVALID;
    std::memset(out, 0, sizeof *out);
    if (!ctx->mg) {
        out->world = out->local_ranks = 1;
        out->owned = out->total = ctx->n;
        return SPH_OK;
    }
    Multi& M = *ctx->mg;
    out->world = M.world;
    out->local_ranks = (int32_t)M.ranks.size();
    out->rank = M.ranks.empty() ? 0 : M.ranks[0].rank;
    out->total = M.n_total;
    out->rebalances = M.rebalances;
    if (!M.cuts.empty()) out->cut = M.cuts[out->rank];
    for (auto& R : M.ranks) {
        if (!R.c) continue;
        int r = sync_dz(R);
        if (r != SPH_OK) return r;
        out->owned += R.c->o1 - R.c->o0;
    }
    return SPH_OK;
}

}  // extern "C"

// RCCL rank: this process's slab of the scenario (called by sph_init_scenario)
int sph::multi_init_rank(sph_ctx* ctx, const sph_scenario* sc) {
    Multi& M = *ctx->mg;
    const int rank = M.ranks[0].rank;
    if (sc->dim != ctx->cfg.dim) return fail(ctx, SPH_ERR_INVALID, "scenario dim %d != context dim %d", sc->dim, ctx->cfg.dim);
    if (!ctx->params_set) return fail(ctx, SPH_ERR_STATE, "sph_set_params first");
    const sph_params& p = ctx->prm;
    const int G = global_columns(p);
    if (G < 2 * M.world) return fail(ctx, SPH_ERR_INVALID, "%d columns cannot be cut into %d slabs", G, M.world);
    const std::vector<int64_t> per = lattice_columns(*sc, p);
    int skew = 0;
    if (int r = read_switches(M, ctx, &skew)) return r;
    M.cuts = balanced_cuts(per, M.world);
    skew_cuts(M.cuts, skew);
    M.n_total = (int64_t)sc->nx * sc->ny * (sc->dim == 3 ? sc->nz : 1);
    const int64_t per_x = (int64_t)sc->ny * (sc->dim == 3 ? sc->nz : 1);
    int64_t maxcol = 0, own = 0;
    for (int64_t v : per) maxcol = std::max(maxcol, v * per_x);
    for (int c = M.cuts[rank].cx_lo; c < M.cuts[rank].cx_hi; ++c) own += per[c] * per_x;
    const double share = std::max((double)M.n_total / M.world, (double)own);
    const int64_t cap = (int64_t)((share + 2.0 * (double)maxcol) * 1.5) + 4096;
    if (cap > INT32_MAX) return fail(ctx, SPH_ERR_CAPACITY, "slab needs %lld slots", (long long)cap);
    rank_free(M.ranks[0]);
    if (ctx->slab) {   // a second scenario: start from a plain context again
        ctx->slab = false;
        ctx->grid = ctx->gglobal;
    }
    if (cap > ctx->capacity) {
        int r = sph_resize(ctx, (int32_t)cap);
        if (r != SPH_OK) return r;
    }
    int r = sph_slab_set(ctx, &M.cuts[rank]);
    if (r == SPH_OK) r = sph_slab_init_scenario(ctx, sc);
    if (r == SPH_OK) r = rank_setup(M, M.ranks[0], ctx, rank);
    if (r == SPH_OK) r = put_dz(M.ranks[0]);
    if (r != SPH_OK) return r;
    M.steps = 0;
    M.ready = true;
    return SPH_OK;
}
