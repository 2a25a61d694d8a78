// host.h — host-side state of libsphhip.so: the context behind the C ABI (include/sphhip.h) and the
// helpers the ABI files share (host_ctx.cpp: memory and profiling; host_step.cpp: the per-step
// launch sequences; abi.cpp: the single-domain ABI; abi_slab.cpp: the slab decomposition and
// the multi-GPU step).
//
// Host orchestration of the reference's per-frame GPU work, MI355X-first:
//   ParticleSystemController.Update() (ParticleSystemController.cs:244-351) issues
//   ~9 Dispatches plus two full-buffer H2D clears and two synchronous D2H readbacks every
//   frame. sph_step() issues hash → radix sort → reorder → cell-start → pass 1 → pass 2
//   on one HIP stream with no host synchronisation, no per-step allocation and no
//   readback. Readback is an explicit call (sph_read_*).
// Device memory is owned here and sized once per capacity (InitializeBuffers :373-451).
#pragma once
#include "common.h"
#include "sphhip.h"

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace sph {

struct Multi;   // the multi-GPU step's state (abi_multi.cpp)
// z sub-cells per 2h cell (SPEC_SPH.md §0). 6 trims the neighbour windows closer than 4 (C3: both passes
// −8 us each) while the sub-cell crossings it adds cost the re-sort 2 us; 8 costs it 14 us
// (profiles/r01_zsub_ab.log).
static const int32_t SPH_ZSUB = 6;
// x sub-columns per 2h column for Model S 3D (SPEC_SPH.md §0; 1 or 2). With 2 the neighbour rows are h wide
// in x: 19% fewer candidates per target and pass 2's plane walks better balanced, but measured slower (five
// staging phases, 15 row windows, twice the cells: 0.338 -> 0.404 ms/step from rest, 0.382 -> 0.403
// mid-collapse; DESIGN.md §9, profiles/r03_xsub_ab.log). The environment variable SPH_XSUB (1 or 2) selects
// it per context; the oracle reads the same variable with the same default (tests/test_abi_cpu.py).
#define SPH_XSUB_DEFAULT 1
int32_t model_s_xsub();

struct KStat {
    std::string name;
    int64_t launches = 0;
    double total_ms = 0.0;
    double bytes = 0.0;
    int64_t timed = 0;   // launches whose events were resolved into total_ms
};

struct Pending {
    int k;
    hipEvent_t a, b;
};

}  // namespace sph

struct sph_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    sph_config cfg{};
    sph_params prm{};
    bool params_set = false;
    int32_t capacity = 0;
    int32_t n = 0;
    sph::GridDesc grid{};
    int32_t key_bits = 1;
    sph::SphConst sc{};
    // particle state, cell-sorted slot order; *2 = ping-pong partner
    float4 *pos = nullptr, *vel = nullptr, *pos2 = nullptr, *vel2 = nullptr;
    float4 *omg = nullptr, *rot = nullptr, *aux = nullptr, *omg2 = nullptr, *rot2 = nullptr, *aux2 = nullptr;
    int32_t *id = nullptr, *id2 = nullptr, *mode = nullptr, *mode2 = nullptr;
    float2* rp = nullptr;        // Model S (ρ, P/ρ²)
    int32_t* torque = nullptr;   // Model R int torque of the last step (slot order)
    int32_t* slot_of = nullptr;  // Model R particle index -> slot (bond pass)
    // adhesion bonds (Model R, §8f-1): device SoA, host copy of the ends for the incidence lists
    int32_t nbonds = 0, bond_cap = 0;
    int2* b_ends = nullptr;
    float4 *b_spring = nullptr, *b_relq = nullptr, *b_anc_a = nullptr, *b_anc_b = nullptr;
    int4* b_terms = nullptr;
    uint32_t *b_off = nullptr, *b_ent = nullptr;
    int32_t b_off_cap = 0;
    std::vector<int2> bonds_host;
    std::vector<uint32_t> b_off_host, b_ent_host;
    int32_t b_index_n = -1;      // particle count the incidence lists were built for (-1: stale)
    // sort / grid
    uint32_t *keys = nullptr, *keys2 = nullptr, *vals = nullptr, *vals2 = nullptr;
    uint32_t *hist = nullptr, *bin_total = nullptr;
    uint32_t* cs = nullptr;
    uint32_t cs_cap = 0;
    uint32_t* cs2 = nullptr;   // the incremental re-sort's new cell-start table (swapped with cs)
    uint32_t cs2_cap = 0;
    uint4* gaps = nullptr;       // cell-start long-gap queue
    uint32_t gaps_cap = 0;
    void* staging = nullptr;
    size_t staging_bytes = 0;
    bool keys_valid = false;
    bool dz_next = false;   // multi-GPU step: SlabSizes n / nl / no / nr hold the next step's layout (abi_multi.cpp issue_next_rec)
    int32_t keys_active = -1;
    // incremental re-sort (resort.hip): sorted keys of the current slot order, and scratch
    uint32_t *sk_cur = nullptr, *sk_next = nullptr;
    uint32_t *mv_mi = nullptr, *mv_mk = nullptr, *mv_mo = nullptr, *mv_mx = nullptr, *mv_mos = nullptr;
    uint64_t* mv_ms = nullptr;
    uint32_t* mv_count = nullptr;   // [3] mover counters: Model S and slabs ping-pong over two; Model R cycles three
    int mv_par = 0;                 // counter the next force pass appends into
    uint32_t *mv_mi2 = nullptr, *mv_mk2 = nullptr, *mv_mo2 = nullptr;   // Model R's second mover list (one-launch step)
    bool fz_ready = false;          // the one-launch step's append counter is known to be zero
    int fused_mode = 1;             // env SPH_FUSED: Model R one-launch step, 0 never, 1 up to contact_fused_max()
    bool sk_valid = false;       // sk_cur matches the slot order and cs (set by a Model S sort)
    // env SPH_RESORT: 0 full radix sort every step, 1 (default) incremental re-sort unless the last
    // seen mover count exceeds resort_limit(n), 2 incremental whenever possible (tests)
    int resort_mode = 1;
    int ct_team = 0;                // env SPH_CT_TEAM: Model R lanes per target (0 = by size; tests)
    int small_mode = 1;             // env SPH_SMALL: Model S wave-per-target passes, 0 never, 1 up to SMALL_N (default), 2 always
    // the tiled passes' y-band schedule (schedule.hip): env SPH_SCHED 0 off (default: measured slower),
    // 1 on; rebuilt every SCHED_EVERY steps and whenever the slot count or the grid changed (any table is a partition)
    int sched_mode = 0;
    uint2* sched = nullptr;
    int32_t sched_cap = 0, sched_ent = 0, sched_n = -1;
    bool sched_valid = false;
    uint32_t* mv_host = nullptr;    // pinned, mapped: the mover count of a recent step (k_mv_rank writes it, mv_host_dev)
    uint32_t* mv_host_dev = nullptr;
    bool sorted_full = false;       // this step took the full radix sort (no k_mv_rank: the count is copied back)
    int64_t steps = 0;
    double sim_time = 0.0;
    sph_drag_input drag{-1, {0.f, 0.f, 0.f}, 0.f};
    std::string err;
    bool profiling = false;
    int32_t prof_every = 1;   // profiling: time the launches of one step in prof_every (sph_set_profile_every)
    std::vector<sph::KStat> kstats;
    std::vector<sph::Pending> pending;
    std::vector<hipEvent_t> ev_pool;
    int64_t device_bytes = 0;
    uint32_t* paths = nullptr;   // [24] path counters of the neighbour passes (sph_read_path_counts, _mask_counts;
                                 // [8, 16): lane-utilisation counters of -DSPH_DIAG builds; [16, 24): the re-sort's,
                                 // always counted, sph_read_resort_counts)
    bool count_paths = false;    // armed by the first counter read: counted launches pay for atomics
    uint32_t* hmask = nullptr;   // Model S: HM_WORDS x capacity hit-mask words (pass 1 -> pass 2)
    bool hm_valid = false;       // hmask describes the current slot order (a density pass ran since the last sort)
    // slab decomposition (SPEC_SPH.md §3)
    bool slab = false;
    sph_slab sl{};
    bool has_left = false, has_right = false;
    sph::GridDesc gglobal{};
    int32_t o0 = 0, o1 = 0;      // owned sorted slots
    int32_t rng[10] = {0};
    int32_t send_counts[2] = {0, 0};
    uint32_t* sblk = nullptr;    // compaction block counts [2][nblk]
    uint32_t* sdev = nullptr;    // small device scratch (totals, picks; [8], [9]: cell-start gap counters; [15]: Model R
                                 // radius bound, SDEV_RMAX)
    int gap_par = 0;             // which of sdev[8], sdev[9] the next cell-start call uses
    uint32_t* rng_host = nullptr;   // pinned: column-start picks of the last assemble
    hipEvent_t rng_ev = nullptr;    // recorded after their device->host copy
    bool rng_pending = false;       // rng[] / o0 / o1 not yet updated from rng_host
    int32_t dropped = 0;            // own particles the last assemble dropped (outside the window)
    // asynchronous readback (AsyncGPUReadback, controller:1115-1159): index-order copies on the
    // device, D2H on a side stream into pinned host buffers
    hipStream_t rb_stream = nullptr;
    hipEvent_t rb_src = nullptr, rb_ready = nullptr;
    void* rb_dev[3] = {nullptr, nullptr, nullptr};
    void* rb_host[3] = {nullptr, nullptr, nullptr};
    size_t rb_cap[3] = {0, 0, 0};
    int32_t rb_fields = 0;          // fields of the outstanding request (0: none)
    int32_t rb_count = 0;           // particles it holds
    // multi-GPU (abi_multi.cpp): a local group (sph_config.ndev > 1) or an RCCL rank (sph_comm_init)
    sph::Multi* mg = nullptr;
    sph::SlabSizes* dz = nullptr;   // a rank of the in-library step: its sizes on the device
    bool dz_ahead = false;          // the device sizes are newer than o0 / o1 / n / rng (slab_sync_ranges reads them)
};

namespace sph {

inline int fail(sph_ctx* c, int code, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return code;
}

#define HIPCHK(call)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess) return fail(ctx, SPH_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_)); \
    } while (0)

template <class T>
int dalloc(sph_ctx* ctx, T** p, size_t count) {
    if (*p) { (void)hipFree(*p); *p = nullptr; }
    if (count == 0) return SPH_OK;
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, count * sizeof(T));
    if (e != hipSuccess) return fail(ctx, SPH_ERR_NOMEM, "hipMalloc(%zu): %s", count * sizeof(T), hipGetErrorString(e));
    *p = (T*)q;
    ctx->device_bytes += (int64_t)(count * sizeof(T));
    return SPH_OK;
}

template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

void free_all(sph_ctx* c);
int bit_width(uint32_t v);
inline bool is_contact(const sph_ctx* c) { return c->cfg.model == SPH_MODEL_CONTACT; }
int alloc_particles(sph_ctx* ctx, int32_t cap);
int ensure_cells(sph_ctx* ctx);
int derive(sph_ctx* ctx);
// Every mutation of the particle slots (upload, init, split, index-range set, resize, window change)
// makes the sorted keys, the old-key table of the incremental re-sort and the movers stale: the next
// step runs the full radix sort.
void invalidate_sort(sph_ctx* c);
int kstat_index(sph_ctx* c, const char* name);
hipEvent_t take_event(sph_ctx* c);
void resolve_pending(sph_ctx* c);

// Times a scope of launches when profiling. ext: the scope's kernels launch through SPH_LAUNCH, and the
// events ride in their dispatch packets (common.h LaunchEvents); otherwise the events are recorded around
// the scope on `st` (the stream the scope launches on; default the context's).
struct KTimer {
    sph_ctx* c;
    int k;
    bool ext, on;
    hipStream_t s;
    hipEvent_t a = nullptr;
    LaunchEvents le;
    LaunchEvents* prev = nullptr;
    KTimer(sph_ctx* ctx, const char* name, double bytes, bool ext_events = false, hipStream_t st = nullptr)
        : c(ctx), k(kstat_index(ctx, name)), ext(ext_events),
          on(ctx->profiling && (ctx->prof_every <= 1 || ctx->steps % ctx->prof_every == 0)),
          s(st ? st : ctx->stream) {
        c->kstats[k].launches++;
        c->kstats[k].bytes = bytes;
        if (!on) return;
        a = take_event(c);
        if (ext) {
            le.start = a;
            le.stop = take_event(c);
            prev = g_launch_events;
            g_launch_events = &le;
        } else {
            (void)hipEventRecord(a, s);
        }
    }
    ~KTimer() {
        if (!on) return;
        if (ext) {
            g_launch_events = prev;
            if (le.launches == 0) {   // nothing launched: no time
                c->ev_pool.push_back(le.start);
                c->ev_pool.push_back(le.stop);
                return;
            }
            c->pending.push_back({k, le.start, le.stop});
        } else {
            hipEvent_t b = take_event(c);
            (void)hipEventRecord(b, s);
            c->pending.push_back({k, a, b});
        }
        if (c->pending.size() > 8192) resolve_pending(c);
    }
};

// per-step launch sequences (host_step.cpp)
void swap_sv(sph_ctx* c);
void swap_cs(sph_ctx* c);
int sort_and_reorder(sph_ctx* ctx, int32_t n_active_id, const uint32_t** sorted_keys = nullptr);
// Model S pass 1 -> pass 2 (common.h): the density pass writes the mask (and marks it valid for the
// current slot order); the force pass reads it only while valid, else scans by distance. Every change
// of the slot order (sorts, uploads, assembles, re-cuts) invalidates it.
HitMask hit_mask_write(sph_ctx* ctx);
HitMask hit_mask_read(const sph_ctx* ctx);
inline uint32_t* path_ctr(const sph_ctx* ctx) { return ctx->count_paths ? ctx->paths : nullptr; }
void density_range(sph_ctx* ctx, int32_t b, int32_t e, Sched sch = Sched{});
void force_range(sph_ctx* ctx, int32_t b, int32_t e, float dt, float fext, MoverSink mv = MoverSink{}, Sched sch = Sched{});
ResortScratch resort_scratch(sph_ctx* ctx);
MoverSink mover_sink(sph_ctx* ctx);
uint32_t resort_limit(int32_t n);
float forcing(const sph_ctx* ctx);
int step_wcsph(sph_ctx* ctx, float dt);
void free_bonds(sph_ctx* c);
int32_t contact_active(const sph_ctx* c);
int step_contact(sph_ctx* ctx, float dt);
// slab decomposition (abi_slab.cpp)
int slab_local_grid(sph_ctx* ctx);
int slab_sync_ranges(sph_ctx* ctx);   // waits for the ranges of the last assemble (host or device sized)
int32_t col_start(const sph_ctx* c, int32_t local_col);
int slab_assemble(sph_ctx* ctx, const void* dev_left, int32_t nl, const void* dev_right, int32_t nr, bool force_full);
// multi-GPU step (abi_multi.cpp)
void multi_free(sph_ctx* ctx);
bool is_group(const sph_ctx* ctx);   // sph_config.ndev > 1: the context holds one slab context per GPU
int multi_state_changed(sph_ctx* ctx);   // host-side state changed between steps: no early sends for the next step
// sph_set_params on a multi-GPU context whose scenario is initialised: grid-changing updates are refused
// (re-initialise the scenario), others hold the next step's early sends and drop the pre-issued record kernel
int multi_params_changing(sph_ctx* ctx, const sph_params& next);
int multi_create_group(sph_ctx* ctx);
int multi_init_scenario(sph_ctx* ctx, const sph_scenario* sc);   // local group
int multi_init_rank(sph_ctx* ctx, const sph_scenario* sc);       // RCCL rank
int multi_step(sph_ctx* ctx, float dt, int32_t nsteps);
int multi_read(sph_ctx* ctx, int field, float* dst, int32_t count);   // 0 positions, 1 velocities, 2 density
std::vector<sph_ctx*> multi_kids(const sph_ctx* ctx);

}  // namespace sph
