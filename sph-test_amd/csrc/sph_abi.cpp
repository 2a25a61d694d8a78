// sph_abi.cpp — the C ABI of libsphhip.so (include/sphhip.h) and the host-side step.
//
// Host orchestration of the reference's per-frame GPU work, MI355X-first:
//   ParticleSystemController.Update() (ParticleSystemController.cs:244-351) issues
//   ~9 Dispatches plus two full-buffer H2D clears and two synchronous D2H readbacks every
//   frame. sph_step() issues hash → radix sort → reorder → cell-start → pass 1 → pass 2
//   on one HIP stream with no host synchronisation, no per-step allocation and no
//   readback. Readback is an explicit call (sph_read_*).
// Device memory is owned here and sized once per capacity (InitializeBuffers :373-451).
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

using namespace sph;

// z sub-cells per 2h cell (SPEC_SPH.md §0). 6 trims the neighbour windows closer than 4 (C3: both passes
// −8 us each) while the sub-cell crossings it adds cost the re-sort 2 us; 8 costs it 14 us
// (profiles/r01_zsub_ab.log).
static const int32_t SPH_ZSUB = 6;

namespace {

struct KStat {
    std::string name;
    int64_t launches = 0;
    double total_ms = 0.0;
    double bytes = 0.0;
};

struct Pending {
    int k;
    hipEvent_t a, b;
};

}  // namespace

struct sph_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    sph_config cfg{};
    sph_params prm{};
    bool params_set = false;
    int32_t capacity = 0;
    int32_t n = 0;
    GridDesc grid{};
    int32_t key_bits = 1;
    SphConst sc{};
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
    uint4* gaps = nullptr;       // cell-start long-gap queue
    uint32_t gaps_cap = 0;
    void* staging = nullptr;
    size_t staging_bytes = 0;
    bool keys_valid = false;
    int32_t keys_active = -1;
    // incremental re-sort (resort.hip): sorted keys of the current slot order, and scratch
    uint32_t *sk_cur = nullptr, *sk_next = nullptr;
    uint32_t *mv_mi = nullptr, *mv_mk = nullptr, *mv_mo = nullptr, *mv_rank = nullptr, *mv_mx = nullptr, *mv_mos = nullptr;
    uint64_t* mv_ms = nullptr;
    uint32_t* mv_count = nullptr;   // [2] mover counters, ping-pong by step
    int mv_par = 0;                 // counter the next force pass appends into
    bool sk_valid = false;       // sk_cur matches the slot order and cs (set by a Model S sort)
    // env SPH_RESORT: 0 full radix sort every step, 1 (default) incremental re-sort unless the last
    // seen mover count exceeds resort_limit(n), 2 incremental whenever possible (tests)
    int resort_mode = 1;
    int ct_team = 0;                // env SPH_CT_TEAM: Model R lanes per target (0 = by size; tests)
    uint32_t* mv_host = nullptr;    // pinned: the mover count of the latest step copied back
    int64_t steps = 0;
    double sim_time = 0.0;
    sph_drag_input drag{-1, {0.f, 0.f, 0.f}, 0.f};
    std::string err;
    bool profiling = false;
    std::vector<KStat> kstats;
    std::vector<Pending> pending;
    std::vector<hipEvent_t> ev_pool;
    int64_t device_bytes = 0;
    int nb_variant = 1;          // neighbour passes: 0 direct (L1/L2 gathers), 1 LDS-tiled
    // slab decomposition (SPEC_SPH.md §3)
    bool slab = false;
    sph_slab sl{};
    bool has_left = false, has_right = false;
    GridDesc gglobal{};
    int32_t o0 = 0, o1 = 0;      // owned sorted slots
    int32_t rng[10] = {0};
    int32_t send_counts[2] = {0, 0};
    uint32_t* sblk = nullptr;    // compaction block counts [2][nblk]
    uint32_t* sdev = nullptr;    // small device scratch (totals, picks; [8], [9]: cell-start gap counters)
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
};

namespace {

int fail(sph_ctx* c, int code, const char* fmt, ...) {
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

void free_all(sph_ctx* c) {
    dfree(c->pos); dfree(c->vel); dfree(c->pos2); dfree(c->vel2);
    dfree(c->omg); dfree(c->rot); dfree(c->aux); dfree(c->omg2); dfree(c->rot2); dfree(c->aux2);
    dfree(c->id); dfree(c->id2); dfree(c->mode); dfree(c->mode2);
    dfree(c->rp); dfree(c->torque); dfree(c->slot_of);
    dfree(c->keys); dfree(c->keys2); dfree(c->vals); dfree(c->vals2); dfree(c->hist); dfree(c->bin_total);
    dfree(c->cs); dfree(c->gaps);
    c->gaps_cap = 0;
    dfree(c->sblk); dfree(c->sdev);
    dfree(c->sk_cur); dfree(c->sk_next);
    dfree(c->mv_mi); dfree(c->mv_mk); dfree(c->mv_mo); dfree(c->mv_rank); dfree(c->mv_mx); dfree(c->mv_mos);
    dfree(c->mv_ms); dfree(c->mv_count);
    c->sk_valid = false;
    if (c->staging) (void)hipFree(c->staging);
    c->staging = nullptr;
    c->staging_bytes = 0;
    c->cs_cap = 0;
    c->device_bytes = 0;
}

int bit_width(uint32_t v) {
    int b = 0;
    while (v) { ++b; v >>= 1; }
    return b < 1 ? 1 : b;
}

bool is_contact(const sph_ctx* c) { return c->cfg.model == SPH_MODEL_CONTACT; }

int alloc_particles(sph_ctx* ctx, int32_t cap) {
    const size_t n = (size_t)std::max(cap, 1);
    int r;
#define AL(p, cnt) if ((r = dalloc(ctx, &ctx->p, cnt)) != SPH_OK) return r
    AL(pos, n); AL(vel, n); AL(pos2, n); AL(vel2, n);
    AL(id, n); AL(id2, n);
    AL(keys, n); AL(keys2, n); AL(vals, n); AL(vals2, n);
    AL(hist, radix_hist_elems((int32_t)n)); AL(bin_total, 256);
    AL(sblk, 2 * (size_t)slab_compact_blocks(0, (int32_t)n) + 2); AL(sdev, 16);
    HIPCHK(hipMemset(ctx->sdev, 0, 16 * sizeof(uint32_t)));
    ctx->gap_par = 0;
    if (is_contact(ctx)) {
        AL(omg, n); AL(rot, n); AL(aux, n); AL(omg2, n); AL(rot2, n); AL(aux2, n);
        AL(mode, n); AL(mode2, n); AL(torque, 3 * n); AL(slot_of, n);
    } else {
        AL(rp, n);
    }
    // incremental re-sort (both models)
    AL(sk_cur, n); AL(sk_next, n);
    AL(mv_mi, n); AL(mv_mk, n); AL(mv_mo, n); AL(mv_rank, 3 * n); AL(mv_mx, n); AL(mv_mos, n); AL(mv_ms, n);
    AL(mv_count, 2);
    HIPCHK(hipMemset(ctx->mv_count, 0, 2 * sizeof(uint32_t)));
#undef AL
    ctx->staging_bytes = n * 84;
    HIPCHK(hipMalloc(&ctx->staging, ctx->staging_bytes));
    ctx->device_bytes += (int64_t)ctx->staging_bytes;
    return SPH_OK;
}

int ensure_cells(sph_ctx* ctx) {
    const uint32_t need = ctx->grid.ncells + 2;   // + the slab re-sort's cs_old[ncells + 1]
    if (need > ctx->cs_cap) {
        int r = dalloc(ctx, &ctx->cs, need);
        if (r != SPH_OK) return r;
        ctx->cs_cap = need;
    }
    // queued chunks: one per long gap (> 32 cells, so at most (ncells+1)/33) plus one per
    // 8192 cells of gap length
    const uint32_t g = (ctx->grid.ncells + 1) / 33 + (ctx->grid.ncells + 1) / 8192 + 4;
    if (g > ctx->gaps_cap) {
        int r = dalloc(ctx, &ctx->gaps, g);
        if (r != SPH_OK) return r;
        ctx->gaps_cap = g;
    }
    return SPH_OK;
}

// Grid + constants from params (SPEC_SPH.md §0/§2; same float arithmetic as the oracle).
int derive(sph_ctx* ctx) {
    const sph_params& p = ctx->prm;
    GridDesc g{};
    if (is_contact(ctx)) {
        // SimulateParticles.compute:16-18,102-105: 32^3 cells of 4.0 anchored at -spawnRadius
        g.ox = g.oy = g.oz = -p.spawn_radius;
        g.inv_cell = 0.25f;
        g.inv_cz = 0.25f;
        g.gx = g.gy = g.gz = 32;
        g.zsub = 1;
        g.zwin = 1;
    } else {
        if (!(p.h > 0.f) || !(p.dx > 0.f) || !(p.rho0 > 0.f))
            return fail(ctx, SPH_ERR_INVALID, "Model S needs dx, h, rho0 > 0");
        const float cell = 2.0f * p.h;
        const int32_t zsub = ctx->cfg.dim == 3 ? SPH_ZSUB : 1;
        const float cz = cell / (float)zsub;
        g.ox = g.oy = g.oz = 0.f;
        g.inv_cell = 1.0f / cell;
        g.inv_cz = 1.0f / cz;
        g.zsub = zsub;
        g.zwin = zsub + 1;
        int32_t G[3];
        for (int a = 0; a < 3; ++a) {
            G[a] = (int32_t)floorf(p.box[a] / (a == 2 ? cz : cell)) + 1;
            if (G[a] < 1) G[a] = 1;
        }
        if (ctx->cfg.dim == 2) G[2] = 1;
        g.gx = G[0]; g.gy = G[1]; g.gz = G[2];
        const double nc = (double)G[0] * G[1] * G[2];
        if (nc > 2.0e9) return fail(ctx, SPH_ERR_INVALID, "grid too large (%g cells)", nc);
        const float PI = 3.14159265358979f, d = p.dx, h = p.h;
        SphConst& s = ctx->sc;
        s.mass = p.rho0 * d * d * (ctx->cfg.dim == 3 ? d : 1.0f);
        s.B = p.c0 * p.c0 * p.rho0 / 7.0f;
        s.sigma = ctx->cfg.dim == 3 ? 1.0f / (PI * h * h * h) : 10.0f / (7.0f * PI * h * h);
        s.inv_h = 1.0f / h;
        s.four_h2 = 4.0f * h * h;
        s.sigma_h = s.sigma * s.inv_h;
        s.sigma_h2 = s.sigma * s.inv_h * s.inv_h;
        s.inv_rho0 = 1.0f / p.rho0;
        s.h = h;
        s.eta2 = 0.01f * h * h;
        s.ac0 = p.alpha * p.c0;
        s.eps = p.xsph_eps;
        s.gx = p.gravity[0]; s.gy = p.gravity[1]; s.gz = p.gravity[2];
        s.Lx = p.box[0]; s.Ly = p.box[1]; s.Lz = ctx->cfg.dim == 3 ? p.box[2] : 0.f;
        s.wall_e = p.wall_restitution;
    }
    g.cx0 = 0;
    g.gx_all = g.gx;
    g.ncells = (uint32_t)g.gx * (uint32_t)g.gy * (uint32_t)g.gz;
    ctx->grid = g;
    ctx->key_bits = bit_width(g.ncells);   // the sentinel key == ncells must sort last
    ctx->keys_valid = false;
    ctx->sk_valid = false;
    return ensure_cells(ctx);
}

// ---------------------------------------------------------------- profiling
int kstat_index(sph_ctx* c, const char* name) {
    for (size_t i = 0; i < c->kstats.size(); ++i)
        if (c->kstats[i].name == name) return (int)i;
    KStat k;
    k.name = name;
    c->kstats.push_back(k);
    return (int)c->kstats.size() - 1;
}

hipEvent_t take_event(sph_ctx* c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

void resolve_pending(sph_ctx* c) {
    for (auto& p : c->pending) {
        (void)hipEventSynchronize(p.b);
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) c->kstats[p.k].total_ms += ms;
        c->ev_pool.push_back(p.a);
        c->ev_pool.push_back(p.b);
    }
    c->pending.clear();
}

struct KTimer {
    sph_ctx* c;
    int k;
    hipEvent_t a = nullptr;
    KTimer(sph_ctx* ctx, const char* name, double bytes) : c(ctx), k(kstat_index(ctx, name)) {
        c->kstats[k].launches++;
        c->kstats[k].bytes = bytes;
        if (c->profiling) {
            a = take_event(c);
            (void)hipEventRecord(a, c->stream);
        }
    }
    ~KTimer() {
        if (c->profiling) {
            hipEvent_t b = take_event(c);
            (void)hipEventRecord(b, c->stream);
            c->pending.push_back({k, a, b});
            if (c->pending.size() > 8192) resolve_pending(c);
        }
    }
};

// ---------------------------------------------------------------- steps
void swap_sv(sph_ctx* c) {
    std::swap(c->pos, c->pos2);
    std::swap(c->vel, c->vel2);
}

int sort_and_reorder(sph_ctx* ctx, int32_t n_active_id, const uint32_t** sorted_keys = nullptr) {
    const int32_t n = ctx->n;
    if (!ctx->keys_valid || ctx->keys_active != n_active_id) {
        KTimer t(ctx, "keys", 20.0 * n);
        launch_keys(ctx->pos, n, is_contact(ctx) ? ctx->id : nullptr, n_active_id, ctx->grid, ctx->keys,
                    ctx->stream);
    }
    int side;
    {
        const int passes = (ctx->key_bits + 7) / 8;
        KTimer t(ctx, "radix_sort", (double)n * (20.0 * passes));
        side = radix_sort(ctx->keys, ctx->vals, ctx->keys2, ctx->vals2, n, ctx->key_bits, true, ctx->hist,
                          ctx->bin_total, ctx->stream);
    }
    const uint32_t* sk = side ? ctx->keys2 : ctx->keys;
    const uint32_t* perm = side ? ctx->vals2 : ctx->vals;
    if (is_contact(ctx)) {
        KTimer t(ctx, "reorder", (double)n * (4 + 2 * (5 * 16 + 8)));
        const GatherR gr{{ctx->pos, ctx->vel, ctx->omg, ctx->rot, ctx->aux},
                         {ctx->pos2, ctx->vel2, ctx->omg2, ctx->rot2, ctx->aux2},
                         {ctx->id, ctx->mode},
                         {ctx->id2, ctx->mode2}};
        launch_gather_r(perm, gr, n, ctx->stream);
        swap_sv(ctx);
        std::swap(ctx->omg, ctx->omg2);
        std::swap(ctx->rot, ctx->rot2);
        std::swap(ctx->aux, ctx->aux2);
        std::swap(ctx->id, ctx->id2);
        std::swap(ctx->mode, ctx->mode2);
    } else {
        KTimer t(ctx, "reorder", (double)n * (4 + 2 * 36));
        launch_gather_s(perm, ctx->pos, ctx->vel, ctx->id, ctx->pos2, ctx->vel2, ctx->id2, n, ctx->stream);
        swap_sv(ctx);
        std::swap(ctx->id, ctx->id2);
    }
    {
        KTimer t(ctx, "cell_start", 4.0 * (ctx->grid.ncells + 1));
        launch_cell_start(sk, n, ctx->cs, ctx->grid.ncells, ctx->gaps, ctx->sdev + 8, &ctx->gap_par, ctx->stream);
    }
    if (sorted_keys) *sorted_keys = sk;
    return SPH_OK;
}

void density_range(sph_ctx* ctx, int32_t b, int32_t e) {
    if (ctx->nb_variant == 0)
        launch_density(ctx->pos, ctx->cs, b, e, ctx->grid, ctx->sc, ctx->rp, ctx->stream);
    else
        launch_density_tiled(ctx->pos, ctx->cs, b, e, ctx->grid, ctx->sc, ctx->rp, ctx->stream);
}

void force_range(sph_ctx* ctx, int32_t b, int32_t e, float dt, float fext, MoverSink mv = MoverSink{}) {
    if (ctx->nb_variant == 0)
        launch_force_integrate(ctx->pos, ctx->vel, ctx->rp, ctx->cs, b, e, ctx->grid, ctx->sc, dt, fext, ctx->pos2,
                               ctx->vel2, ctx->keys, mv, ctx->stream);
    else
        launch_force_tiled(ctx->pos, ctx->vel, ctx->rp, ctx->cs, b, e, ctx->grid, ctx->sc, dt, fext, ctx->pos2,
                           ctx->vel2, ctx->keys, mv, ctx->stream);
}

ResortScratch resort_scratch(sph_ctx* ctx) {
    return ResortScratch{ctx->mv_mi, ctx->mv_mk, ctx->mv_mo, ctx->mv_rank, ctx->mv_ms, ctx->mv_mx, ctx->mv_mos,
                         (uint32_t)std::max(ctx->capacity, 1), 0};
}

// The force pass appends movers for the next step's incremental re-sort.
MoverSink mover_sink(sph_ctx* ctx) {
    if (ctx->resort_mode == 0 || !ctx->sk_valid) return MoverSink{};
    return MoverSink{ctx->sk_cur, ctx->mv_count + ctx->mv_par, ctx->mv_mi, ctx->mv_mk, ctx->mv_mo, ctx->mv_rank,
                     (uint32_t)std::max(ctx->capacity, 1)};
}

// Bring the slots into stable (key, index) order: the incremental re-sort when the previous
// step's sorted keys and cell starts describe the current slot order, else the full radix sort.
// Movers above which the full radix sort is cheaper than the incremental re-sort: k_mv_rank's
// all-pairs counts grow as m², the full sort as n (C3: ~12k movers, where the two cross).
uint32_t resort_limit(int32_t n) {
    return std::max<uint32_t>(4096u, (uint32_t)(12.0 * std::sqrt((double)std::max(n, 0))));
}

int sort_wcsph(sph_ctx* ctx) {
    const int32_t n = ctx->n;
    // adaptive mode: the latest mover count the host has seen (a step or more behind the device;
    // both paths give the same permutation, so the choice only affects time)
    const bool many = ctx->resort_mode == 1 && *(volatile uint32_t*)ctx->mv_host > resort_limit(n);
    if (ctx->resort_mode != 0 && !many && ctx->keys_valid && ctx->keys_active == 0 && ctx->sk_valid) {
        {
            KTimer t(ctx, "resort", (double)n * (2 * 4 + 2 * 36));
            const int used = ctx->mv_par;
            launch_resort(asm_plain(ctx->pos, ctx->vel, ctx->id, ctx->sk_cur, ctx->keys, n), ctx->cs,
                          ctx->grid.ncells, n, ctx->mv_count + used, ctx->mv_count + (1 - used), resort_scratch(ctx),
                          ctx->pos2, ctx->vel2, ctx->id2, ctx->sk_next, ctx->stream);
            ctx->mv_par = 1 - used;
        }
        swap_sv(ctx);
        std::swap(ctx->id, ctx->id2);
        std::swap(ctx->sk_cur, ctx->sk_next);
        return SPH_OK;
    }
    const uint32_t* sk = nullptr;
    int r = sort_and_reorder(ctx, 0, &sk);
    if (r != SPH_OK) return r;
    if (n > 0) HIPCHK(hipMemcpyAsync(ctx->sk_cur, sk, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->mv_count, 0, 2 * sizeof(uint32_t), ctx->stream));
    ctx->sk_valid = true;
    return SPH_OK;
}

int step_wcsph(sph_ctx* ctx, float dt) {
    const int32_t n = ctx->n;
    int r = sort_wcsph(ctx);
    if (r != SPH_OK) return r;
    {
        KTimer t(ctx, "density", 24.0 * n);
        density_range(ctx, 0, n);
    }
    const sph_params& p = ctx->prm;
    const float tt = (float)ctx->sim_time;
    const float fext = p.forcing_amp != 0.0f ? p.forcing_amp * sinf(6.28318530718f * p.forcing_freq * tt) : 0.0f;
    const MoverSink mv = mover_sink(ctx);
    {
        KTimer t(ctx, "force_integrate", 76.0 * n);
        force_range(ctx, 0, n, dt, fext, mv);
    }
    // this step's mover count, for the next steps' sort choice (no host wait); every 8th step, as the
    // copy is a ~4 us blit and the count drifts slowly
    if (mv.sk && (ctx->steps & 7) == 0)
        HIPCHK(hipMemcpyAsync(ctx->mv_host, mv.count, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    swap_sv(ctx);
    ctx->keys_valid = true;
    ctx->keys_active = 0;
    return SPH_OK;
}

// ---------------------------------------------------------------- adhesion bonds (§8f-1)
void free_bonds(sph_ctx* c) {
    dfree(c->b_ends); dfree(c->b_spring); dfree(c->b_relq); dfree(c->b_anc_a); dfree(c->b_anc_b);
    dfree(c->b_terms); dfree(c->b_off); dfree(c->b_ent);
    c->bond_cap = 0;
    c->b_off_cap = 0;
    c->b_index_n = -1;
}

BondSet bond_set(const sph_ctx* c) {
    return BondSet{c->b_ends, c->b_spring, c->b_relq, c->b_anc_a, c->b_anc_b, c->nbonds};
}

// The per-particle incidence lists (CSR by particle index) of the current bonds, rebuilt on the
// host when the bonds or the particle count changed. Bonds naming an index outside [0, n) are
// skipped by the reference (compute:432), so they have no entries (their terms stay zero).
int bond_index(sph_ctx* ctx) {
    const int32_t n = ctx->n;
    if (ctx->b_index_n == n) return SPH_OK;
    HIPCHK(hipStreamSynchronize(ctx->stream));   // the previous lists may still be in flight
    std::vector<uint32_t>& off = ctx->b_off_host;
    std::vector<uint32_t>& ent = ctx->b_ent_host;
    off.assign((size_t)n + 1, 0u);
    for (const int2& e : ctx->bonds_host)
        if (e.x >= 0 && e.y >= 0 && e.x < n && e.y < n) { off[(size_t)e.x + 1]++; off[(size_t)e.y + 1]++; }
    for (int32_t i = 0; i < n; ++i) off[(size_t)i + 1] += off[(size_t)i];
    ent.assign(off[(size_t)n] > 0 ? off[(size_t)n] : 1u, 0u);
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    for (int32_t b = 0; b < ctx->nbonds; ++b) {
        const int2 e = ctx->bonds_host[(size_t)b];
        if (!(e.x >= 0 && e.y >= 0 && e.x < n && e.y < n)) continue;
        ent[fill[(size_t)e.x]++] = (uint32_t)b << 1;
        ent[fill[(size_t)e.y]++] = ((uint32_t)b << 1) | 1u;
    }
    int r;
    if ((int64_t)n + 1 > ctx->b_off_cap) {
        if ((r = dalloc(ctx, &ctx->b_off, (size_t)n + 1)) != SPH_OK) return r;
        ctx->b_off_cap = n + 1;
    }
    if ((r = dalloc(ctx, &ctx->b_ent, ent.size())) != SPH_OK) return r;
    HIPCHK(hipMemcpyAsync(ctx->b_off, off.data(), off.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->b_ent, ent.data(), ent.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    ctx->b_index_n = n;
    return SPH_OK;
}

int32_t contact_active(const sph_ctx* c) {
    int32_t a = c->prm.active_particle_count;
    if (a <= 0 || a > c->n) a = c->n;
    return a;
}

// Model R's sort: the incremental re-sort (movers appended by the previous contact pass) while the
// previous step's sorted keys describe the slot order, else the full sort. Both give the same
// permutation (tests/test_gpu_resort.py), so results never depend on the choice.
int sort_contact(sph_ctx* ctx, int32_t act) {
    const int32_t n = ctx->n;
    const bool many = ctx->resort_mode == 1 && *(volatile uint32_t*)ctx->mv_host > resort_limit(n);
    if (ctx->resort_mode != 0 && !many && ctx->keys_valid && ctx->keys_active == act && ctx->sk_valid && n > 0) {
        KTimer t(ctx, "resort", (double)n * (2 * 4 + 2 * 88));
        const int used = ctx->mv_par;
        const ResortExtra ex{ctx->omg, ctx->rot, ctx->aux, ctx->mode, ctx->omg2, ctx->rot2, ctx->aux2, ctx->mode2};
        launch_resort(asm_plain(ctx->pos, ctx->vel, ctx->id, ctx->sk_cur, ctx->keys, n), ctx->cs, ctx->grid.ncells, n,
                      ctx->mv_count + used, ctx->mv_count + (1 - used), resort_scratch(ctx), ctx->pos2, ctx->vel2,
                      ctx->id2, ctx->sk_next, ctx->stream, CsPick{{0}, 0, nullptr, nullptr}, ex);
        ctx->mv_par = 1 - used;
        swap_sv(ctx);
        std::swap(ctx->id, ctx->id2);
        std::swap(ctx->omg, ctx->omg2);
        std::swap(ctx->rot, ctx->rot2);
        std::swap(ctx->aux, ctx->aux2);
        std::swap(ctx->mode, ctx->mode2);
        std::swap(ctx->sk_cur, ctx->sk_next);
        return SPH_OK;
    }
    const uint32_t* sk = nullptr;
    int r = sort_and_reorder(ctx, act, &sk);
    if (r != SPH_OK) return r;
    if (ctx->resort_mode != 0 && n > 0) {
        HIPCHK(hipMemcpyAsync(ctx->sk_cur, sk, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream));
        HIPCHK(hipMemsetAsync(ctx->mv_count, 0, 2 * sizeof(uint32_t), ctx->stream));
    }
    ctx->sk_valid = ctx->resort_mode != 0;
    return SPH_OK;
}

int step_contact(sph_ctx* ctx, float dt) {
    const int32_t n = ctx->n;
    const int32_t act = contact_active(ctx);
    int r = sort_contact(ctx, act);
    if (r != SPH_OK) return r;
    const MoverSink mv = mover_sink(ctx);
    const sph_params& p = ctx->prm;
    ContactConst c{};
    c.dt = dt;
    c.spawn_radius = p.spawn_radius;
    c.global_drag = p.global_drag_multiplier;
    c.torque_factor = p.torque_factor;
    c.torque_damping = p.torque_damping;
    c.boundary_friction = p.boundary_friction;
    c.roll_mult = p.rolling_contact_radius_multiplier;
    c.repulsion_strength = p.repulsion_strength;
    c.drag_id = ctx->drag.selected_id;
    c.drag_tx = ctx->drag.target[0];
    c.drag_ty = ctx->drag.target[1];
    c.drag_tz = ctx->drag.target[2];
    c.drag_strength = ctx->drag.strength;
    if (ctx->nbonds == 0) {
        KTimer t(ctx, "contact_step", (double)n * (2 * 64 + 4 + 12 + 4));
        launch_contact_step(ctx->pos, ctx->vel, ctx->omg, ctx->rot, ctx->aux, ctx->id, ctx->cs, act, n, ctx->grid,
                            c, ctx->pos2, ctx->vel2, ctx->omg2, ctx->rot2, ctx->torque, ctx->keys, ctx->ct_team, mv,
                            ctx->stream);
    } else {
        // adhesion (controller:284-310): forces, bond terms, then deltas + drag + motion + rotation
        r = bond_index(ctx);
        if (r != SPH_OK) return r;
        {
            KTimer t(ctx, "contact_forces", (double)n * (3 * 16 + 4 + 2 * 16 + 12 + 4));
            launch_contact_forces(ctx->pos, ctx->vel, ctx->omg, ctx->id, ctx->cs, act, n, ctx->grid, c, ctx->vel2,
                                  ctx->omg2, ctx->torque, ctx->slot_of, ctx->ct_team, ctx->stream);
        }
        {
            KTimer t(ctx, "bond_terms", (double)ctx->nbonds * (8 + 4 * 16 + 2 * (4 + 3 * 16) + 64));
            launch_bond_terms(bond_set(ctx), ctx->slot_of, n, ctx->pos, ctx->vel2, ctx->rot, dt, ctx->b_terms,
                              ctx->stream);
        }
        {
            KTimer t(ctx, "contact_finish", (double)n * (5 * 16 + 4 + 12 + 8 + 4 * 16 + 4) + 4.0 * ctx->nbonds * 36);
            BondView bv{ctx->nbonds, ctx->b_index_n, ctx->b_off, ctx->b_ent, ctx->b_terms};
            launch_contact_finish(ctx->pos, ctx->rot, ctx->aux, ctx->id, ctx->torque, act, n, ctx->grid, c, bv,
                                  ctx->vel2, ctx->omg2, ctx->pos2, ctx->rot2, ctx->keys, mv, ctx->stream);
        }
    }
    if (mv.sk && (ctx->steps & 7) == 0)   // the mover count for the next steps' sort choice (no wait)
        HIPCHK(hipMemcpyAsync(ctx->mv_host, mv.count, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    swap_sv(ctx);
    std::swap(ctx->omg, ctx->omg2);
    std::swap(ctx->rot, ctx->rot2);
    ctx->keys_valid = true;
    ctx->keys_active = act;
    return SPH_OK;
}

}  // namespace

static int slab_local_grid(sph_ctx* ctx);

// ====================================================================== ABI
extern "C" {

int32_t sph_abi_version(void) { return SPH_ABI_VERSION; }

const char* sph_last_error(const sph_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int sph_create(const sph_config* cfg, int32_t device, sph_ctx** out) {
    if (!cfg || !out) return SPH_ERR_INVALID;
    *out = nullptr;
    if (cfg->model != SPH_MODEL_CONTACT && cfg->model != SPH_MODEL_WCSPH) return SPH_ERR_INVALID;
    if (cfg->dim != 2 && cfg->dim != 3) return SPH_ERR_INVALID;
    if (cfg->model == SPH_MODEL_CONTACT && cfg->dim != 3) return SPH_ERR_INVALID;
    if (cfg->capacity < 0) return SPH_ERR_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SPH_ERR_HIP;
    if (device < 0 || device >= ndev) return SPH_ERR_INVALID;
    sph_ctx* ctx = new sph_ctx();
    ctx->cfg = *cfg;
    ctx->device = device;
    ctx->profiling = (cfg->flags & SPH_FLAG_PROFILE) != 0;
    if (const char* v = std::getenv("SPH_NB_VARIANT")) ctx->nb_variant = std::atoi(v);
    if (const char* v = std::getenv("SPH_RESORT")) ctx->resort_mode = std::atoi(v);
    if (const char* v = std::getenv("SPH_CT_TEAM")) ctx->ct_team = std::atoi(v);
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&ctx->mv_host, sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
        delete ctx;
        return SPH_ERR_HIP;
    }
    *ctx->mv_host = 0u;
    ctx->own_stream = true;
    ctx->capacity = cfg->capacity;
    int r = alloc_particles(ctx, cfg->capacity);
    if (r != SPH_OK) {
        free_all(ctx);
        (void)hipStreamDestroy(ctx->stream);
        delete ctx;
        return r;
    }
    // reference defaults (ParticleSystemController.cs:12-24)
    sph_params& p = ctx->prm;
    p.spawn_radius = 15.f; p.min_radius = 1.5f; p.max_radius = 2.0f; p.global_drag_multiplier = 1.f;
    p.torque_factor = 1.f; p.torque_damping = 0.5f; p.boundary_friction = 0.8f;
    p.rolling_contact_radius_multiplier = 5.f; p.density = 0.1f; p.repulsion_strength = 200.f;
    p.active_particle_count = 0;
    if (is_contact(ctx)) {
        r = derive(ctx);
        if (r != SPH_OK) { sph_destroy(ctx); return r; }
        ctx->params_set = true;
    }
    *out = ctx;
    return SPH_OK;
}

void sph_destroy(sph_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    resolve_pending(ctx);
    for (auto e : ctx->ev_pool) (void)hipEventDestroy(e);
    if (ctx->rng_ev) (void)hipEventDestroy(ctx->rng_ev);
    if (ctx->rng_host) (void)hipHostFree(ctx->rng_host);
    free_all(ctx);
    free_bonds(ctx);
    for (int f = 0; f < 3; ++f) {
        if (ctx->rb_dev[f]) (void)hipFree(ctx->rb_dev[f]);
        if (ctx->rb_host[f]) (void)hipHostFree(ctx->rb_host[f]);
    }
    if (ctx->rb_src) (void)hipEventDestroy(ctx->rb_src);
    if (ctx->rb_ready) (void)hipEventDestroy(ctx->rb_ready);
    if (ctx->rb_stream) (void)hipStreamDestroy(ctx->rb_stream);
    if (ctx->mv_host) (void)hipHostFree(ctx->mv_host);
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int sph_set_stream(sph_ctx* ctx, void* s) {
    if (!ctx) return SPH_ERR_INVALID;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (s == nullptr) {
        if (!ctx->own_stream) {
            HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
            ctx->own_stream = true;
        }
        return SPH_OK;
    }
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
    ctx->stream = (hipStream_t)s;
    ctx->own_stream = false;
    return SPH_OK;
}

int sph_get_stream(sph_ctx* ctx, void** s) {
    if (!ctx || !s) return SPH_ERR_INVALID;
    *s = (void*)ctx->stream;
    return SPH_OK;
}

int sph_set_params(sph_ctx* ctx, const sph_params* params) {
    if (!ctx || !params) return SPH_ERR_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    const sph_params old = ctx->prm;
    ctx->prm = *params;
    int r = derive(ctx);
    if (r != SPH_OK) { ctx->prm = old; return r; }
    ctx->params_set = true;
    if (ctx->slab) {                 // keep the slab's window of the (new) global grid
        ctx->gglobal = ctx->grid;
        return slab_local_grid(ctx);
    }
    return SPH_OK;
}

int sph_get_params(const sph_ctx* ctx, sph_params* params) {
    if (!ctx || !params) return SPH_ERR_INVALID;
    *params = ctx->prm;
    return SPH_OK;
}

int sph_scenario_params(const sph_scenario* sc, sph_params* out, float* dt_out) {
    if (!sc || !out) return SPH_ERR_INVALID;
    if (sc->dim != 2 && sc->dim != 3) return SPH_ERR_INVALID;
    if (!(sc->dx > 0.f) || sc->nx <= 0 || sc->ny <= 0 || (sc->dim == 3 && sc->nz <= 0)) return SPH_ERR_INVALID;
    std::memset(out, 0, sizeof *out);
    const double dx = sc->dx, g = 9.81;
    const double H = sc->ny * dx;               // initial fluid height (y up)
    const double c0 = 10.0 * std::sqrt(2.0 * g * H);
    out->dx = (float)dx;
    out->h = (float)(1.2 * dx);
    out->rho0 = 1000.f;
    out->c0 = (float)c0;
    out->alpha = 0.02f;
    out->xsph_eps = 0.5f;
    out->gravity[0] = 0.f; out->gravity[1] = (float)-g; out->gravity[2] = 0.f;
    out->box[0] = (float)(sc->tx * dx);
    out->box[1] = (float)(sc->ty * dx);
    out->box[2] = sc->dim == 3 ? (float)(sc->tz * dx) : 0.f;
    out->wall_restitution = 0.5f;
    if (sc->kind == SPH_SCENARIO_SLOSHING) {
        const double L = sc->tx * dx, PI = 3.14159265358979323846;
        out->forcing_amp = (float)(0.1 * g);
        out->forcing_freq = (float)(std::sqrt(g * PI / L * std::tanh(PI * H / L)) / (2.0 * PI));
    }
    // reference uniforms keep their defaults (ParticleSystemController.cs:12-24)
    out->spawn_radius = 15.f; out->min_radius = 1.5f; out->max_radius = 2.0f;
    out->global_drag_multiplier = 1.f; out->torque_factor = 1.f; out->torque_damping = 0.5f;
    out->boundary_friction = 0.8f; out->rolling_contact_radius_multiplier = 5.f;
    out->density = 0.1f; out->repulsion_strength = 200.f;
    if (dt_out) *dt_out = (float)(0.25 * (1.2 * dx) / c0);
    return SPH_OK;
}

int sph_upload_particles_aos84(sph_ctx* ctx, const void* src, int32_t count) {
    if (!ctx || (!src && count > 0) || count < 0) return SPH_ERR_INVALID;
    if (count > ctx->capacity) return fail(ctx, SPH_ERR_CAPACITY, "count %d > capacity %d", count, ctx->capacity);
    HIPCHK(hipSetDevice(ctx->device));
    if (count > 0) {
        HIPCHK(hipMemcpyAsync(ctx->staging, src, (size_t)count * 84, hipMemcpyHostToDevice, ctx->stream));
        launch_aos84_to_soa(ctx->staging, count, ctx->pos, ctx->vel, ctx->omg, ctx->rot, ctx->aux, ctx->mode,
                            ctx->id, ctx->stream);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->n = count;
    ctx->keys_valid = false;
    ctx->sk_valid = false;
    ctx->steps = 0;
    ctx->sim_time = 0.0;
    return SPH_OK;
}

int sph_download_particles_aos84(sph_ctx* ctx, void* dst, int32_t count) {
    if (!ctx || (!dst && count > 0)) return SPH_ERR_INVALID;
    if (count < ctx->n) return fail(ctx, SPH_ERR_INVALID, "count %d < active particles %d", count, ctx->n);
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->n > 0) {
        launch_soa_to_aos84(ctx->pos, ctx->vel, ctx->omg, ctx->rot, ctx->aux, ctx->mode, ctx->id, ctx->n,
                            ctx->staging, ctx->stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(dst, ctx->staging, (size_t)ctx->n * 84, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

int sph_upload_state(sph_ctx* ctx, const float* pos3, const float* vel3, int32_t count) {
    if (!ctx || (!pos3 && count > 0) || count < 0) return SPH_ERR_INVALID;
    if (is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "sph_upload_state is Model S only; use aos84");
    if (count > ctx->capacity) return fail(ctx, SPH_ERR_CAPACITY, "count %d > capacity %d", count, ctx->capacity);
    HIPCHK(hipSetDevice(ctx->device));
    if (count > 0) {
        float* sp = (float*)ctx->staging;
        float* sv = vel3 ? sp + 3 * (size_t)count : nullptr;
        HIPCHK(hipMemcpyAsync(sp, pos3, (size_t)count * 12, hipMemcpyHostToDevice, ctx->stream));
        if (vel3) HIPCHK(hipMemcpyAsync(sv, vel3, (size_t)count * 12, hipMemcpyHostToDevice, ctx->stream));
        launch_pack_sv(sp, sv, count, ctx->pos, ctx->vel, ctx->id, ctx->stream);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->n = count;
    ctx->keys_valid = false;
    ctx->sk_valid = false;
    ctx->steps = 0;
    ctx->sim_time = 0.0;
    return SPH_OK;
}

int sph_init_scenario(sph_ctx* ctx, const sph_scenario* sc) {
    if (!ctx || !sc) return SPH_ERR_INVALID;
    if (is_contact(ctx)) {
        if (sc->kind != SPH_SCENARIO_SPHERE) return fail(ctx, SPH_ERR_INVALID, "Model R scenarios: SPH_SCENARIO_SPHERE");
        return sph_init_particles(ctx, sc->nx, sc->nx, 0, 0);
    }
    if (sc->dim != ctx->cfg.dim) return fail(ctx, SPH_ERR_INVALID, "scenario dim %d != context dim %d", sc->dim, ctx->cfg.dim);
    const int64_t n = (int64_t)sc->nx * sc->ny * (sc->dim == 3 ? sc->nz : 1);
    if (n <= 0) return fail(ctx, SPH_ERR_INVALID, "empty scenario");
    if (n > ctx->capacity) return fail(ctx, SPH_ERR_CAPACITY, "scenario needs %lld > capacity %d", (long long)n, ctx->capacity);
    HIPCHK(hipSetDevice(ctx->device));
    launch_lattice(sc->dim, sc->nx, sc->ny, sc->nz, sc->dx, 0.f, 0.f, 0.f, sc->seed, sc->jitter * sc->dx, ctx->pos,
                   ctx->vel, ctx->id, ctx->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->n = (int32_t)n;
    ctx->keys_valid = false;
    ctx->sk_valid = false;
    ctx->steps = 0;
    ctx->sim_time = 0.0;
    return SPH_OK;
}

static_assert(sizeof(sph_split) == 92 && sizeof(SplitRec) == sizeof(sph_split), "CellSplitData layout");

static int ensure_staging(sph_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->staging_bytes) return SPH_OK;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (ctx->staging) (void)hipFree(ctx->staging);
    ctx->staging = nullptr;
    ctx->staging_bytes = 0;
    HIPCHK(hipMalloc(&ctx->staging, bytes));
    ctx->staging_bytes = bytes;
    return SPH_OK;
}

int sph_init_particles(sph_ctx* ctx, int32_t count, int32_t active, int32_t genome_modes, int32_t default_mode) {
    if (!ctx || count < 0 || active < 0 || active > count || genome_modes < 0) return SPH_ERR_INVALID;
    if (!is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "sph_init_particles is Model R (InitParticles) only");
    if (count > ctx->capacity) return fail(ctx, SPH_ERR_CAPACITY, "count %d > capacity %d", count, ctx->capacity);
    HIPCHK(hipSetDevice(ctx->device));
    const sph_params& p = ctx->prm;
    InitConst c{p.spawn_radius, p.min_radius, p.max_radius, p.density, count, genome_modes, default_mode};
    launch_init_sphere(count, active, c, ctx->pos, ctx->vel, ctx->omg, ctx->rot, ctx->aux, ctx->mode, ctx->id,
                       ctx->torque, ctx->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->n = count;
    ctx->prm.active_particle_count = active;
    ctx->keys_valid = false;
    ctx->steps = 0;
    ctx->sim_time = 0.0;
    return SPH_OK;
}

// Grow the particle arrays to `capacity` on the device, keeping the current slots (D2D copies).
static int grow_d2d(sph_ctx* ctx, int32_t capacity) {
    const int32_t n = ctx->n;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    float4 *pos = ctx->pos, *vel = ctx->vel, *omg = ctx->omg, *rot = ctx->rot, *aux = ctx->aux;
    int32_t *id = ctx->id, *mode = ctx->mode;
    ctx->pos = ctx->vel = ctx->omg = ctx->rot = ctx->aux = nullptr;
    ctx->id = ctx->mode = nullptr;
    free_all(ctx);
    ctx->capacity = capacity;
    int r = alloc_particles(ctx, capacity);
    if (r == SPH_OK && ctx->params_set) r = derive(ctx);
    hipError_t e = hipSuccess;
    const size_t f4 = (size_t)n * sizeof(float4), i4 = (size_t)n * 4;
    if (r == SPH_OK && n > 0) {
        e = hipMemcpyAsync(ctx->pos, pos, f4, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(ctx->vel, vel, f4, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(ctx->id, id, i4, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess && omg) e = hipMemcpyAsync(ctx->omg, omg, f4, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess && rot) e = hipMemcpyAsync(ctx->rot, rot, f4, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess && aux) e = hipMemcpyAsync(ctx->aux, aux, f4, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess && mode) e = hipMemcpyAsync(ctx->mode, mode, i4, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    }
    dfree(pos); dfree(vel); dfree(omg); dfree(rot); dfree(aux); dfree(id); dfree(mode);
    if (r != SPH_OK) return r;
    if (e != hipSuccess) return fail(ctx, SPH_ERR_HIP, "resize copy: %s", hipGetErrorString(e));
    ctx->keys_valid = false;
    ctx->sk_valid = false;
    return SPH_OK;
}

int sph_split_particles(sph_ctx* ctx, const sph_split* splits, int32_t count, int32_t* active_out) {
    if (!ctx || count < 0 || (count > 0 && !splits)) return SPH_ERR_INVALID;
    if (!is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "cell division is Model R only");
    if (ctx->slab) return fail(ctx, SPH_ERR_STATE, "slab mode");
    HIPCHK(hipSetDevice(ctx->device));
    const int32_t active = contact_active(ctx);
    if (count == 0) {
        if (active_out) *active_out = active;
        return SPH_OK;
    }
    std::vector<unsigned char> seen((size_t)active, 0);
    for (int32_t k = 0; k < count; ++k) {
        const int32_t p = splits[k].parent_index;
        if (p < 0 || p >= active) return fail(ctx, SPH_ERR_INVALID, "split %d: parent %d not in [0, %d)", k, p, active);
        if (seen[(size_t)p]++) return fail(ctx, SPH_ERR_INVALID, "split %d: parent %d split twice", k, p);
    }
    const int64_t need = (int64_t)active + count;
    if (need > INT32_MAX) return fail(ctx, SPH_ERR_CAPACITY, "too many particles");
    if (need > ctx->capacity) {   // controller:788-792
        const int64_t cap = std::max<int64_t>(need, std::min<int64_t>(2 * (int64_t)ctx->capacity, INT32_MAX));
        int r = grow_d2d(ctx, (int32_t)cap);
        if (r != SPH_OK) return r;
    }
    int r = ensure_staging(ctx, (size_t)count * sizeof(sph_split));
    if (r != SPH_OK) return r;
    const int32_t n_old = ctx->n;
    HIPCHK(hipMemcpyAsync(ctx->staging, splits, (size_t)count * sizeof(sph_split), hipMemcpyHostToDevice, ctx->stream));
    launch_slot_map(ctx->id, n_old, ctx->slot_of, ctx->stream);
    launch_split((const SplitRec*)ctx->staging, count, active, n_old, ctx->slot_of, ctx->pos, ctx->vel, ctx->omg,
                 ctx->rot, ctx->aux, ctx->mode, ctx->id, ctx->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));   // the split records live in the caller's memory
    ctx->n = std::max<int32_t>(n_old, (int32_t)need);
    ctx->prm.active_particle_count = (int32_t)need;
    ctx->keys_valid = false;
    if (active_out) *active_out = (int32_t)need;
    return SPH_OK;
}

static int range_args(sph_ctx* ctx, int32_t first, int32_t count, const void* buf) {
    if (!ctx || first < 0 || count < 0 || (count > 0 && !buf)) return SPH_ERR_INVALID;
    if (!is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "84-byte particle ranges are Model R only");
    if ((int64_t)first + count > ctx->n)
        return fail(ctx, SPH_ERR_INVALID, "range [%d, %d) outside the %d particles", first, first + count, ctx->n);
    return SPH_OK;
}

int sph_get_particles_aos84(sph_ctx* ctx, int32_t first, int32_t count, void* dst) {
    int r = range_args(ctx, first, count, dst);
    if (r != SPH_OK || count == 0) return r;
    HIPCHK(hipSetDevice(ctx->device));
    launch_slot_map(ctx->id, ctx->n, ctx->slot_of, ctx->stream);
    launch_get_range(ctx->pos, ctx->vel, ctx->omg, ctx->rot, ctx->aux, ctx->mode, ctx->slot_of, first, count,
                     ctx->staging, ctx->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(dst, ctx->staging, (size_t)count * 84, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

int sph_set_particles_aos84(sph_ctx* ctx, int32_t first, int32_t count, const void* src) {
    int r = range_args(ctx, first, count, src);
    if (r != SPH_OK || count == 0) return r;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemcpyAsync(ctx->staging, src, (size_t)count * 84, hipMemcpyHostToDevice, ctx->stream));
    launch_slot_map(ctx->id, ctx->n, ctx->slot_of, ctx->stream);
    launch_set_range(ctx->staging, ctx->slot_of, first, count, ctx->pos, ctx->vel, ctx->omg, ctx->rot, ctx->aux,
                     ctx->mode, ctx->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->keys_valid = false;
    return SPH_OK;
}

int sph_step(sph_ctx* ctx, float dt, int32_t nsteps) {
    if (!ctx || nsteps < 0 || !(dt >= 0.f)) return SPH_ERR_INVALID;
    if (ctx->slab) return fail(ctx, SPH_ERR_STATE, "slab mode: the host drives sph_slab_* phases");
    if (!ctx->params_set) return fail(ctx, SPH_ERR_STATE, "sph_set_params first");
    HIPCHK(hipSetDevice(ctx->device));
    for (int32_t s = 0; s < nsteps; ++s) {
        if (ctx->n > 0) {
            int r = is_contact(ctx) ? step_contact(ctx, dt) : step_wcsph(ctx, dt);
            if (r != SPH_OK) return r;
        }
        ctx->steps++;
        ctx->sim_time += (double)dt;
    }
    HIPCHK(hipGetLastError());
    return SPH_OK;
}

int sph_set_drag(sph_ctx* ctx, const sph_drag_input* drag) {
    if (!ctx || !drag) return SPH_ERR_INVALID;
    ctx->drag = *drag;
    return SPH_OK;
}

int sph_set_adhesion(sph_ctx* ctx, const void* conn84, int32_t count) {
    if (!ctx || count < 0 || (count > 0 && !conn84)) return SPH_ERR_INVALID;
    if (!is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "adhesion bonds are Model R only");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipStreamSynchronize(ctx->stream));   // earlier steps may still read the old bonds
    if (count > ctx->bond_cap) {
        int r;
        const size_t cap = (size_t)count;
        if ((r = dalloc(ctx, &ctx->b_ends, cap)) != SPH_OK || (r = dalloc(ctx, &ctx->b_spring, cap)) != SPH_OK ||
            (r = dalloc(ctx, &ctx->b_relq, cap)) != SPH_OK || (r = dalloc(ctx, &ctx->b_anc_a, cap)) != SPH_OK ||
            (r = dalloc(ctx, &ctx->b_anc_b, cap)) != SPH_OK || (r = dalloc(ctx, &ctx->b_terms, 4 * cap)) != SPH_OK) {
            free_bonds(ctx);
            ctx->nbonds = 0;
            ctx->bonds_host.clear();
            return r;
        }
        ctx->bond_cap = count;
    }
    // AdhesionConnection (compute:43-55; CellAdhesionManager.cs:511-524), 84 bytes:
    //  0 particleA, 4 particleB, 8 restLength, 12 springStiffness, 16 springDamping,
    //  20 connectionColor[4], 36 initialRelOrientation[4], 52 anchorLocalPosA[3],
    //  64 anchorLocalPosB[3], 76 anchorConstraintStiffness, 80 enableAnchorConstraint
    const unsigned char* src = (const unsigned char*)conn84;
    std::vector<int2> ends((size_t)count);
    std::vector<float4> spring((size_t)count), relq((size_t)count), anc_a((size_t)count), anc_b((size_t)count);
    for (int32_t b = 0; b < count; ++b) {
        const unsigned char* r = src + (size_t)b * 84;
        int32_t i[2], en;
        float f[3], q[4], a[3], bb[3], ks;
        std::memcpy(i, r, 8);
        std::memcpy(f, r + 8, 12);
        std::memcpy(q, r + 36, 16);
        std::memcpy(a, r + 52, 12);
        std::memcpy(bb, r + 64, 12);
        std::memcpy(&ks, r + 76, 4);
        std::memcpy(&en, r + 80, 4);
        float enf;
        std::memcpy(&enf, &en, 4);
        ends[(size_t)b] = make_int2(i[0], i[1]);
        spring[(size_t)b] = make_float4(f[0], f[1], f[2], ks);
        relq[(size_t)b] = make_float4(q[0], q[1], q[2], q[3]);
        anc_a[(size_t)b] = make_float4(a[0], a[1], a[2], enf);
        anc_b[(size_t)b] = make_float4(bb[0], bb[1], bb[2], 0.f);
    }
    if (count > 0) {
        HIPCHK(hipMemcpy(ctx->b_ends, ends.data(), (size_t)count * sizeof(int2), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(ctx->b_spring, spring.data(), (size_t)count * sizeof(float4), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(ctx->b_relq, relq.data(), (size_t)count * sizeof(float4), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(ctx->b_anc_a, anc_a.data(), (size_t)count * sizeof(float4), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(ctx->b_anc_b, anc_b.data(), (size_t)count * sizeof(float4), hipMemcpyHostToDevice));
    }
    ctx->bonds_host.swap(ends);
    ctx->nbonds = count;
    ctx->b_index_n = -1;
    return SPH_OK;
}

int sph_read_adhesion_terms(sph_ctx* ctx, int32_t* terms16, int32_t count) {
    if (!ctx || count < 0 || (count > 0 && !terms16)) return SPH_ERR_INVALID;
    if (!is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "adhesion bonds are Model R only");
    if (count < ctx->nbonds) return fail(ctx, SPH_ERR_INVALID, "count %d < bonds %d", count, ctx->nbonds);
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->nbonds > 0)
        HIPCHK(hipMemcpyAsync(terms16, ctx->b_terms, (size_t)ctx->nbonds * 64, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

static int read_f4(sph_ctx* ctx, const float4* src, float* dst, int32_t count, int comps) {
    if (!ctx || (!dst && count > 0)) return SPH_ERR_INVALID;
    if (ctx->slab) return fail(ctx, SPH_ERR_STATE, "slab mode: use sph_slab_read_owned");
    if (count < ctx->n) return fail(ctx, SPH_ERR_INVALID, "count %d < active particles %d", count, ctx->n);
    if (!src) return fail(ctx, SPH_ERR_STATE, "field not held by this model");
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->n > 0) {
        launch_scatter_f4_by_id(src, ctx->id, ctx->n, (float*)ctx->staging, comps, ctx->stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(dst, ctx->staging, (size_t)ctx->n * comps * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

int sph_read_positions(sph_ctx* ctx, float* xyz, int32_t count) {
    return ctx ? read_f4(ctx, ctx->pos, xyz, count, 3) : SPH_ERR_INVALID;
}
int sph_read_velocities(sph_ctx* ctx, float* xyz, int32_t count) {
    return ctx ? read_f4(ctx, ctx->vel, xyz, count, 3) : SPH_ERR_INVALID;
}
int sph_read_rotations(sph_ctx* ctx, float* xyzw, int32_t count) {
    return ctx ? read_f4(ctx, ctx->rot, xyzw, count, 4) : SPH_ERR_INVALID;
}
int sph_read_angular_velocities(sph_ctx* ctx, float* xyz, int32_t count) {
    return ctx ? read_f4(ctx, ctx->omg, xyz, count, 3) : SPH_ERR_INVALID;
}

int sph_read_density(sph_ctx* ctx, float* rho, int32_t count) {
    if (!ctx || (!rho && count > 0)) return SPH_ERR_INVALID;
    if (is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "density is Model S only");
    if (ctx->slab) return fail(ctx, SPH_ERR_STATE, "slab mode: use sph_slab_read_owned");
    if (count < ctx->n) return fail(ctx, SPH_ERR_INVALID, "count %d < active particles %d", count, ctx->n);
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->n > 0) {
        // rp is in the slot order of the last step's density pass; id was reordered before it
        launch_scatter_f2x_by_id(ctx->rp, ctx->id, ctx->n, (float*)ctx->staging, ctx->stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(rho, ctx->staging, (size_t)ctx->n * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

int sph_read_torque_int(sph_ctx* ctx, int32_t* xyz, int32_t count) {
    if (!ctx || (!xyz && count > 0)) return SPH_ERR_INVALID;
    if (!is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "torque is Model R only");
    if (count < ctx->n) return fail(ctx, SPH_ERR_INVALID, "count %d < active particles %d", count, ctx->n);
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->n > 0) {
        launch_scatter_i3_by_id(ctx->torque, ctx->id, ctx->n, (int32_t*)ctx->staging, ctx->stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(xyz, ctx->staging, (size_t)ctx->n * 12, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

// ---------------------------------------------------------------- async readback / render interop
static const size_t RB_BYTES[3] = {12, 16, 84};   // positions, rotations, 84-byte particles

int sph_request_readback(sph_ctx* ctx, int32_t fields) {
    if (!ctx || fields <= 0 || (fields & ~(SPH_READBACK_POSITIONS | SPH_READBACK_ROTATIONS | SPH_READBACK_PARTICLES)))
        return SPH_ERR_INVALID;
    if (ctx->slab) return fail(ctx, SPH_ERR_STATE, "slab mode: use sph_slab_read_owned");
    if ((fields & (SPH_READBACK_ROTATIONS | SPH_READBACK_PARTICLES)) && !is_contact(ctx))
        return fail(ctx, SPH_ERR_STATE, "rotations / 84-byte particles are Model R fields");
    HIPCHK(hipSetDevice(ctx->device));
    if (!ctx->rb_stream) {
        HIPCHK(hipStreamCreateWithFlags(&ctx->rb_stream, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&ctx->rb_src, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ctx->rb_ready, hipEventDisableTiming));
    }
    const int32_t n = ctx->n;
    // the previous request's copy must finish before its buffers are overwritten (device-side wait)
    if (ctx->rb_fields) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->rb_ready, 0));
    for (int f = 0; f < 3; ++f) {
        if (!(fields & (1 << f))) continue;
        const size_t need = (size_t)std::max(n, 1) * RB_BYTES[f];
        if (need > ctx->rb_cap[f]) {
            HIPCHK(hipStreamSynchronize(ctx->rb_stream));
            if (ctx->rb_dev[f]) (void)hipFree(ctx->rb_dev[f]);
            if (ctx->rb_host[f]) (void)hipHostFree(ctx->rb_host[f]);
            ctx->rb_dev[f] = ctx->rb_host[f] = nullptr;
            ctx->rb_cap[f] = 0;
            HIPCHK(hipMalloc(&ctx->rb_dev[f], need));
            HIPCHK(hipHostMalloc(&ctx->rb_host[f], need, hipHostMallocDefault));
            ctx->rb_cap[f] = need;
        }
        if (n == 0) continue;
        if (f == 0) launch_scatter_f4_by_id(ctx->pos, ctx->id, n, (float*)ctx->rb_dev[0], 3, ctx->stream);
        if (f == 1) launch_scatter_f4_by_id(ctx->rot, ctx->id, n, (float*)ctx->rb_dev[1], 4, ctx->stream);
        if (f == 2)
            launch_soa_to_aos84(ctx->pos, ctx->vel, ctx->omg, ctx->rot, ctx->aux, ctx->mode, ctx->id, n, ctx->rb_dev[2],
                                ctx->stream);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ctx->rb_src, ctx->stream));
    HIPCHK(hipStreamWaitEvent(ctx->rb_stream, ctx->rb_src, 0));
    for (int f = 0; f < 3; ++f)
        if ((fields & (1 << f)) && n > 0)
            HIPCHK(hipMemcpyAsync(ctx->rb_host[f], ctx->rb_dev[f], (size_t)n * RB_BYTES[f], hipMemcpyDeviceToHost,
                                  ctx->rb_stream));
    HIPCHK(hipEventRecord(ctx->rb_ready, ctx->rb_stream));
    ctx->rb_fields = fields;
    ctx->rb_count = n;
    return SPH_OK;
}

int sph_readback_status(sph_ctx* ctx) {
    if (!ctx) return SPH_ERR_INVALID;
    if (!ctx->rb_fields) return fail(ctx, SPH_ERR_STATE, "no readback requested");
    HIPCHK(hipSetDevice(ctx->device));
    const hipError_t e = hipEventQuery(ctx->rb_ready);
    if (e == hipSuccess) return SPH_OK;
    if (e == hipErrorNotReady) return SPH_READBACK_PENDING;
    return fail(ctx, SPH_ERR_HIP, "readback: %s", hipGetErrorString(e));
}

int sph_readback_get(sph_ctx* ctx, int32_t field, void* dst, int32_t count) {
    if (!ctx || (!dst && count > 0)) return SPH_ERR_INVALID;
    int f = field == SPH_READBACK_POSITIONS ? 0 : field == SPH_READBACK_ROTATIONS ? 1 : field == SPH_READBACK_PARTICLES ? 2 : -1;
    if (f < 0) return SPH_ERR_INVALID;
    if (!(ctx->rb_fields & field)) return fail(ctx, SPH_ERR_STATE, "field %d was not requested", field);
    if (count < ctx->rb_count) return fail(ctx, SPH_ERR_INVALID, "count %d < %d particles read back", count, ctx->rb_count);
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipEventSynchronize(ctx->rb_ready));
    if (ctx->rb_count > 0) std::memcpy(dst, ctx->rb_host[f], (size_t)ctx->rb_count * RB_BYTES[f]);
    return SPH_OK;
}

int sph_readback_count(sph_ctx* ctx, int32_t* count) {
    if (!ctx || !count) return SPH_ERR_INVALID;
    *count = ctx->rb_fields ? ctx->rb_count : 0;
    return SPH_OK;
}

int sph_export_aos84_device(sph_ctx* ctx, void* dev_dst, int32_t count) {
    if (!ctx || (!dev_dst && count > 0)) return SPH_ERR_INVALID;
    if (ctx->slab) return fail(ctx, SPH_ERR_STATE, "slab mode");
    if (count < ctx->n) return fail(ctx, SPH_ERR_INVALID, "count %d < particles %d", count, ctx->n);
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->n > 0)
        launch_soa_to_aos84(ctx->pos, ctx->vel, ctx->omg, ctx->rot, ctx->aux, ctx->mode, ctx->id, ctx->n, dev_dst,
                            ctx->stream);
    HIPCHK(hipGetLastError());
    return SPH_OK;
}

int sph_write_draw_args(sph_ctx* ctx, void* dev_args) {
    if (!ctx || !dev_args) return SPH_ERR_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    const int32_t inst = is_contact(ctx) ? contact_active(ctx) : ctx->n;
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)((uint32_t*)dev_args + 1), inst, 1, ctx->stream));
    return SPH_OK;
}

int sph_synchronize(sph_ctx* ctx) {
    if (!ctx) return SPH_ERR_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

int sph_get_stats(sph_ctx* ctx, sph_stats* out) {
    if (!ctx || !out) return SPH_ERR_INVALID;
    out->steps = ctx->steps;
    out->sim_time = ctx->sim_time;
    out->active = ctx->n;
    out->capacity = ctx->capacity;
    out->grid[0] = ctx->grid.gx; out->grid[1] = ctx->grid.gy; out->grid[2] = ctx->grid.gz;
    out->key_bits = ctx->key_bits;
    out->device_bytes = ctx->device_bytes;
    return SPH_OK;
}

int sph_get_kernel_stat(sph_ctx* ctx, int32_t index, sph_kernel_stat* out) {
    if (!ctx || !out) return SPH_ERR_INVALID;
    if (!ctx->pending.empty()) resolve_pending(ctx);
    if (index < 0 || index >= (int32_t)ctx->kstats.size()) return SPH_ERR_INVALID;
    const KStat& k = ctx->kstats[index];
    std::memset(out, 0, sizeof *out);
    std::snprintf(out->name, sizeof out->name, "%s", k.name.c_str());
    out->launches = k.launches;
    out->total_ms = k.total_ms;
    out->bytes_per_launch = k.bytes;
    return SPH_OK;
}

int sph_reset_kernel_stats(sph_ctx* ctx) {
    if (!ctx) return SPH_ERR_INVALID;
    if (!ctx->pending.empty()) resolve_pending(ctx);
    for (auto& k : ctx->kstats) { k.launches = 0; k.total_ms = 0.0; }
    return SPH_OK;
}

int sph_read_sorted_ids(sph_ctx* ctx, int32_t* ids, int32_t count) {
    if (!ctx || (!ids && count > 0)) return SPH_ERR_INVALID;
    if (count < ctx->n) return fail(ctx, SPH_ERR_INVALID, "count %d < active particles %d", count, ctx->n);
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->n > 0) HIPCHK(hipMemcpyAsync(ids, ctx->id, (size_t)ctx->n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

int sph_read_cell_start(sph_ctx* ctx, uint32_t* cs, int32_t count) {
    if (!ctx || (!cs && count > 0)) return SPH_ERR_INVALID;
    if ((uint32_t)count < ctx->grid.ncells + 1)
        return fail(ctx, SPH_ERR_INVALID, "count %d < ncells+1 = %u", count, ctx->grid.ncells + 1);
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemcpyAsync(cs, ctx->cs, (size_t)(ctx->grid.ncells + 1) * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

int sph_debug_radix_sort(sph_ctx* ctx, const uint32_t* keys, int32_t count, int32_t key_bits, uint32_t* perm_out,
                         uint32_t* sorted_keys_out) {
    if (!ctx || count < 0 || (count > 0 && !keys) || key_bits < 1 || key_bits > 32) return SPH_ERR_INVALID;
    if (count == 0) return SPH_OK;
    HIPCHK(hipSetDevice(ctx->device));
    uint32_t *ka = nullptr, *kb = nullptr, *va = nullptr, *vb = nullptr, *hist = nullptr, *bt = nullptr;
    const size_t nb = (size_t)count * 4;
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipMalloc(&ka, nb);
    if (e == hipSuccess) e = hipMalloc(&kb, nb);
    if (e == hipSuccess) e = hipMalloc(&va, nb);
    if (e == hipSuccess) e = hipMalloc(&vb, nb);
    if (e == hipSuccess) e = hipMalloc(&hist, radix_hist_elems(count) * 4);
    if (e == hipSuccess) e = hipMalloc(&bt, 256 * 4);
    int side = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(ka, keys, nb, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) {
        side = radix_sort(ka, va, kb, vb, count, key_bits, true, hist, bt, ctx->stream);
        e = hipGetLastError();
    }
    if (e == hipSuccess && perm_out) e = hipMemcpyAsync(perm_out, side ? vb : va, nb, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && sorted_keys_out)
        e = hipMemcpyAsync(sorted_keys_out, side ? kb : ka, nb, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(ka); (void)hipFree(kb); (void)hipFree(va); (void)hipFree(vb); (void)hipFree(hist); (void)hipFree(bt);
    if (e != hipSuccess) return fail(ctx, SPH_ERR_HIP, "debug radix sort: %s", hipGetErrorString(e));
    return SPH_OK;
}

int sph_resize(sph_ctx* ctx, int32_t capacity) {
    if (!ctx || capacity < 0) return SPH_ERR_INVALID;
    if (capacity < ctx->n) return fail(ctx, SPH_ERR_CAPACITY, "capacity %d < active particles %d", capacity, ctx->n);
    if (ctx->slab) return fail(ctx, SPH_ERR_STATE, "slab mode");
    HIPCHK(hipSetDevice(ctx->device));
    // keep the particles: device-to-device copies of the slot arrays (no host round trip)
    return grow_d2d(ctx, capacity);
}

// ---------------------------------------------------------------- slab decomposition
// Wait for the last assemble's range copy and publish rng / o0 / o1 (no-op when up to date).
static int slab_sync_ranges(sph_ctx* ctx) {
    if (!ctx->rng_pending) return SPH_OK;
    HIPCHK(hipEventSynchronize(ctx->rng_ev));
    ctx->rng_pending = false;
    const uint32_t* v = ctx->rng_host;
    int32_t* r = ctx->rng;
    r[0] = (int32_t)v[0]; r[1] = (int32_t)v[1];                          // ghost left
    r[2] = (int32_t)v[1]; r[3] = (int32_t)v[4];                          // owned
    r[4] = (int32_t)v[4]; r[5] = (int32_t)v[5];                          // ghost right
    r[6] = (int32_t)v[1]; r[7] = (int32_t)v[2];                          // boundary column cx_lo
    r[8] = (int32_t)v[3]; r[9] = (int32_t)v[4];                          // boundary column cx_hi-1
    ctx->o0 = r[2];
    ctx->o1 = r[3];
    if (r[5] > ctx->n) return fail(ctx, SPH_ERR_STATE, "slab assemble: %d slots > %d particles", r[5], ctx->n);
    ctx->dropped = ctx->n - r[5];   // own particles outside the held columns, already sent away
    ctx->n = r[5];
    return SPH_OK;
}

static int slab_local_grid(sph_ctx* ctx) {
    const GridDesc& G = ctx->gglobal;
    GridDesc g = G;
    ctx->has_left = ctx->sl.cx_lo > 0;
    ctx->has_right = ctx->sl.cx_hi < G.gx;
    g.cx0 = ctx->sl.cx_lo - (ctx->has_left ? 1 : 0);
    g.gx = ctx->sl.cx_hi + (ctx->has_right ? 1 : 0) - g.cx0;
    g.gx_all = G.gx;
    g.ncells = (uint32_t)g.gx * (uint32_t)g.gy * (uint32_t)g.gz;
    ctx->grid = g;
    ctx->key_bits = bit_width(g.ncells);
    ctx->keys_valid = false;
    ctx->sk_valid = false;
    return ensure_cells(ctx);
}

static inline int32_t col_start(const sph_ctx* c, int32_t local_col) {
    return local_col * c->grid.gy * c->grid.gz;
}

int sph_slab_set(sph_ctx* ctx, const sph_slab* slab) {
    if (!ctx || !slab) return SPH_ERR_INVALID;
    if (is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "slab decomposition is Model S only");
    if (!ctx->params_set) return fail(ctx, SPH_ERR_STATE, "sph_set_params first");
    HIPCHK(hipSetDevice(ctx->device));
    if (!ctx->slab) ctx->gglobal = ctx->grid;
    const int32_t GX = ctx->gglobal.gx;
    if (slab->cx_lo < 0 || slab->cx_hi > GX || slab->cx_lo >= slab->cx_hi)
        return fail(ctx, SPH_ERR_INVALID, "slab [%d,%d) outside 0..%d", slab->cx_lo, slab->cx_hi, GX);
    if (!ctx->rng_host) HIPCHK(hipHostMalloc((void**)&ctx->rng_host, 16 * sizeof(uint32_t), hipHostMallocDefault));
    if (!ctx->rng_ev) HIPCHK(hipEventCreateWithFlags(&ctx->rng_ev, hipEventDisableTiming));
    ctx->slab = true;
    ctx->sl = *slab;
    ctx->n = ctx->o0 = ctx->o1 = 0;
    ctx->rng_pending = false;
    return slab_local_grid(ctx);
}

int sph_slab_recut(sph_ctx* ctx, const sph_slab* slab) {
    if (!ctx || !slab) return SPH_ERR_INVALID;
    if (!ctx->slab) return fail(ctx, SPH_ERR_STATE, "sph_slab_set first");
    const int32_t GX = ctx->gglobal.gx;
    if (slab->cx_lo < 0 || slab->cx_hi > GX || slab->cx_lo >= slab->cx_hi)
        return fail(ctx, SPH_ERR_INVALID, "slab [%d,%d) outside 0..%d", slab->cx_lo, slab->cx_hi, GX);
    if (int rc = slab_sync_ranges(ctx)) return rc;
    HIPCHK(hipSetDevice(ctx->device));
    // the owned slots [o0, o1) keep their particles; only the held window moves. Their keys are
    // recomputed in the new window by the next count_sends.
    ctx->sl = *slab;
    return slab_local_grid(ctx);
}

int sph_slab_column_counts(sph_ctx* ctx, int64_t* counts, int32_t ncols) {
    if (!ctx || !counts) return SPH_ERR_INVALID;
    if (!ctx->slab) return fail(ctx, SPH_ERR_STATE, "not in slab mode");
    if (ncols < ctx->gglobal.gx) return fail(ctx, SPH_ERR_INVALID, "ncols %d < columns %d", ncols, ctx->gglobal.gx);
    if (int rc = slab_sync_ranges(ctx)) return rc;
    HIPCHK(hipSetDevice(ctx->device));
    for (int32_t c = 0; c < ncols; ++c) counts[c] = 0;
    const int32_t m = ctx->sl.cx_hi - ctx->sl.cx_lo + 1;
    std::vector<uint32_t> st(m);
    const uint32_t gyz = (uint32_t)ctx->grid.gy * (uint32_t)ctx->grid.gz;
    launch_column_starts(ctx->cs, gyz, ctx->sl.cx_lo - ctx->grid.cx0, m, (uint32_t*)ctx->staging, ctx->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(st.data(), ctx->staging, (size_t)m * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (int32_t k = 0; k + 1 < m; ++k) counts[ctx->sl.cx_lo + k] = (int64_t)st[k + 1] - (int64_t)st[k];
    return SPH_OK;
}

int sph_slab_init_scenario(sph_ctx* ctx, const sph_scenario* sc) {
    if (!ctx || !sc) return SPH_ERR_INVALID;
    if (!ctx->slab) return fail(ctx, SPH_ERR_STATE, "sph_slab_set first");
    const int64_t N = (int64_t)sc->nx * sc->ny * (sc->dim == 3 ? sc->nz : 1);
    if (N <= 0 || N > 0x7fffffff) return fail(ctx, SPH_ERR_INVALID, "bad scenario size");
    HIPCHK(hipSetDevice(ctx->device));
    float4 *gp = nullptr, *gv = nullptr;
    int32_t* gi = nullptr;
    uint32_t* blk = nullptr;
    const int32_t nb = slab_compact_blocks(0, (int32_t)N);
    hipError_t e = hipMalloc(&gp, N * sizeof(float4));
    if (e == hipSuccess) e = hipMalloc(&gv, N * sizeof(float4));
    if (e == hipSuccess) e = hipMalloc(&gi, N * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&blk, (2 * (size_t)nb + 2) * sizeof(uint32_t));
    uint32_t total = 0;
    if (e == hipSuccess) {
        launch_lattice(sc->dim, sc->nx, sc->ny, sc->nz, sc->dx, 0.f, 0.f, 0.f, sc->seed, sc->jitter * sc->dx, gp, gv,
                       gi, ctx->stream);
        // count first: the owned part must fit the context
        launch_slab_select_columns(gp, gv, gi, (int32_t)N, ctx->gglobal, ctx->sl.cx_lo, ctx->sl.cx_hi, blk,
                                   ctx->sdev, nullptr, nullptr, nullptr, ctx->stream);
        e = hipMemcpyAsync(&total, ctx->sdev, 4, hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    }
    if (e == hipSuccess && (int64_t)total > ctx->capacity) {
        (void)hipFree(gp); (void)hipFree(gv); (void)hipFree(gi); (void)hipFree(blk);
        return fail(ctx, SPH_ERR_CAPACITY, "slab owns %u particles > capacity %d", total, ctx->capacity);
    }
    if (e == hipSuccess) {
        launch_slab_select_columns(gp, gv, gi, (int32_t)N, ctx->gglobal, ctx->sl.cx_lo, ctx->sl.cx_hi, blk,
                                   ctx->sdev, ctx->pos, ctx->vel, ctx->id, ctx->stream);
        e = hipStreamSynchronize(ctx->stream);
    }
    (void)hipFree(gp); (void)hipFree(gv); (void)hipFree(gi); (void)hipFree(blk);
    if (e != hipSuccess) return fail(ctx, SPH_ERR_HIP, "slab init: %s", hipGetErrorString(e));
    ctx->n = ctx->o1 = (int32_t)total;
    ctx->o0 = 0;
    ctx->keys_valid = false;
    ctx->sk_valid = false;
    ctx->steps = 0;
    ctx->sim_time = 0.0;
    return SPH_OK;
}

static int slab_count(sph_ctx* ctx, int64_t* dev_counts) {
    if (int rc = slab_sync_ranges(ctx)) return rc;
    const int32_t no = ctx->o1 - ctx->o0;
    if (!ctx->keys_valid && no > 0) {
        KTimer t(ctx, "keys", 20.0 * no);
        launch_keys(ctx->pos + ctx->o0, no, nullptr, 0, ctx->grid, ctx->keys + ctx->o0, ctx->stream);
        ctx->keys_valid = true;
    }
    const uint32_t gyz = (uint32_t)ctx->grid.gy * (uint32_t)ctx->grid.gz;
    const int32_t col_le = ctx->has_left ? ctx->sl.cx_lo - ctx->grid.cx0 : -1;
    const int32_t col_ge = ctx->has_right ? ctx->sl.cx_hi - 1 - ctx->grid.cx0 : 0x7fffffff;
    KTimer t(ctx, "slab_count", 4.0 * no);
    launch_slab_count(ctx->keys, ctx->o0, ctx->o1, gyz, col_le, col_ge, ctx->sblk, ctx->sdev, ctx->stream, dev_counts);
    return SPH_OK;
}

int sph_slab_count_sends_async(sph_ctx* ctx, int64_t* dev_counts) {
    if (!ctx || !dev_counts) return SPH_ERR_INVALID;
    if (!ctx->slab) return fail(ctx, SPH_ERR_STATE, "not in slab mode");
    HIPCHK(hipSetDevice(ctx->device));
    if (int rc = slab_count(ctx, dev_counts)) return rc;
    HIPCHK(hipGetLastError());
    ctx->send_counts[0] = ctx->send_counts[1] = -1;   // known on the device only
    return SPH_OK;
}

int sph_slab_send_capacity(sph_ctx* ctx, int32_t* capacity) {
    if (!ctx || !capacity) return SPH_ERR_INVALID;
    if (int rc = slab_sync_ranges(ctx)) return rc;
    *capacity = std::max(ctx->o1 - ctx->o0, 1);
    return SPH_OK;
}

int sph_slab_count_sends(sph_ctx* ctx, int32_t counts[2]) {
    if (!ctx || !counts) return SPH_ERR_INVALID;
    if (!ctx->slab) return fail(ctx, SPH_ERR_STATE, "not in slab mode");
    HIPCHK(hipSetDevice(ctx->device));
    if (int rc = slab_count(ctx, nullptr)) return rc;
    uint32_t tot[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(tot, ctx->sdev, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    counts[0] = ctx->send_counts[0] = (int32_t)tot[0];
    counts[1] = ctx->send_counts[1] = (int32_t)tot[1];
    return SPH_OK;
}

int sph_slab_pack_send(sph_ctx* ctx, int32_t side, void* dev_records, int32_t capacity) {
    if (!ctx || side < 0 || side > 1) return SPH_ERR_INVALID;
    if (!ctx->slab) return fail(ctx, SPH_ERR_STATE, "not in slab mode");
    if (ctx->send_counts[side] == 0) return SPH_OK;
    // exact count known on the host (count_sends), or only on the device (count_sends_async):
    // then the buffer must hold every owned particle
    const int32_t need = ctx->send_counts[side] > 0 ? ctx->send_counts[side] : ctx->o1 - ctx->o0;
    if (!dev_records || capacity < need)
        return fail(ctx, SPH_ERR_CAPACITY, "send buffer %d < %d records", capacity, need);
    HIPCHK(hipSetDevice(ctx->device));
    const uint32_t gyz = (uint32_t)ctx->grid.gy * (uint32_t)ctx->grid.gz;
    const int32_t col_le = ctx->has_left ? ctx->sl.cx_lo - ctx->grid.cx0 : -1;
    const int32_t col_ge = ctx->has_right ? ctx->sl.cx_hi - 1 - ctx->grid.cx0 : 0x7fffffff;
    KTimer t(ctx, "slab_pack", 36.0 * ctx->send_counts[side]);
    // old sorted keys travel with the records (global keys) for the receiver's incremental re-sort
    launch_slab_pack(ctx->keys, ctx->pos, ctx->vel, ctx->id, ctx->sk_valid ? ctx->sk_cur : nullptr,
                     (uint32_t)ctx->grid.cx0 * gyz, ctx->o0, ctx->o1, gyz, side, col_le, col_ge, ctx->sblk,
                     (float4*)dev_records, ctx->stream);
    HIPCHK(hipGetLastError());
    return SPH_OK;
}

// The slab step's sort. [from left | own | from right] is the canonical pre-sort order: both ranks
// sharing a column then break key ties identically (SPEC_SPH.md §3). Its OLD keys are sorted: the
// own block keeps the previous sorted order, and the neighbours' records carry their old keys, all
// below (left) or above (right) the owned columns. So the incremental re-sort applies to the whole
// assembled array, with movers = every slot whose key changed (records included), and gives the
// same permutation as the full radix sort (tests/test_gpu_slab.py compares the two bit for bit).
// The full radix sort runs after any window change (no valid old keys) and while the last seen
// mover count exceeds resort_limit.
int sph_slab_assemble(sph_ctx* ctx, const void* dev_left, int32_t nl, const void* dev_right, int32_t nr) {
    if (!ctx || nl < 0 || nr < 0 || (nl > 0 && !dev_left) || (nr > 0 && !dev_right)) return SPH_ERR_INVALID;
    if (!ctx->slab) return fail(ctx, SPH_ERR_STATE, "not in slab mode");
    HIPCHK(hipSetDevice(ctx->device));
    const int32_t no = ctx->o1 - ctx->o0;
    const int64_t n = (int64_t)nl + no + nr;
    if (n > ctx->capacity) return fail(ctx, SPH_ERR_CAPACITY, "slab needs %lld slots > capacity %d", (long long)n, ctx->capacity);
    hipStream_t s = ctx->stream;
    const uint32_t gyz = (uint32_t)ctx->grid.gy * (uint32_t)ctx->grid.gz;
    const uint32_t key_base = (uint32_t)ctx->grid.cx0 * gyz;
    const bool many = ctx->resort_mode == 1 && *(volatile uint32_t*)ctx->mv_host > resort_limit((int32_t)n);
    // ranges from the cell table at column starts: picked on the device (density reads them there)
    // and written to mapped pinned memory; slab_sync_ranges waits for the event after the sort
    const int32_t lc_lo = ctx->sl.cx_lo - ctx->grid.cx0, lc_hi = ctx->sl.cx_hi - ctx->grid.cx0;
    const int32_t idx[6] = {col_start(ctx, 0), col_start(ctx, lc_lo), col_start(ctx, lc_lo + 1),
                            col_start(ctx, lc_hi - 1), col_start(ctx, lc_hi), col_start(ctx, ctx->grid.gx)};
    if (ctx->resort_mode != 0 && !many && ctx->sk_valid && n > 0) {
        // incremental: the re-sort reads [left records | own slots | right records] in place. The force
        // pass already appended the own movers (window keys); the records' keys and movers join here.
        const AsmSrc src{ctx->pos, ctx->vel, ctx->id, ctx->sk_cur, ctx->keys, ctx->o0 - nl, (const float4*)dev_left,
                         (const float4*)dev_right, ctx->keys2, ctx->vals, nl, nl + no};
        const int used = ctx->mv_par;
        const MoverSink mv{ctx->keys2, ctx->mv_count + used, ctx->mv_mi, ctx->mv_mk, ctx->mv_mo, ctx->mv_rank,
                           (uint32_t)std::max(ctx->capacity, 1)};
        {
            KTimer t(ctx, "slab_assemble", 40.0 * (double)(nl + nr));
            launch_slab_rec(src, (int32_t)n, ctx->grid, key_base, ctx->vals, ctx->keys2, mv, s);
        }
        KTimer t(ctx, "resort", (double)n * (2 * 4 + 2 * 36));
        launch_slab_cs_old(ctx->cs, ctx->grid.ncells, gyz, (uint32_t)ctx->grid.gx, ctx->has_left, ctx->has_right,
                           nl - ctx->o0, ctx->keys2, nl, no, nr, s);
        CsPick pick{{0}, 6, ctx->sdev, ctx->rng_host};   // the ranges, read as the cell table completes
        for (int k = 0; k < 6; ++k) pick.idx[k] = idx[k];
        ResortScratch w = resort_scratch(ctx);
        w.mi_off = nl - ctx->o0;   // own movers were appended by slot in the previous order
        launch_resort(src, ctx->cs, ctx->grid.ncells, (int32_t)n, ctx->mv_count + used, ctx->mv_count + (1 - used), w,
                      ctx->pos2, ctx->vel2, ctx->id2, ctx->sk_next, s, pick);
        if ((ctx->steps & 7) == 0)
            HIPCHK(hipMemcpyAsync(ctx->mv_host, ctx->mv_count + used, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        ctx->mv_par = 1 - used;
        swap_sv(ctx);
        std::swap(ctx->id, ctx->id2);
        std::swap(ctx->sk_cur, ctx->sk_next);
    } else {
        {
            KTimer t(ctx, "slab_assemble", 64.0 * (double)n);
            launch_slab_unpack((const float4*)dev_left, nl, ctx->pos2, ctx->vel2, ctx->id2, s);
            if (no > 0) {
                HIPCHK(hipMemcpyAsync(ctx->pos2 + nl, ctx->pos + ctx->o0, (size_t)no * 16, hipMemcpyDeviceToDevice, s));
                HIPCHK(hipMemcpyAsync(ctx->vel2 + nl, ctx->vel + ctx->o0, (size_t)no * 16, hipMemcpyDeviceToDevice, s));
                HIPCHK(hipMemcpyAsync(ctx->id2 + nl, ctx->id + ctx->o0, (size_t)no * 4, hipMemcpyDeviceToDevice, s));
            }
            launch_slab_unpack((const float4*)dev_right, nr, ctx->pos2 + nl + no, ctx->vel2 + nl + no,
                               ctx->id2 + nl + no, s);
            // own particles outside the held columns were sent away this step: they sort last and drop
            launch_keys(ctx->pos2, (int32_t)n, nullptr, 0, ctx->grid, ctx->keys, s, true);
        }
        int side;
        {
            const int passes = (ctx->key_bits + 7) / 8;
            KTimer t(ctx, "radix_sort", (double)n * (20.0 * passes));
            side = radix_sort(ctx->keys, ctx->vals, ctx->keys2, ctx->vals2, (int32_t)n, ctx->key_bits, true, ctx->hist,
                              ctx->bin_total, s);
        }
        const uint32_t* sk = side ? ctx->keys2 : ctx->keys;
        const uint32_t* perm = side ? ctx->vals2 : ctx->vals;
        {
            KTimer t(ctx, "reorder", (double)n * (4 + 2 * 36));
            launch_gather_s(perm, ctx->pos2, ctx->vel2, ctx->id2, ctx->pos, ctx->vel, ctx->id, (int32_t)n, s);
        }
        {
            KTimer t(ctx, "cell_start", 4.0 * (ctx->grid.ncells + 1));
            launch_cell_start(sk, (int32_t)n, ctx->cs, ctx->grid.ncells, ctx->gaps, ctx->sdev + 8, &ctx->gap_par, s);
        }
        // the sorted keys of the new slot order: the next step's old keys
        if (ctx->resort_mode != 0 && n > 0)
            HIPCHK(hipMemcpyAsync(ctx->sk_cur, sk, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemsetAsync(ctx->mv_count, 0, 2 * sizeof(uint32_t), s));
        launch_pick(ctx->cs, idx, 6, ctx->sdev, s, ctx->rng_host);
    }
    HIPCHK(hipEventRecord(ctx->rng_ev, s));
    ctx->rng_pending = true;
    ctx->n = (int32_t)n;
    ctx->keys_valid = false;
    ctx->sk_valid = ctx->resort_mode != 0;
    return SPH_OK;
}

int sph_slab_ranges(sph_ctx* ctx, int32_t ranges[10]) {
    if (!ctx || !ranges) return SPH_ERR_INVALID;
    int rc = slab_sync_ranges(ctx);
    if (rc != SPH_OK) return rc;
    std::memcpy(ranges, ctx->rng, sizeof ctx->rng);
    return SPH_OK;
}

int sph_slab_density(sph_ctx* ctx) {
    if (!ctx) return SPH_ERR_INVALID;
    if (!ctx->slab) return fail(ctx, SPH_ERR_STATE, "not in slab mode");
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->rng_pending) {   // owned range [sdev[1], sdev[4]) on the device; grid sized for all slots
        KTimer t(ctx, "density", 24.0 * ctx->n);
        const DevRange dr{ctx->sdev + 1, ctx->sdev + 4};
        if (ctx->nb_variant == 0)
            launch_density(ctx->pos, ctx->cs, 0, ctx->n, ctx->grid, ctx->sc, ctx->rp, ctx->stream, dr);
        else
            launch_density_tiled(ctx->pos, ctx->cs, 0, ctx->n, ctx->grid, ctx->sc, ctx->rp, ctx->stream, dr);
        HIPCHK(hipGetLastError());
        return SPH_OK;
    }
    KTimer t(ctx, "density", 24.0 * (ctx->o1 - ctx->o0));
    density_range(ctx, ctx->o0, ctx->o1);
    HIPCHK(hipGetLastError());
    return SPH_OK;
}

int sph_slab_pack_rho(sph_ctx* ctx, int32_t side, void* dev, int32_t capacity) {
    if (!ctx || side < 0 || side > 1) return SPH_ERR_INVALID;
    if (int rc = slab_sync_ranges(ctx)) return rc;
    const int32_t b = ctx->rng[6 + 2 * side], e = ctx->rng[7 + 2 * side];
    if (e == b) return SPH_OK;
    if (!dev || capacity < e - b) return fail(ctx, SPH_ERR_CAPACITY, "rho buffer %d < %d", capacity, e - b);
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemcpyAsync(dev, ctx->rp + b, (size_t)(e - b) * sizeof(float2), hipMemcpyDeviceToDevice, ctx->stream));
    return SPH_OK;
}

int sph_slab_unpack_rho(sph_ctx* ctx, int32_t side, const void* dev, int32_t count) {
    if (!ctx || side < 0 || side > 1) return SPH_ERR_INVALID;
    if (int rc = slab_sync_ranges(ctx)) return rc;
    const int32_t b = ctx->rng[4 * side], e = ctx->rng[4 * side + 1];
    if (count != e - b)
        return fail(ctx, SPH_ERR_STATE, "ghost column %d holds %d particles but %d densities arrived", side, e - b, count);
    if (count == 0) return SPH_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemcpyAsync(ctx->rp + b, dev, (size_t)count * sizeof(float2), hipMemcpyDeviceToDevice, ctx->stream));
    return SPH_OK;
}

static void slab_force_range(sph_ctx* ctx, float dt, int32_t b, int32_t e) {
    if (e <= b) return;
    const sph_params& p = ctx->prm;
    const float tt = (float)ctx->sim_time;
    const float fext = p.forcing_amp != 0.0f ? p.forcing_amp * sinf(6.28318530718f * p.forcing_freq * tt) : 0.0f;
    KTimer t(ctx, "force_integrate", 76.0 * (e - b));
    force_range(ctx, b, e, dt, fext, mover_sink(ctx));   // own movers for the next assemble's re-sort
}

int sph_slab_force(sph_ctx* ctx, float dt, int32_t part) {
    if (!ctx || part < 0 || part > 2) return SPH_ERR_INVALID;
    if (!ctx->slab) return fail(ctx, SPH_ERR_STATE, "not in slab mode");
    if (int rc = slab_sync_ranges(ctx)) return rc;
    HIPCHK(hipSetDevice(ctx->device));
    const int32_t* r = ctx->rng;
    // interior = owned slots whose neighbourhood holds no ghost
    const int32_t ib = ctx->has_left ? r[7] : r[2];
    const int32_t ie = ctx->has_right ? r[8] : r[3];
    if (part == 0) {
        slab_force_range(ctx, dt, r[2], r[3]);
    } else if (part == 1) {
        slab_force_range(ctx, dt, ib, std::max(ib, ie));
    } else {
        if (ie < ib) {                  // one-column slab: boundary columns coincide
            slab_force_range(ctx, dt, r[2], r[3]);
        } else {
            slab_force_range(ctx, dt, r[2], ib);
            slab_force_range(ctx, dt, ie, r[3]);
        }
    }
    HIPCHK(hipGetLastError());
    return SPH_OK;
}

int sph_slab_finish_step(sph_ctx* ctx, float dt) {
    if (!ctx) return SPH_ERR_INVALID;
    swap_sv(ctx);
    ctx->keys_valid = true;
    ctx->steps++;
    ctx->sim_time += (double)dt;
    return SPH_OK;
}

int sph_slab_read_owned(sph_ctx* ctx, float* rec, int32_t count, int32_t* n_owned) {
    if (!ctx || !n_owned) return SPH_ERR_INVALID;
    if (int rc = slab_sync_ranges(ctx)) return rc;
    const int32_t no = ctx->o1 - ctx->o0;
    *n_owned = no;
    if (count < no || (no > 0 && !rec)) return fail(ctx, SPH_ERR_INVALID, "count %d < owned %d", count, no);
    HIPCHK(hipSetDevice(ctx->device));
    if (no > 0) {
        launch_pack_owned(ctx->pos, ctx->vel, ctx->id, ctx->rp, ctx->o0, no, (float*)ctx->staging, ctx->stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(rec, ctx->staging, (size_t)no * 32, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

}  // extern "C"
