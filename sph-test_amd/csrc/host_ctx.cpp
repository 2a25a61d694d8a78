// host_ctx.cpp — context memory, grid derivation and per-kernel profiling (see host.h).
#include <cstdlib>
#include "host.h"

namespace sph {

void free_all(sph_ctx* c) {
    dfree(c->pos); dfree(c->vel); dfree(c->pos2); dfree(c->vel2);
    dfree(c->omg); dfree(c->rot); dfree(c->aux); dfree(c->omg2); dfree(c->rot2); dfree(c->aux2);
    dfree(c->id); dfree(c->id2); dfree(c->mode); dfree(c->mode2);
    dfree(c->rp); dfree(c->torque); dfree(c->slot_of);
    dfree(c->keys); dfree(c->keys2); dfree(c->vals); dfree(c->vals2); dfree(c->hist); dfree(c->bin_total);
    dfree(c->cs); dfree(c->cs2); dfree(c->gaps);
    c->gaps_cap = 0;
    dfree(c->sblk); dfree(c->sdev); dfree(c->paths); dfree(c->hmask);
    dfree(c->sk_cur); dfree(c->sk_next);
    dfree(c->mv_mi); dfree(c->mv_mk); dfree(c->mv_mo); dfree(c->mv_mx); dfree(c->mv_mos);
    dfree(c->mv_ms); dfree(c->mv_count); dfree(c->mv_mi2); dfree(c->mv_mk2); dfree(c->mv_mo2);
    c->fz_ready = false;
    dfree(c->sched);
    c->sched_cap = 0;
    c->sched_valid = false;
    c->sk_valid = false;
    if (c->staging) (void)hipFree(c->staging);
    c->staging = nullptr;
    c->staging_bytes = 0;
    c->cs_cap = 0;
    c->cs2_cap = 0;
    c->device_bytes = 0;
}

int bit_width(uint32_t v) {
    int b = 0;
    while (v) { ++b; v >>= 1; }
    return b < 1 ? 1 : b;
}


int alloc_particles(sph_ctx* ctx, int32_t cap) {
    const size_t n = (size_t)std::max(cap, 1);
    int r;
#define AL(p, cnt) if ((r = dalloc(ctx, &ctx->p, cnt)) != SPH_OK) return r
    AL(pos, n); AL(vel, n); AL(pos2, n); AL(vel2, n);
    AL(id, n); AL(id2, n);
    AL(keys, n); AL(keys2, n); AL(vals, n); AL(vals2, n);
    AL(hist, radix_hist_elems((int32_t)n)); AL(bin_total, 256);
    AL(sblk, 2 * (size_t)slab_compact_blocks(0, (int32_t)n) + 2); AL(sdev, 16); AL(paths, 24);
    HIPCHK(hipMemset(ctx->sdev, 0, 16 * sizeof(uint32_t)));
    {   // the contact pass's radius bound: +inf (no cell skipped) until the first key pass computes it
        const uint32_t inf = 0x7f800000u;
        HIPCHK(hipMemcpy(ctx->sdev + SDEV_RMAX, &inf, sizeof inf, hipMemcpyHostToDevice));
    }
    HIPCHK(hipMemset(ctx->paths, 0, 24 * sizeof(uint32_t)));
    ctx->gap_par = 0;
    if (is_contact(ctx)) {
        AL(omg, n); AL(rot, n); AL(aux, n); AL(omg2, n); AL(rot2, n); AL(aux2, n);
        AL(mode, n); AL(mode2, n); AL(torque, 3 * n); AL(slot_of, n);
    } else {
        AL(rp, n);
        AL(hmask, (size_t)(HM_WORDS + 1) * n);   // + the writer's overflow row (wcsph_tiled.hip)
    }
    // incremental re-sort (both models)
    AL(sk_cur, n); AL(sk_next, n);
    AL(mv_mi, n); AL(mv_mk, n); AL(mv_mo, n); AL(mv_mx, n); AL(mv_mos, n); AL(mv_ms, n);
    AL(mv_count, 3);
    HIPCHK(hipMemset(ctx->mv_count, 0, 3 * sizeof(uint32_t)));
    if (is_contact(ctx)) { AL(mv_mi2, n); AL(mv_mk2, n); AL(mv_mo2, n); }
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
    if (need > ctx->cs2_cap) {
        int r = dalloc(ctx, &ctx->cs2, need);
        if (r != SPH_OK) return r;
        ctx->cs2_cap = need;
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

int32_t model_s_xsub() {
    if (const char* v = std::getenv("SPH_XSUB")) {
        const int x = std::atoi(v);
        if (x == 1 || x == 2) return x;
    }
    return SPH_XSUB_DEFAULT;
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
        g.xsub = 1;
        g.inv_cxs = g.inv_cell;
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
        g.xsub = ctx->cfg.dim == 3 ? model_s_xsub() : 1;
        g.inv_cxs = g.inv_cell * (float)g.xsub;   // exact (xsub is 1 or 2)
        int32_t G[3];
        for (int a = 0; a < 3; ++a) {
            G[a] = (int32_t)floorf(p.box[a] / (a == 2 ? cz : cell)) + 1;
            if (G[a] < 1) G[a] = 1;
        }
        if (ctx->cfg.dim == 2) G[2] = 1;
        g.gx = G[0]; g.gy = G[1]; g.gz = G[2];
        const double nc = (double)G[0] * g.xsub * G[1] * G[2];
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
        s.inv_h2 = s.inv_h * s.inv_h;
        s.two_h = 2.0f * h;
        s.m6h = -6.0f * h;
        s.four_h3 = 4.0f * h * h * h;
        s.rho_scale = s.mass * s.sigma / s.four_h3;
    }
    g.cx0 = 0;
    g.gx_all = g.gx;
    g.ncells = (uint32_t)g.gx * col_keys(g);
    ctx->grid = g;
    ctx->key_bits = bit_width(g.ncells);   // the sentinel key == ncells must sort last
    invalidate_sort(ctx);
    return ensure_cells(ctx);
}

void invalidate_sort(sph_ctx* c) {
    c->keys_valid = false;
    c->sk_valid = false;
    c->hm_valid = false;
    c->sched_valid = false;
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

thread_local LaunchEvents* g_launch_events = nullptr;

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
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            c->kstats[p.k].total_ms += ms;
            c->kstats[p.k].timed++;
        }
        c->ev_pool.push_back(p.a);
        c->ev_pool.push_back(p.b);
    }
    c->pending.clear();
}

}  // namespace sph
