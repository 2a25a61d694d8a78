// host_step.cpp — the per-step launch sequences of both models (see host.h).
#include "host.h"

namespace sph {

void swap_sv(sph_ctx* c) {
    std::swap(c->pos, c->pos2);
    std::swap(c->vel, c->vel2);
}

int sort_and_reorder(sph_ctx* ctx, int32_t n_active_id, const uint32_t** sorted_keys) {
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

HitMask hit_mask_write(sph_ctx* ctx) {
    ctx->hm_valid = ctx->hmask != nullptr;
    return HitMask{ctx->hmask, (uint32_t)std::max(ctx->capacity, 1)};
}

HitMask hit_mask_read(const sph_ctx* ctx) {
    return ctx->hm_valid ? HitMask{ctx->hmask, (uint32_t)std::max(ctx->capacity, 1)} : HitMask{};
}

void density_range(sph_ctx* ctx, int32_t b, int32_t e) {
    launch_density_tiled(ctx->pos, ctx->cs, b, e, ctx->grid, ctx->sc, ctx->rp, hit_mask_write(ctx), path_ctr(ctx), ctx->stream);
}

void force_range(sph_ctx* ctx, int32_t b, int32_t e, float dt, float fext, MoverSink mv) {
    launch_force_tiled(ctx->pos, ctx->vel, ctx->rp, ctx->cs, b, e, ctx->grid, ctx->sc, dt, fext, ctx->pos2, ctx->vel2,
                       ctx->keys, mv, hit_mask_read(ctx), path_ctr(ctx), ctx->stream);
}

// f_ext(t) of SPEC_SPH.md §2 at the context's simulated time (sloshing; 0 otherwise)
float forcing(const sph_ctx* ctx) {
    const sph_params& p = ctx->prm;
    const float tt = (float)ctx->sim_time;
    return p.forcing_amp != 0.0f ? p.forcing_amp * sinf(6.28318530718f * p.forcing_freq * tt) : 0.0f;
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
    ctx->hm_valid = false;
    // adaptive mode: the latest mover count the host has seen (a step or more behind the device;
    // both paths give the same permutation, so the choice only affects time)
    const bool many = ctx->resort_mode == 1 && *(volatile uint32_t*)ctx->mv_host > resort_limit(n);
    if (ctx->resort_mode != 0 && !many && ctx->keys_valid && ctx->keys_active == 0 && ctx->sk_valid) {
        {
            KTimer t(ctx, "resort", (double)n * (2 * 4 + 2 * 36), true);
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

// ---------------------------------------------------------------- chunked neighbour passes
// The density pass ends in a tail of partly filled CUs (its last round of workgroups), and so does
// the force pass: at C3 ~20% and ~14% of their spans. Cut at x-planes into S chunks of
// about equal particle counts, the density chunks run in order on the context stream and the force
// chunks on a second stream, force chunk k after density chunk k + 1: its targets' neighbours lie
// within one plane, and chunk k + 1 holds at least one plane. Each pass's tail then overlaps the
// other pass's workgroups. Every target is computed exactly as in one launch (same windows, same
// order), so results are bit-identical for any S.
void free_chunks(sph_ctx* c) {
    if (c->stream2) {
        (void)hipStreamSynchronize(c->stream2);
        (void)hipStreamDestroy(c->stream2);
        c->stream2 = nullptr;
    }
    for (auto& e : c->ev_chunk)
        if (e) { (void)hipEventDestroy(e); e = nullptr; }
    if (c->plane_ev) { (void)hipEventDestroy(c->plane_ev); c->plane_ev = nullptr; }
    if (c->plane_host) { (void)hipHostFree(c->plane_host); c->plane_host = nullptr; }
    c->plane_host_cap = 0;
    c->plane_pending = false;
}

static int ensure_chunks(sph_ctx* ctx) {
    if (ctx->stream2) return SPH_OK;
    HIPCHK(hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking));
    for (auto& e : ctx->ev_chunk) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ctx->plane_ev, hipEventDisableTiming));
    return SPH_OK;
}

// the current plane starts (cs at every x-plane) into pinned memory, on the context stream
static int plane_copy(sph_ctx* ctx) {
    const int32_t gx = ctx->grid.gx;
    if (ctx->plane_host_cap < gx + 1) {
        if (ctx->plane_host) HIPCHK(hipHostFree(ctx->plane_host));
        ctx->plane_host = nullptr;
        HIPCHK(hipHostMalloc((void**)&ctx->plane_host, (size_t)(gx + 1) * sizeof(uint32_t), hipHostMallocMapped));
        ctx->plane_host_cap = gx + 1;
    }
    launch_plane_starts(ctx->cs, (uint32_t)ctx->grid.gy * (uint32_t)ctx->grid.gz, gx, ctx->plane_host, ctx->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ctx->plane_ev, ctx->stream));
    ctx->plane_pending = true;
    ctx->plane_step = ctx->steps;
    return SPH_OK;
}

// S cuts at planes, about equal particle counts, strictly increasing (every chunk holds a plane)
static void choose_cuts(sph_ctx* ctx, int S, std::vector<int32_t>& est) {
    const int32_t gx = ctx->grid.gx;
    const uint32_t* ps = ctx->plane_host;
    const double total = (double)ps[gx];
    std::vector<int32_t>& cut = ctx->chunk_cx;
    cut.assign((size_t)S + 1, 0);
    for (int k = 1; k < S; ++k) {
        const double target = total * k / S;
        int32_t c = (int32_t)(std::lower_bound(ps, ps + gx + 1, (uint32_t)target) - ps);
        c = std::max(c, cut[(size_t)k - 1] + 1);
        c = std::min(c, gx - (S - k));
        cut[(size_t)k] = c;
    }
    cut[(size_t)S] = gx;
    est.assign((size_t)S, 0);
    for (int k = 0; k < S; ++k) est[(size_t)k] = (int32_t)(ps[cut[(size_t)k + 1]] - ps[cut[(size_t)k]]);
}

static int step_wcsph_chunked(sph_ctx* ctx, float dt, int S) {
    int r = ensure_chunks(ctx);
    if (r != SPH_OK) return r;
    // the cuts: from plane starts copied asynchronously (every 32 steps; particles cross planes slowly),
    // or, when none are known for this grid, copied and waited for now. The counts only balance the
    // chunks and size their grids: the kernels read their bounds from cs and loop over extra tiles.
    if (ctx->plane_pending && hipEventQuery(ctx->plane_ev) == hipSuccess) {
        choose_cuts(ctx, S, ctx->chunk_est);
        ctx->plane_pending = false;
    }
    if ((int)ctx->chunk_cx.size() != S + 1) {
        if ((r = plane_copy(ctx)) != SPH_OK) return r;
        HIPCHK(hipEventSynchronize(ctx->plane_ev));
        choose_cuts(ctx, S, ctx->chunk_est);
        ctx->plane_pending = false;
    } else if (!ctx->plane_pending && ctx->steps - ctx->plane_step >= 32) {
        if ((r = plane_copy(ctx)) != SPH_OK) return r;
    }
    const uint32_t gyz = (uint32_t)ctx->grid.gy * (uint32_t)ctx->grid.gz;
    hipStream_t s1 = ctx->stream, s2 = ctx->stream2;
    auto range = [&](int k) {
        return DevRange{ctx->cs + (size_t)ctx->chunk_cx[(size_t)k] * gyz, ctx->cs + (size_t)ctx->chunk_cx[(size_t)k + 1] * gyz};
    };
    auto est = [&](int k) {   // grid size: the count seen a few steps ago, +1/16 (tiles past it loop)
        const int32_t e = ctx->chunk_est[(size_t)k];
        return std::max<int32_t>(e + e / 16 + 256, 1);
    };
    const HitMask hw = hit_mask_write(ctx);
    for (int k = 0; k < S; ++k) {
        {
            KTimer t(ctx, "density", 24.0 * est(k), true);
            launch_density_tiled(ctx->pos, ctx->cs, 0, est(k), ctx->grid, ctx->sc, ctx->rp, hw, path_ctr(ctx), s1,
                                 range(k));
        }
        HIPCHK(hipEventRecord(ctx->ev_chunk[k], s1));
    }
    const MoverSink mv = mover_sink(ctx);
    const HitMask hr = hit_mask_read(ctx);
    const float fext = forcing(ctx);
    for (int k = 0; k < S; ++k) {
        HIPCHK(hipStreamWaitEvent(s2, ctx->ev_chunk[std::min(k + 1, S - 1)], 0));
        KTimer t(ctx, "force_integrate", 76.0 * est(k), true);
        launch_force_tiled(ctx->pos, ctx->vel, ctx->rp, ctx->cs, 0, est(k), ctx->grid, ctx->sc, dt, fext, ctx->pos2,
                           ctx->vel2, ctx->keys, mv, hr, path_ctr(ctx), s2, range(k));
    }
    HIPCHK(hipEventRecord(ctx->ev_chunk[SPH_MAX_CHUNKS], s2));
    HIPCHK(hipStreamWaitEvent(s1, ctx->ev_chunk[SPH_MAX_CHUNKS], 0));   // the step ends on the context stream
    HIPCHK(hipGetLastError());
    if (mv.sk && (ctx->steps & 7) == 0)
        HIPCHK(hipMemcpyAsync(ctx->mv_host, mv.count, sizeof(uint32_t), hipMemcpyDeviceToHost, s1));
    swap_sv(ctx);
    ctx->keys_valid = true;
    ctx->keys_active = 0;
    return SPH_OK;
}

int step_wcsph(sph_ctx* ctx, float dt) {
    const int32_t n = ctx->n;
    int r = sort_wcsph(ctx);
    if (r != SPH_OK) return r;
    // chunked passes from C2's size up (smaller steps are launch-bound: more launches cost more)
    const int S = std::min(ctx->chunks, ctx->grid.gx);
    if (S > 1 && n >= CHUNK_MIN_PARTICLES) return step_wcsph_chunked(ctx, dt, S);
    {
        KTimer t(ctx, "density", 24.0 * n, true);
        density_range(ctx, 0, n);
    }
    const MoverSink mv = mover_sink(ctx);
    {
        KTimer t(ctx, "force_integrate", 76.0 * n, true);
        force_range(ctx, 0, n, dt, forcing(ctx), mv);
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

}  // namespace sph
