// host_step.cpp — the per-step launch sequences of both models (see host.h).
#include "host.h"

namespace sph {

void swap_sv(sph_ctx* c) {
    std::swap(c->pos, c->pos2);
    std::swap(c->vel, c->vel2);
}

// the incremental re-sort wrote the new cell-start table into cs2
void swap_cs(sph_ctx* c) {
    std::swap(c->cs, c->cs2);
    std::swap(c->cs_cap, c->cs2_cap);
}

int sort_and_reorder(sph_ctx* ctx, int32_t n_active_id, const uint32_t** sorted_keys) {
    const int32_t n = ctx->n;
    if (!ctx->keys_valid || ctx->keys_active != n_active_id) {
        KTimer t(ctx, "keys", 20.0 * n);
        // Model R: the radius bound of the contact pass's cell skipping, recomputed with the keys after any change
        uint32_t* rmax = is_contact(ctx) ? ctx->sdev + SDEV_RMAX : nullptr;
        if (rmax) HIPCHK(hipMemsetAsync(rmax, 0, sizeof(uint32_t), ctx->stream));
        launch_keys(ctx->pos, n, is_contact(ctx) ? ctx->id : nullptr, n_active_id, ctx->grid, ctx->keys,
                    ctx->stream, false, rmax);
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

void density_range(sph_ctx* ctx, int32_t b, int32_t e, Sched sch) {
    launch_density_tiled(ctx->pos, ctx->cs, b, e, ctx->grid, ctx->sc, ctx->rp, hit_mask_write(ctx), path_ctr(ctx), ctx->stream,
                         DevRange{}, RhoOut{}, sch);
}

void force_range(sph_ctx* ctx, int32_t b, int32_t e, float dt, float fext, MoverSink mv, Sched sch) {
    launch_force_tiled(ctx->pos, ctx->vel, ctx->rp, ctx->cs, b, e, ctx->grid, ctx->sc, dt, fext, ctx->pos2, ctx->vel2,
                       ctx->keys, mv, hit_mask_read(ctx), path_ctr(ctx), ctx->stream, DevRange{}, DevRange{}, 0, SendBins{},
                       sch);
}

// The single context's y-band schedule for the tiled passes of this step (schedule.hip), or none.
constexpr int64_t SCHED_EVERY = 8;
Sched step_schedule(sph_ctx* ctx) {
    const int32_t n = ctx->n;
    if (ctx->sched_mode == 0 || n <= 0 || !schedule_fits(ctx->grid)) return Sched{};
    const int32_t ent = schedule_entries(n, ctx->grid);
    if (ent + 1 > ctx->sched_cap) {
        if (dalloc(ctx, &ctx->sched, (size_t)ent + 1) != SPH_OK) return Sched{};
        ctx->sched_cap = ent + 1;
        ctx->sched_valid = false;
    }
    if (!ctx->sched_valid || ctx->sched_n != n || ctx->sched_ent != ent || ctx->steps % SCHED_EVERY == 0) {
        KTimer t(ctx, "schedule", 4.0 * ctx->grid.gx * ctx->grid.xsub * ctx->grid.gy + 8.0 * ent, true);
        launch_schedule(ctx->cs, ctx->grid, n, ctx->sched, ent, ctx->stream);
        ctx->sched_valid = true;
        ctx->sched_n = n;
        ctx->sched_ent = ent;
    }
    return Sched{ctx->sched, ent};
}

// f_ext(t) of SPEC_SPH.md §2 at the context's simulated time (sloshing; 0 otherwise)
float forcing(const sph_ctx* ctx) {
    const sph_params& p = ctx->prm;
    const float tt = (float)ctx->sim_time;
    return p.forcing_amp != 0.0f ? p.forcing_amp * sinf(6.28318530718f * p.forcing_freq * tt) : 0.0f;
}

ResortScratch resort_scratch(sph_ctx* ctx) {
    ResortScratch w{ctx->mv_mi, ctx->mv_mk, ctx->mv_mo, ctx->mv_ms, ctx->mv_mx, ctx->mv_mos,
                    (uint32_t)std::max(ctx->capacity, 1), 0};
    w.host_count = ctx->mv_host_dev;
    w.stats = ctx->paths + 16;
    return w;
}

// The force pass appends movers for the next step's incremental re-sort.
MoverSink mover_sink(sph_ctx* ctx) {
    if (ctx->resort_mode == 0 || !ctx->sk_valid) return MoverSink{};
    return MoverSink{ctx->sk_cur, ctx->mv_count + ctx->mv_par, ctx->mv_mi, ctx->mv_mk, ctx->mv_mo,
                     (uint32_t)std::max(ctx->capacity, 1)};
}

// Bring the slots into stable (key, index) order: the incremental re-sort when the previous
// step's sorted keys and cell starts describe the current slot order, else the full radix sort.
// Movers above which the full radix sort is taken instead of the incremental re-sort. k_mv_rank's work is O(m) per
// workgroup plus its slots (every workgroup streams the mover list), so the full sort (three 8-bit passes, a gather
// and the cell starts over n) pays only when a large share moves; capped so that a range's entries stay within LDS.
uint32_t resort_limit(int32_t n) {
    return std::max<uint32_t>(4096u, std::min<uint32_t>((uint32_t)std::max(n, 0) / 16u, 262144u));
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
            launch_resort(asm_plain(ctx->pos, ctx->vel, ctx->id, ctx->sk_cur, ctx->keys, n), ctx->cs, ctx->cs2,
                          ctx->grid.ncells, n, ctx->mv_count + used, ctx->mv_count + (1 - used), resort_scratch(ctx),
                          ctx->pos2, ctx->vel2, ctx->id2, ctx->sk_next, ctx->stream);
            ctx->mv_par = 1 - used;
        }
        swap_cs(ctx);
        ctx->sorted_full = false;
        swap_sv(ctx);
        std::swap(ctx->id, ctx->id2);
        std::swap(ctx->sk_cur, ctx->sk_next);
        return SPH_OK;
    }
    ctx->sorted_full = true;
    const uint32_t* sk = nullptr;
    int r = sort_and_reorder(ctx, 0, &sk);
    if (r != SPH_OK) return r;
    if (n > 0) HIPCHK(hipMemcpyAsync(ctx->sk_cur, sk, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->mv_count, 0, 2 * sizeof(uint32_t), ctx->stream));
    ctx->sk_valid = true;
    return SPH_OK;
}

// Model S's two-launch step at the reference's scale: re-sort + pass 1 in one launch (wcsph_tiled.hip
// k_density_fused), then pass 2 on the sorted arrays it wrote; while the incremental re-sort's state holds.
bool fused_s_ok(const sph_ctx* ctx) {
    const int32_t n = ctx->n;
    return ctx->fused_mode != 0 && n > 0 && n <= density_fused_max() && (ctx->small_mode == 2 || (ctx->small_mode == 1 && n <= SMALL_N)) &&
           ctx->resort_mode != 0 && ctx->keys_valid && ctx->keys_active == 0 && ctx->sk_valid;
}

int step_wcsph_fused(sph_ctx* ctx, float dt) {
    const int32_t n = ctx->n;
    const int cur = ctx->mv_par, nxt = 1 - cur;
    ctx->hm_valid = false;
    const FusedIOS io{ctx->pos, ctx->vel, ctx->id, ctx->sk_cur, ctx->cs, ctx->mv_mi, ctx->mv_mk, ctx->mv_count + cur,
                      ctx->pos2, ctx->vel2, ctx->id2, ctx->sk_next, ctx->cs2, ctx->rp, ctx->mv_count + nxt,
                      ctx->mv_host_dev};
    {
        KTimer t(ctx, "density_fused", (double)n * (2 * 36 + 24), true);
        launch_density_fused(io, n, ctx->grid, ctx->sc, ctx->stream);
    }
    swap_cs(ctx);
    std::swap(ctx->id, ctx->id2);
    std::swap(ctx->sk_cur, ctx->sk_next);
    ctx->mv_par = nxt;
    ctx->sorted_full = false;
    // the sorted arrays are pos2 / vel2 now; pass 2 integrates them back into pos / vel
    const MoverSink mv = mover_sink(ctx);
    {
        KTimer t(ctx, "force_integrate", 56.0 * n, true);
        launch_force_small(ctx->pos2, ctx->vel2, ctx->rp, ctx->cs, n, ctx->grid, ctx->sc, dt, forcing(ctx), ctx->pos,
                           ctx->vel, ctx->keys, mv, ctx->stream);
    }
    ctx->keys_valid = true;
    ctx->keys_active = 0;
    return SPH_OK;
}

int step_wcsph(sph_ctx* ctx, float dt) {
    const int32_t n = ctx->n;
    if (fused_s_ok(ctx)) return step_wcsph_fused(ctx, dt);
    int r = sort_wcsph(ctx);
    if (r != SPH_OK) return r;
    const MoverSink mv = mover_sink(ctx);
    // the reference's scale: one wave per target (bit-identical to the tiled passes, wcsph_tiled.hip small N)
    const bool small = ctx->small_mode == 2 || (ctx->small_mode == 1 && n <= SMALL_N);
    if (small) {
        {
            KTimer t(ctx, "density", 24.0 * n, true);
            launch_density_small(ctx->pos, ctx->cs, n, ctx->grid, ctx->sc, ctx->rp, ctx->stream);
        }
        KTimer t(ctx, "force_integrate", 56.0 * n, true);
        launch_force_small(ctx->pos, ctx->vel, ctx->rp, ctx->cs, n, ctx->grid, ctx->sc, dt, forcing(ctx), ctx->pos2,
                           ctx->vel2, ctx->keys, mv, ctx->stream);
    } else {
        const Sched sch = step_schedule(ctx);
        {
            KTimer t(ctx, "density", 24.0 * n, true);
            density_range(ctx, 0, n, sch);
        }
        KTimer t(ctx, "force_integrate", 76.0 * n, true);
        force_range(ctx, 0, n, dt, forcing(ctx), mv, sch);
    }
    // the mover count for the next steps' sort choice (no host wait): the next incremental re-sort's k_mv_rank stores
    // it; after a full sort (no k_mv_rank) it is copied back every 8th step (a ~4 us blit; the count drifts slowly)
    if (mv.sk && ctx->sorted_full && (ctx->steps & 7) == 0)
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
        const int used = ctx->mv_par, next = (used + 1) % 3;   // Model R cycles three counters (the one-launch step)
        const ResortExtra ex{ctx->omg, ctx->rot, ctx->aux, ctx->mode, ctx->omg2, ctx->rot2, ctx->aux2, ctx->mode2};
        launch_resort(asm_plain(ctx->pos, ctx->vel, ctx->id, ctx->sk_cur, ctx->keys, n), ctx->cs, ctx->cs2, ctx->grid.ncells, n,
                      ctx->mv_count + used, ctx->mv_count + next, resort_scratch(ctx), ctx->pos2, ctx->vel2,
                      ctx->id2, ctx->sk_next, ctx->stream, CsPick{{0}, 0, nullptr, nullptr}, ex);
        ctx->mv_par = next;
        ctx->fz_ready = false;
        swap_cs(ctx);
        ctx->sorted_full = false;
        swap_sv(ctx);
        std::swap(ctx->id, ctx->id2);
        std::swap(ctx->omg, ctx->omg2);
        std::swap(ctx->rot, ctx->rot2);
        std::swap(ctx->aux, ctx->aux2);
        std::swap(ctx->mode, ctx->mode2);
        std::swap(ctx->sk_cur, ctx->sk_next);
        return SPH_OK;
    }
    ctx->sorted_full = true;
    const uint32_t* sk = nullptr;
    int r = sort_and_reorder(ctx, act, &sk);
    if (r != SPH_OK) return r;
    if (ctx->resort_mode != 0 && n > 0) {
        HIPCHK(hipMemcpyAsync(ctx->sk_cur, sk, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream));
        HIPCHK(hipMemsetAsync(ctx->mv_count, 0, 3 * sizeof(uint32_t), ctx->stream));
    }
    ctx->fz_ready = false;
    ctx->sk_valid = ctx->resort_mode != 0;
    return SPH_OK;
}

ContactConst contact_const(const sph_ctx* ctx, float dt) {
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
    c.rmax = ctx->sdev + SDEV_RMAX;
    return c;
}

// The one-launch step (contact.hip k_contact_fused) while the previous step's order, movers and cell starts hold:
// at the reference's scale, no bonds. Same results as sort_contact + the contact pass.
bool fused_step_ok(const sph_ctx* ctx, int32_t act) {
    return ctx->fused_mode != 0 && ctx->n > 0 && ctx->n <= contact_fused_max() && ctx->nbonds == 0 &&
           ctx->resort_mode != 0 && ctx->keys_valid && ctx->keys_active == act && ctx->sk_valid;
}

int step_contact_fused(sph_ctx* ctx, float dt, int32_t act) {
    const int32_t n = ctx->n;
    const int cur = ctx->mv_par, nxt = (cur + 1) % 3, zro = (cur + 2) % 3;
    if (!ctx->fz_ready) HIPCHK(hipMemsetAsync(ctx->mv_count + nxt, 0, sizeof(uint32_t), ctx->stream));
    const FusedIO io{ctx->pos, ctx->vel, ctx->omg, ctx->rot, ctx->aux, ctx->id, ctx->mode, ctx->sk_cur, ctx->cs,
                     ctx->mv_mi, ctx->mv_mk, ctx->mv_count + cur,
                     ctx->pos2, ctx->vel2, ctx->omg2, ctx->rot2, ctx->aux2, ctx->id2, ctx->mode2, ctx->torque,
                     ctx->sk_next, ctx->keys2, ctx->cs2,
                     ctx->mv_mi2, ctx->mv_mk2, ctx->mv_mo2, ctx->mv_count + nxt, ctx->mv_count + zro, ctx->mv_host_dev,
                     (uint32_t)std::max(ctx->capacity, 1)};
    {
        KTimer t(ctx, "contact_fused", (double)n * (2 * 88 + 2 * 64 + 4 + 12 + 4), true);
        launch_contact_fused(io, act, n, ctx->grid, contact_const(ctx, dt), ctx->stream);
    }
    swap_sv(ctx);
    std::swap(ctx->omg, ctx->omg2);
    std::swap(ctx->rot, ctx->rot2);
    std::swap(ctx->aux, ctx->aux2);
    std::swap(ctx->id, ctx->id2);
    std::swap(ctx->mode, ctx->mode2);
    std::swap(ctx->sk_cur, ctx->sk_next);
    std::swap(ctx->keys, ctx->keys2);
    swap_cs(ctx);
    std::swap(ctx->mv_mi, ctx->mv_mi2);
    std::swap(ctx->mv_mk, ctx->mv_mk2);
    std::swap(ctx->mv_mo, ctx->mv_mo2);
    ctx->mv_par = nxt;
    ctx->fz_ready = true;
    ctx->sorted_full = false;
    ctx->keys_valid = true;
    ctx->keys_active = act;
    return SPH_OK;
}

int step_contact(sph_ctx* ctx, float dt) {
    const int32_t n = ctx->n;
    const int32_t act = contact_active(ctx);
    if (fused_step_ok(ctx, act)) return step_contact_fused(ctx, dt, act);
    int r = sort_contact(ctx, act);
    if (r != SPH_OK) return r;
    const MoverSink mv = mover_sink(ctx);
    const ContactConst c = contact_const(ctx, dt);   // the one-launch step's constants, field for field
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
    if (mv.sk && ctx->sorted_full && (ctx->steps & 7) == 0)   // the mover count after a full sort (as step_wcsph)
        HIPCHK(hipMemcpyAsync(ctx->mv_host, mv.count, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    swap_sv(ctx);
    std::swap(ctx->omg, ctx->omg2);
    std::swap(ctx->rot, ctx->rot2);
    ctx->keys_valid = true;
    ctx->keys_active = act;
    return SPH_OK;
}

}  // namespace sph
