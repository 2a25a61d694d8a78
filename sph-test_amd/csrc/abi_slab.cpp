// abi_slab.cpp — the slab decomposition of the Model S step (SPEC_SPH.md §3): the per-phase C ABI
// a host drives rank by rank (sph_slab_*).
#include "host.h"

using namespace sph;

// ---------------------------------------------------------------- slab decomposition
// Wait for the last assemble's range copy and publish rng / o0 / o1 (no-op when up to date).
int sph::slab_sync_ranges(sph_ctx* ctx) {
    if (ctx->dz_ahead) {   // after the in-library step's device-sized steps: one wait, then the device sizes
        ctx->dz_ahead = false;
        HIPCHK(hipSetDevice(ctx->device));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        SlabSizes h;
        HIPCHK(hipMemcpy(&h, ctx->dz, sizeof h, hipMemcpyDeviceToHost));
        if (h.flags)
            return fail(ctx, SPH_ERR_CAPACITY, "slab step:%s%s%s%s%s", (h.flags & SZ_OVF_MSG) ? " halo message overflow" : "",
                        (h.flags & SZ_OVF_CAP) ? " slots over capacity" : "",
                        (h.flags & SZ_RHO_MISMATCH) ? " ghost density count mismatch" : "",
                        (h.flags & SZ_OVF_MOVERS) ? " mover list / re-sort destination out of range" : "",
                        (h.flags & SZ_JUMP) ? " a particle left the held columns in one step" : "");
        for (int k = 0; k < 10; ++k) ctx->rng[k] = (int32_t)h.rg[k];
        ctx->o0 = (int32_t)h.o0;
        ctx->o1 = (int32_t)h.o1;
        // the slots of the last step's order; after the next step's record kernel ran (abi_multi.cpp issue_next_rec),
        // SlabSizes.n holds the next assembled layout's and rg[5] (k_slab_lag) this order's
        ctx->n = (int32_t)(ctx->dz_next ? h.rg[5] : h.n);
        ctx->dropped = (int32_t)h.dropped;
        ctx->rng_pending = false;
        return SPH_OK;
    }
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

int sph::slab_local_grid(sph_ctx* ctx) {
    const GridDesc& G = ctx->gglobal;
    GridDesc g = G;
    ctx->has_left = ctx->sl.cx_lo > 0;
    ctx->has_right = ctx->sl.cx_hi < G.gx;
    g.cx0 = ctx->sl.cx_lo - (ctx->has_left ? 1 : 0);
    g.gx = ctx->sl.cx_hi + (ctx->has_right ? 1 : 0) - g.cx0;
    g.gx_all = G.gx;
    g.ncells = (uint32_t)g.gx * col_keys(g);
    ctx->grid = g;
    ctx->key_bits = bit_width(g.ncells);
    invalidate_sort(ctx);
    return ensure_cells(ctx);
}

int32_t sph::col_start(const sph_ctx* c, int32_t local_col) {
    return local_col * (int32_t)col_keys(c->grid);
}

extern "C" {

int sph_slab_set(sph_ctx* ctx, const sph_slab* slab) {
    if (!ctx || !slab) return SPH_ERR_INVALID;
    if (is_group(ctx)) return fail(ctx, SPH_ERR_STATE, "a multi-GPU (ndev > 1) context cuts its own slabs");
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
    const uint32_t gyz = col_keys(ctx->grid);
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
    invalidate_sort(ctx);
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
    const uint32_t gyz = col_keys(ctx->grid);
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
    const uint32_t gyz = col_keys(ctx->grid);
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
    return slab_assemble(ctx, dev_left, nl, dev_right, nr, false);
}

}  // extern "C"

// The assemble with host-known record counts (the per-phase ABI above, and the in-library step's
// full-sort steps). force_full: take the full radix sort even when the incremental one is possible.
int sph::slab_assemble(sph_ctx* ctx, const void* dev_left, int32_t nl, const void* dev_right, int32_t nr,
                       bool force_full) {
    ctx->hm_valid = false;   // a new slot order
    const int32_t no = ctx->o1 - ctx->o0;
    const int64_t n = (int64_t)nl + no + nr;
    if (n > ctx->capacity) return fail(ctx, SPH_ERR_CAPACITY, "slab needs %lld slots > capacity %d", (long long)n, ctx->capacity);
    hipStream_t s = ctx->stream;
    const uint32_t gyz = col_keys(ctx->grid);
    const uint32_t key_base = (uint32_t)ctx->grid.cx0 * gyz;
    const bool many = ctx->resort_mode == 1 && *(volatile uint32_t*)ctx->mv_host > resort_limit((int32_t)n);
    // ranges from the cell table at column starts: picked on the device (density reads them there)
    // and written to mapped pinned memory; slab_sync_ranges waits for the event after the sort
    const int32_t lc_lo = ctx->sl.cx_lo - ctx->grid.cx0, lc_hi = ctx->sl.cx_hi - ctx->grid.cx0;
    const int32_t idx[8] = {col_start(ctx, 0), col_start(ctx, lc_lo), col_start(ctx, lc_lo + 1),
                            col_start(ctx, lc_hi - 1), col_start(ctx, lc_hi), col_start(ctx, ctx->grid.gx),
                            col_start(ctx, std::min(lc_lo + 2, lc_hi)), col_start(ctx, std::max(lc_hi - 2, lc_lo))};
    if (ctx->resort_mode != 0 && !many && !force_full && ctx->sk_valid && n > 0) {
        // incremental: the re-sort reads [left records | own slots | right records] in place. The force
        // pass already appended the own movers (window keys); the records' keys and movers join here.
        const AsmSrc src{ctx->pos, ctx->vel, ctx->id, ctx->sk_cur, ctx->keys, ctx->o0 - nl, (const float4*)dev_left,
                         (const float4*)dev_right, ctx->keys2, ctx->vals, nl, nl + no};
        const int used = ctx->mv_par;
        const MoverSink mv{ctx->keys2, ctx->mv_count + used, ctx->mv_mi, ctx->mv_mk, ctx->mv_mo,
                           (uint32_t)std::max(ctx->capacity, 1)};
        {
            KTimer t(ctx, "slab_assemble", 40.0 * (double)(nl + nr));
            launch_slab_rec(src, (int32_t)n, ctx->grid, key_base, ctx->vals, ctx->keys2, mv, s);
        }
        KTimer t(ctx, "resort", (double)n * (2 * 4 + 2 * 36));
        launch_slab_cs_old(ctx->cs, ctx->grid.ncells, gyz, (uint32_t)ctx->grid.gx, ctx->has_left, ctx->has_right,
                           nl - ctx->o0, ctx->keys2, nl, no, nr, s);
        CsPick pick{{0}, 8, ctx->sdev, ctx->rng_host};   // the ranges, read as the cell table completes
        for (int k = 0; k < 8; ++k) pick.idx[k] = idx[k];
        ResortScratch w = resort_scratch(ctx);
        w.mi_off = nl - ctx->o0;   // own movers were appended by slot in the previous order
        launch_resort(src, ctx->cs, ctx->cs2, ctx->grid.ncells, (int32_t)n, ctx->mv_count + used,
                      ctx->mv_count + (1 - used), w, ctx->pos2, ctx->vel2, ctx->id2, ctx->sk_next, s, pick);
        swap_cs(ctx);
        ctx->mv_par = 1 - used;   // (k_mv_rank stored the mover count for the host)
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
        // taken for a large mover count: the host's next choice needs the count the last force pass appended
        // (k_mv_rank, which otherwise stores it, did not run), or the context would stay on this path for good
        if (many) HIPCHK(hipMemcpyAsync(ctx->mv_host, ctx->mv_count + ctx->mv_par, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemsetAsync(ctx->mv_count, 0, 2 * sizeof(uint32_t), s));
        launch_pick(ctx->cs, idx, 8, ctx->sdev, s, ctx->rng_host);
    }
    HIPCHK(hipEventRecord(ctx->rng_ev, s));
    ctx->rng_pending = true;
    ctx->n = (int32_t)n;
    ctx->keys_valid = false;
    ctx->sk_valid = ctx->resort_mode != 0;
    return SPH_OK;
}

extern "C" {

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
        launch_density_tiled(ctx->pos, ctx->cs, 0, ctx->n, ctx->grid, ctx->sc, ctx->rp, hit_mask_write(ctx), path_ctr(ctx), ctx->stream, dr);
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
    KTimer t(ctx, "force_integrate", 76.0 * (e - b));
    force_range(ctx, b, e, dt, forcing(ctx), mover_sink(ctx));   // own movers for the next assemble's re-sort
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
