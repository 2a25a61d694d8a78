// abi.cpp — the single-domain C ABI of libsphhip.so (include/sphhip.h); the step itself is in
// host_step.cpp, the slab decomposition in abi_slab.cpp.
#include "host.h"

using namespace sph;

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
    if (cfg->capacity < 0 || cfg->ndev < 0) return SPH_ERR_INVALID;
    const bool group = cfg->ndev > 1;
    if (group && cfg->model != SPH_MODEL_WCSPH) return SPH_ERR_INVALID;   // the decomposed step is Model S
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SPH_ERR_HIP;
    if (device < 0 || device >= ndev) return SPH_ERR_INVALID;
    sph_ctx* ctx = new sph_ctx();
    ctx->cfg = *cfg;
    ctx->device = device;
    ctx->profiling = (cfg->flags & SPH_FLAG_PROFILE) != 0;
    if (const char* v = std::getenv("SPH_RESORT")) ctx->resort_mode = std::atoi(v);
    if (const char* v = std::getenv("SPH_CT_TEAM")) ctx->ct_team = std::atoi(v);
    if (const char* v = std::getenv("SPH_SMALL")) ctx->small_mode = std::atoi(v);
    if (const char* v = std::getenv("SPH_FUSED")) ctx->fused_mode = std::atoi(v);
    if (const char* v = std::getenv("SPH_SCHED")) ctx->sched_mode = std::atoi(v);   // default off
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&ctx->mv_host, sizeof(uint32_t), hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)&ctx->mv_host_dev, ctx->mv_host, 0) != hipSuccess) {
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
        delete ctx;
        return SPH_ERR_HIP;
    }
    *ctx->mv_host = 0u;
    ctx->own_stream = true;
    ctx->capacity = group ? 0 : cfg->capacity;   // a group's slots live in its per-GPU slab contexts
    int r = alloc_particles(ctx, ctx->capacity);
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
    if (group && (r = multi_create_group(ctx)) != SPH_OK) { sph_destroy(ctx); return r; }
    *out = ctx;
    return SPH_OK;
}

// the entry points that address one GPU's slot arrays directly have no meaning on a group
#define NOT_GROUP(ctx) \
    if (is_group(ctx)) return fail(ctx, SPH_ERR_STATE, "%s: not available on a multi-GPU (ndev > 1) context", __func__)

void sph_destroy(sph_ctx* ctx) {
    if (!ctx) return;
    multi_free(ctx);
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
    NOT_GROUP(ctx);
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
    if (int r = multi_params_changing(ctx, *params)) return r;
    if (is_group(ctx)) {   // kept for the slab contexts (made at sph_init_scenario), applied to existing ones
        if (!(params->h > 0.f) || !(params->dx > 0.f) || !(params->rho0 > 0.f))
            return fail(ctx, SPH_ERR_INVALID, "Model S needs dx, h, rho0 > 0");
        ctx->prm = *params;
        ctx->params_set = true;
        for (sph_ctx* k : multi_kids(ctx))
            if (int r = sph_set_params(k, params)) return fail(ctx, r, "%s", sph_last_error(k));
        return SPH_OK;
    }
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
    NOT_GROUP(ctx);
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
    invalidate_sort(ctx);
    ctx->steps = 0;
    ctx->sim_time = 0.0;
    return SPH_OK;
}

int sph_download_particles_aos84(sph_ctx* ctx, void* dst, int32_t count) {
    if (!ctx || (!dst && count > 0)) return SPH_ERR_INVALID;
    NOT_GROUP(ctx);
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
    NOT_GROUP(ctx);
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
    invalidate_sort(ctx);
    ctx->steps = 0;
    ctx->sim_time = 0.0;
    return SPH_OK;
}

int sph_init_scenario(sph_ctx* ctx, const sph_scenario* sc) {
    if (!ctx || !sc) return SPH_ERR_INVALID;
    if (ctx->mg) {   // multi-GPU: this process's slabs of the scenario
        HIPCHK(hipSetDevice(ctx->device));
        return is_group(ctx) ? multi_init_scenario(ctx, sc) : multi_init_rank(ctx, sc);
    }
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
    invalidate_sort(ctx);
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
    invalidate_sort(ctx);
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
    invalidate_sort(ctx);
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
    invalidate_sort(ctx);
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
    invalidate_sort(ctx);
    return SPH_OK;
}

int sph_step(sph_ctx* ctx, float dt, int32_t nsteps) {
    if (!ctx || nsteps < 0 || !(dt >= 0.f)) return SPH_ERR_INVALID;
    if (ctx->mg) return multi_step(ctx, dt, nsteps);
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

int sph_set_sim_time(sph_ctx* ctx, double t) {
    if (!ctx || !(t >= 0.0)) return SPH_ERR_INVALID;
    if (is_group(ctx)) return fail(ctx, SPH_ERR_STATE, "sph_set_sim_time: one-GPU contexts and RCCL ranks only");
    ctx->sim_time = t;
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
    if (ctx && is_group(ctx)) return (!xyz && count > 0) ? SPH_ERR_INVALID : multi_read(ctx, 0, xyz, count);
    return ctx ? read_f4(ctx, ctx->pos, xyz, count, 3) : SPH_ERR_INVALID;
}
int sph_read_velocities(sph_ctx* ctx, float* xyz, int32_t count) {
    if (ctx && is_group(ctx)) return (!xyz && count > 0) ? SPH_ERR_INVALID : multi_read(ctx, 1, xyz, count);
    return ctx ? read_f4(ctx, ctx->vel, xyz, count, 3) : SPH_ERR_INVALID;
}
int sph_read_rotations(sph_ctx* ctx, float* xyzw, int32_t count) {
    return ctx ? read_f4(ctx, ctx->rot, xyzw, count, 4) : SPH_ERR_INVALID;
}
int sph_read_angular_velocities(sph_ctx* ctx, float* xyz, int32_t count) {
    return ctx ? read_f4(ctx, ctx->omg, xyz, count, 3) : SPH_ERR_INVALID;
}

static int read_rp(sph_ctx* ctx, float* dst, int32_t count, int32_t comp) {
    if (!ctx || (!dst && count > 0)) return SPH_ERR_INVALID;
    if (is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "density is Model S only");
    if (ctx->slab) return fail(ctx, SPH_ERR_STATE, "slab mode: use sph_slab_read_owned");
    if (count < ctx->n) return fail(ctx, SPH_ERR_INVALID, "count %d < active particles %d", count, ctx->n);
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->n > 0) {
        // rp is in the slot order of the last step's density pass; id was reordered before it
        launch_scatter_f2x_by_id(ctx->rp, ctx->id, ctx->n, (float*)ctx->staging, ctx->stream, comp);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(dst, ctx->staging, (size_t)ctx->n * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

int sph_read_density(sph_ctx* ctx, float* rho, int32_t count) {
    if (ctx && is_group(ctx)) return (!rho && count > 0) ? SPH_ERR_INVALID : multi_read(ctx, 2, rho, count);
    return read_rp(ctx, rho, count, 0);
}

int sph_read_pressure_term(sph_ctx* ctx, float* prho, int32_t count) {
    if (ctx && is_group(ctx)) return fail(ctx, SPH_ERR_STATE, "not available on a multi-GPU context");
    return read_rp(ctx, prho, count, 1);
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
    NOT_GROUP(ctx);
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
    NOT_GROUP(ctx);
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
    NOT_GROUP(ctx);
    HIPCHK(hipSetDevice(ctx->device));
    const int32_t inst = is_contact(ctx) ? contact_active(ctx) : ctx->n;
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)((uint32_t*)dev_args + 1), inst, 1, ctx->stream));
    return SPH_OK;
}

int sph_synchronize(sph_ctx* ctx) {
    if (!ctx) return SPH_ERR_INVALID;
    for (sph_ctx* k : multi_kids(ctx))
        if (int r = sph_synchronize(k)) return fail(ctx, r, "%s", sph_last_error(k));
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
    out->grid[0] = ctx->grid.gx * ctx->grid.xsub; out->grid[1] = ctx->grid.gy; out->grid[2] = ctx->grid.gz;
    out->key_bits = ctx->key_bits;
    out->device_bytes = ctx->device_bytes;
    const std::vector<sph_ctx*> kids = multi_kids(ctx);
    if (!kids.empty()) {   // a group: the global grid, every slab's slots and memory
        sph_decomp d;
        if (int r = sph_get_decomposition(ctx, &d)) return r;
        out->active = (int32_t)d.total;
        out->capacity = 0;
        out->device_bytes = 0;
        for (sph_ctx* k : kids) {
            out->capacity += k->capacity;
            out->device_bytes += k->device_bytes;
        }
        out->grid[0] = kids[0]->gglobal.gx * kids[0]->gglobal.xsub; out->grid[1] = kids[0]->gglobal.gy; out->grid[2] = kids[0]->gglobal.gz;
        out->key_bits = kids[0]->key_bits;
    }
    return SPH_OK;
}

// a group's kernel statistics: its slab contexts' merged by kernel name
static void merge_kid_stats(sph_ctx* ctx) {
    const std::vector<sph_ctx*> kids = multi_kids(ctx);
    if (kids.empty()) return;
    ctx->kstats.clear();
    for (sph_ctx* k : kids) {
        if (!k->pending.empty()) resolve_pending(k);
        for (const KStat& s : k->kstats) {
            const int i = kstat_index(ctx, s.name.c_str());
            ctx->kstats[i].launches += s.launches;
            ctx->kstats[i].total_ms += s.total_ms;
            ctx->kstats[i].timed += s.timed;
            ctx->kstats[i].bytes = s.bytes;
        }
    }
}

int sph_get_kernel_stat(sph_ctx* ctx, int32_t index, sph_kernel_stat* out) {
    if (!ctx || !out) return SPH_ERR_INVALID;
    if (!ctx->pending.empty()) resolve_pending(ctx);
    merge_kid_stats(ctx);
    if (index < 0 || index >= (int32_t)ctx->kstats.size()) return SPH_ERR_INVALID;
    const KStat& k = ctx->kstats[index];
    std::memset(out, 0, sizeof *out);
    std::snprintf(out->name, sizeof out->name, "%s", k.name.c_str());
    out->launches = k.launches;
    out->total_ms = k.total_ms;
    out->bytes_per_launch = k.bytes;
    out->timed = k.timed;
    return SPH_OK;
}

int sph_set_profile_every(sph_ctx* ctx, int32_t every) {
    if (!ctx || every < 1) return SPH_ERR_INVALID;
    ctx->prof_every = every;
    for (sph_ctx* k : multi_kids(ctx)) k->prof_every = every;
    return SPH_OK;
}

int sph_reset_kernel_stats(sph_ctx* ctx) {
    if (!ctx) return SPH_ERR_INVALID;
    for (sph_ctx* k : multi_kids(ctx)) sph_reset_kernel_stats(k);
    if (!ctx->pending.empty()) resolve_pending(ctx);
    for (auto& k : ctx->kstats) {
        k.launches = 0;
        k.timed = 0;
        k.total_ms = 0.0;
    }
    return SPH_OK;
}

int sph_read_sorted_ids(sph_ctx* ctx, int32_t* ids, int32_t count) {
    if (!ctx || (!ids && count > 0)) return SPH_ERR_INVALID;
    NOT_GROUP(ctx);
    if (count < ctx->n) return fail(ctx, SPH_ERR_INVALID, "count %d < active particles %d", count, ctx->n);
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->n > 0) HIPCHK(hipMemcpyAsync(ids, ctx->id, (size_t)ctx->n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

int sph_read_cell_start(sph_ctx* ctx, uint32_t* cs, int32_t count) {
    if (!ctx || (!cs && count > 0)) return SPH_ERR_INVALID;
    NOT_GROUP(ctx);
    if ((uint32_t)count < ctx->grid.ncells + 1)
        return fail(ctx, SPH_ERR_INVALID, "count %d < ncells+1 = %u", count, ctx->grid.ncells + 1);
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemcpyAsync(cs, ctx->cs, (size_t)(ctx->grid.ncells + 1) * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

}  // extern "C"

// counters [first, first + m) of ctx->paths (summed over a local group's slab contexts; word max_at, if any, by
// maximum). arm: from now on the neighbour passes count (the re-sort's counters always count)
static int read_paths(sph_ctx* ctx, int first, int m, uint32_t* counts, int32_t reset, bool arm = true,
                      int max_at = -1) {
    const std::vector<sph_ctx*> kids = sph::multi_kids(ctx);
    if (!kids.empty()) {
        for (int k = 0; k < m; ++k) counts[k] = 0;
        for (sph_ctx* kc : kids) {
            uint32_t c[8];
            if (int r = read_paths(kc, first, m, c, reset, arm, max_at)) return r;
            for (int k = 0; k < m; ++k) counts[k] = k == max_at ? std::max(counts[k], c[k]) : counts[k] + c[k];
        }
        return SPH_OK;
    }
    if (arm) ctx->count_paths = true;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemcpyAsync(counts, ctx->paths + first, m * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    if (reset) HIPCHK(hipMemsetAsync(ctx->paths + first, 0, m * sizeof(uint32_t), ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SPH_OK;
}

extern "C" {

int sph_read_path_counts(sph_ctx* ctx, uint32_t counts[4], int32_t reset) {
    if (!ctx || !counts) return SPH_ERR_INVALID;
    return read_paths(ctx, 0, 4, counts, reset);
}

int sph_read_resort_counts(sph_ctx* ctx, uint32_t counts[8], int32_t reset) {
    if (!ctx || !counts) return SPH_ERR_INVALID;
    return read_paths(ctx, 16, 8, counts, reset, false, 4);
}

int sph_read_mover_count(sph_ctx* ctx, uint32_t* movers) {
    if (!ctx || !movers) return SPH_ERR_INVALID;
    if (ctx->mg) return fail(ctx, SPH_ERR_STATE, "sph_read_mover_count: single contexts only");
    if (is_contact(ctx) || !ctx->mv_count) return fail(ctx, SPH_ERR_STATE, "sph_read_mover_count: Model S only");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    // the last force pass appended into the counter the next re-sort reads (mv_par)
    HIPCHK(hipMemcpy(movers, ctx->mv_count + ctx->mv_par, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return SPH_OK;
}

int sph_read_hit_mask_counts(sph_ctx* ctx, uint32_t counts[2], int32_t reset) {
    if (!ctx || !counts) return SPH_ERR_INVALID;
    return read_paths(ctx, 4, 2, counts, reset);
}

// Lane-utilisation counters of a -DSPH_DIAG build (zero otherwise): pass 1 candidates, 4-candidate
// iterations and tail iterations per wave (summed); pass 2 pairs, flush iterations, flushes, append
// iterations, mask pieces. Diagnostics only (scripts/pass_util.py); not part of include/sphhip.h.
int sph_debug_pass_counts(sph_ctx* ctx, uint32_t counts[8], int32_t reset) {
    if (!ctx || !counts) return SPH_ERR_INVALID;
    return read_paths(ctx, 8, 8, counts, reset);
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

int sph_debug_kick(sph_ctx* ctx, int32_t id, const float dv[3]) {
    if (!ctx || !dv) return SPH_ERR_INVALID;
    if (is_contact(ctx)) return fail(ctx, SPH_ERR_STATE, "sph_debug_kick is Model S only");
    {   // a slab step's early messages hold the velocities before the kick
        const int r = multi_state_changed(ctx);
        if (r != SPH_OK) return r;
    }
    std::vector<sph_ctx*> cs = is_group(ctx) ? multi_kids(ctx) : std::vector<sph_ctx*>{ctx};
    for (sph_ctx* k : cs) {   // every slot up to the capacity: ghosts and stale slots are overwritten before use
        HIPCHK(hipSetDevice(k->device));
        launch_kick(k->id, k->vel, k->capacity, id, dv, k->stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(k->stream));
    }
    return SPH_OK;
}

int sph_resize(sph_ctx* ctx, int32_t capacity) {
    if (!ctx || capacity < 0) return SPH_ERR_INVALID;
    NOT_GROUP(ctx);
    if (capacity < ctx->n) return fail(ctx, SPH_ERR_CAPACITY, "capacity %d < active particles %d", capacity, ctx->n);
    if (ctx->slab) return fail(ctx, SPH_ERR_STATE, "slab mode");
    HIPCHK(hipSetDevice(ctx->device));
    // keep the particles: device-to-device copies of the slot arrays (no host round trip)
    return grow_d2d(ctx, capacity);
}

}  // extern "C"
