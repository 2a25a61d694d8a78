/* sph_oracle.c — CPU restatement of the grid + Model S step (TEST INFRASTRUCTURE ONLY).
 *
 * Grid/sort/cell-start: SPEC_SPH.md §0. GetGridCoord/GridHash of the reference:
 * /root/reference/Assets/Compute/SimulateParticles.compute:102-109 (clamp semantics kept,
 * linearisation x-slowest). Model S: SPEC_SPH.md §2 (build-defined; no reference source).
 * Compiled with -ffp-contract=off so every rounding is the one written here.
 * PARITY UNPINNED by reference fixtures (see oracle.h).
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* x sub-columns per column when SPH_XSUB is unset: the library's SPH_XSUB_DEFAULT (host.h) */
#define OR_XSUB_DEFAULT 1

static inline int32_t or_coord(float x, float origin, float inv_cell, int32_t G) {
    /* compute:103-104 — (uint)((p + R)/cell) with ftou (neg/NaN -> 0), clamp to [0,G-1] */
    float g = (x - origin) * inv_cell;
    if (!(g > 0.0f)) return 0;
    if (g >= (float)(G - 1)) return G - 1;
    return (int32_t)g;
}

/* x counts sub-columns: xsub per column of G[0] (SPEC_SPH.md §0; xsub = 1 is the plain 2h grid) */
uint32_t or_cell_key(const or_grid* g, float x, float y, float z) {
    int32_t cx = or_coord(x, g->origin[0], g->inv_cxs, g->G[0] * g->xsub);
    int32_t cy = or_coord(y, g->origin[1], g->inv_cell, g->G[1]);
    int32_t cz = or_coord(z, g->origin[2], g->inv_cell_z, g->G[2]);
    return ((uint32_t)cx * (uint32_t)g->G[1] + (uint32_t)cy) * (uint32_t)g->G[2] + (uint32_t)cz;
}

void or_keys(const or_grid* g, int n, const float* pos3, uint32_t* keys) {
    for (int i = 0; i < n; ++i) keys[i] = or_cell_key(g, pos3[3 * i], pos3[3 * i + 1], pos3[3 * i + 2]);
}

void or_stable_sort(int n, const uint32_t* keys, uint32_t nkeys, uint32_t* perm) {
    uint32_t* cnt = (uint32_t*)calloc((size_t)nkeys + 1, sizeof(uint32_t));
    for (int i = 0; i < n; ++i) cnt[keys[i] + 1]++;
    for (uint32_t k = 0; k < nkeys; ++k) cnt[k + 1] += cnt[k];
    for (int i = 0; i < n; ++i) perm[cnt[keys[i]]++] = (uint32_t)i;
    free(cnt);
}

void or_cell_start(int n, const uint32_t* sk, uint32_t nkeys, uint32_t* cs) {
    int i = 0;
    for (uint32_t k = 0; k <= nkeys; ++k) {
        while (i < n && sk[i] < k) ++i;
        cs[k] = (uint32_t)i;
    }
}

/* ------------------------------------------------------------------ Model S */

void or_sph_derive(or_sph_params* p) {
    const float PI = 3.14159265358979f;
    float d = p->dx;
    p->mass = p->rho0 * d * d * (p->dim == 3 ? d : 1.0f);
    p->B = p->c0 * p->c0 * p->rho0 / 7.0f;
    p->sigma = p->dim == 3 ? 1.0f / (PI * p->h * p->h * p->h) : 10.0f / (7.0f * PI * p->h * p->h);
    p->inv_h = 1.0f / p->h;
    p->four_h2 = 4.0f * p->h * p->h;
    /* SPEC_SPH.md §0: cells 2h in x, y; z split into zsub = 6 sub-cells (3D) */
    float cell = 2.0f * p->h;
    int32_t zsub = p->dim == 3 ? 6 : 1;
    float cz = cell / (float)zsub;
    p->grid.inv_cell = 1.0f / cell;
    p->grid.inv_cell_z = 1.0f / cz;
    p->grid.zwin = zsub + 1;
    /* x sub-columns: SPH_XSUB (1 or 2) as the library reads it (sph-test_amd/csrc/host.h) */
    int32_t xsub = OR_XSUB_DEFAULT;
    const char* xe = getenv("SPH_XSUB");
    if (xe && (atoi(xe) == 1 || atoi(xe) == 2)) xsub = atoi(xe);
    p->grid.xsub = p->dim == 3 ? xsub : 1;
    p->grid.inv_cxs = p->grid.inv_cell * (float)p->grid.xsub;
    for (int a = 0; a < 3; ++a) {
        p->grid.origin[a] = 0.0f;
        int32_t G = (int32_t)floorf(p->L[a] / (a == 2 ? cz : cell)) + 1;
        if (a == 2 && p->dim == 2) G = 1;
        p->grid.G[a] = G < 1 ? 1 : G;
    }
}

static inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

static inline float lattice_jitter(uint32_t seed, uint32_t id, uint32_t axis, float jitter) {
    uint32_t u = mix32(mix32(seed) ^ (3u * id + axis));
    float r = (float)(u >> 8) * (1.0f / 16777216.0f);
    return (2.0f * r - 1.0f) * jitter;
}

void or_sph_lattice(int dim, int nx, int ny, int nz, float dx, float x0, float y0, float z0,
                    uint32_t seed, float jitter, float* pos3) {
    if (dim == 2) nz = 1;
    for (int iz = 0; iz < nz; ++iz)
        for (int iy = 0; iy < ny; ++iy)
            for (int ix = 0; ix < nx; ++ix) {
                uint32_t id = (uint32_t)ix + (uint32_t)nx * ((uint32_t)iy + (uint32_t)ny * (uint32_t)iz);
                float* q = pos3 + 3 * (size_t)id;
                q[0] = fmaf((float)ix + 0.5f, dx, x0) + lattice_jitter(seed, id, 0, jitter);
                q[1] = fmaf((float)iy + 0.5f, dx, y0) + lattice_jitter(seed, id, 1, jitter);
                q[2] = dim == 3 ? fmaf((float)iz + 0.5f, dx, z0) + lattice_jitter(seed, id, 2, jitter) : 0.0f;
            }
}

/* cubic spline (Monaghan & Lattanzio 1985), SPEC_SPH.md §2 */
static inline void kernel_wf(const or_sph_params* p, float r2, float* W, float* F) {
    float r = sqrtf(r2);
    float q = r * p->inv_h;
    if (q < 1.0f) {
        *W = p->sigma * (1.0f + q * q * (-1.5f + 0.75f * q));
        *F = p->sigma * p->inv_h * p->inv_h * (-3.0f + 2.25f * q);
    } else {
        float t = 2.0f - q;
        *W = p->sigma * 0.25f * t * t * t;
        *F = -p->sigma * p->inv_h * 0.75f * t * t / r;
    }
}

typedef struct { int n; int lo, hi; } row_range;

/* the (2 xsub + 1) x 3 contiguous neighbour rows of SPEC_SPH.md §0 (9 for xsub = 1), in visit order:
 * sub-column offset outer, y offset inner, each over the z sub-cell window [cz - zwin, cz + zwin]
 * (a superset of every row's trimmed window) */
#define OR_MAX_ROWS 15
static int neighbour_rows(const or_grid* g, const uint32_t* cs, uint32_t key, uint32_t ranges[OR_MAX_ROWS][2]) {
    int32_t GY = g->G[1], GZ = g->G[2];
    int32_t cz = (int32_t)(key % (uint32_t)GZ);
    int32_t cy = (int32_t)((key / (uint32_t)GZ) % (uint32_t)GY);
    int32_t cx = (int32_t)(key / ((uint32_t)GZ * (uint32_t)GY));
    int32_t z0 = cz - g->zwin, z1 = cz + g->zwin;
    if (z0 < 0) z0 = 0;
    if (z1 > GZ - 1) z1 = GZ - 1;
    int nr = 0;
    for (int ddx = -g->xsub; ddx <= g->xsub; ++ddx) {
        int32_t x = cx + ddx;
        if (x < 0 || x >= g->G[0] * g->xsub) continue;
        for (int ddy = -1; ddy <= 1; ++ddy) {
            int32_t y = cy + ddy;
            if (y < 0 || y >= GY) continue;
            uint32_t rowk = ((uint32_t)x * (uint32_t)GY + (uint32_t)y) * (uint32_t)GZ;
            ranges[nr][0] = cs[rowk + (uint32_t)z0];
            ranges[nr][1] = cs[rowk + (uint32_t)z1 + 1];
            ++nr;
        }
    }
    return nr;
}

/* pass 1 over sorted targets [i0, i1): density + Tait EOS (SPEC_SPH.md §2) */
void or_sph_density_range(const or_sph_params* p, const float* p2, const uint32_t* sk, const uint32_t* cs,
                          int i0, int i1, float* rho, float* prho, int nthreads) {
    const or_grid* g = &p->grid;
    const float m = p->mass, four_h2 = p->four_h2, inv_rho0 = 1.0f / p->rho0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1024)
    for (int i = i0; i < i1; ++i) {
        uint32_t rg[OR_MAX_ROWS][2];
        int nr = neighbour_rows(g, cs, sk[i], rg);
        float xi = p2[3 * i], yi = p2[3 * i + 1], zi = p2[3 * i + 2];
        float s = 0.0f;
        for (int r = 0; r < nr; ++r)
            for (uint32_t j = rg[r][0]; j < rg[r][1]; ++j) {
                float ddx = xi - p2[3 * j], ddy = yi - p2[3 * j + 1], ddz = zi - p2[3 * j + 2];
                float r2 = ddx * ddx + ddy * ddy + ddz * ddz;
                if (r2 < four_h2) {
                    float W, F;
                    kernel_wf(p, r2, &W, &F);
                    s += W;
                }
            }
        float d = m * s;
        float tr = d * inv_rho0;
        float t2 = tr * tr, t4 = t2 * t2;
        float P = p->B * (t4 * t2 * tr - 1.0f);
        rho[i] = d;
        prho[i] = P / (d * d);
    }
}

static inline double eos_sens(const or_sph_params* p, float rho) {
    const double r = (double)rho, q = r / (double)p->rho0, q7 = q * q * q * q * q * q * q;
    return (double)p->B / (r * r) * (5.0 * q7 + 2.0);
}

/* pass 2 over sorted targets [i0, i1): pressure + viscosity + XSPH + kick-drift + walls.
 * Reads p2/v2/rho/prho (all sorted slots, ghosts included), writes pos_out/vel_out[i]. */
static void force_range_impl(const or_sph_params* p, const float* p2, const float* v2, const float* rho,
                             const float* prho, const uint32_t* sk, const uint32_t* cs, int i0, int i1, float dt,
                             float t, float* pos_out, float* vel_out, float* acc3, float* mag5, int nthreads) {
    const or_grid* g = &p->grid;
    const float m = p->mass, four_h2 = p->four_h2;
    const float h = p->h, eta2 = 0.01f * h * h, ac0 = p->alpha * p->c0, eps = p->eps_xsph;
    const float fx = p->f_amp != 0.0f ? p->f_amp * sinf(6.28318530718f * p->f_freq * t) : 0.0f;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1024)
    for (int i = i0; i < i1; ++i) {
        uint32_t rg[OR_MAX_ROWS][2];
        int nr = neighbour_rows(g, cs, sk[i], rg);
        float xi = p2[3 * i], yi = p2[3 * i + 1], zi = p2[3 * i + 2];
        float ui = v2[3 * i], vi = v2[3 * i + 1], wi = v2[3 * i + 2];
        float rhoi = rho[i], pri = prho[i];
        float ax = 0, ay = 0, az = 0, sx = 0, sy = 0, sz = 0;
        /* diagnostics: am = Σ m|F|r(|Pρ_i| + |Pρ_j| + |Π_ij|), the pressure and viscous pair terms before they
         * cancel; sm = Σ|pair XSPH term|; em = Σ m|F|r(E_i + E_j), E = |dPρ/dρ|·ρ = (B/ρ²)(5(ρ/ρ0)^7 + 2): the
         * acceleration change per unit relative density error of both ends (Tait EOS sensitivity); qa, qs: the
         * support-edge conditioning of am's and sm's terms (oracle.h, OR_DIAG_DQ) */
        double am = 0.0, sm = 0.0, em = 0.0, qa = 0.0, qs = 0.0;
        const double Ei = mag5 ? eos_sens(p, rhoi) : 0.0;
        for (int r = 0; r < nr; ++r)
            for (uint32_t j = rg[r][0]; j < rg[r][1]; ++j) {
                if ((int)j == i) continue;
                float ddx = xi - p2[3 * j], ddy = yi - p2[3 * j + 1], ddz = zi - p2[3 * j + 2];
                float r2 = ddx * ddx + ddy * ddy + ddz * ddz;
                if (!(r2 < four_h2)) continue;
                float W, F;
                kernel_wf(p, r2, &W, &F);
                float du = ui - v2[3 * j], dv = vi - v2[3 * j + 1], dw = wi - v2[3 * j + 2];
                float vr = du * ddx + dv * ddy + dw * ddz;
                float rbar = 0.5f * (rhoi + rho[j]);
                float pi_ij = 0.0f;
                if (vr < 0.0f) {
                    float mu = h * vr / (r2 + eta2);
                    pi_ij = -ac0 * mu / rbar;
                }
                float c = -m * (pri + prho[j] + pi_ij) * F;
                ax += c * ddx; ay += c * ddy; az += c * ddz;
                float cx = eps * m / rbar * W;
                sx -= cx * du; sy -= cx * dv; sz -= cx * dw;
                if (mag5) {
                    const double mfr = (double)m * fabs((double)F) * sqrt((double)r2);
                    const double ta = mfr * (fabs((double)pri) + fabs((double)prho[j]) + fabs((double)pi_ij));
                    const double ts = fabs((double)cx) * sqrt((double)du * du + (double)dv * dv + (double)dw * dw);
                    am += ta;
                    sm += ts;
                    em += mfr * (Ei + eos_sens(p, rho[j]));
                    const double qd = sqrt((double)r2) * (double)p->inv_h;
                    if (qd >= 1.0) {
                        const double te = fmax(2.0 - qd, 1e-12);
                        qa += 2.0 * ta * OR_DIAG_DQ / te;
                        qs += 3.0 * ts * OR_DIAG_DQ / te;
                    }
                }
            }
        if (acc3) { acc3[3 * (size_t)i] = ax; acc3[3 * (size_t)i + 1] = ay; acc3[3 * (size_t)i + 2] = az; }
        if (mag5) {
            float* o = mag5 + 5 * (size_t)i;
            o[0] = (float)am; o[1] = (float)sm; o[2] = (float)em; o[3] = (float)qa; o[4] = (float)qs;
        }
        float nu = ui + (ax + p->g[0] + fx) * dt;
        float nv = vi + (ay + p->g[1]) * dt;
        float nw = wi + (az + p->g[2]) * dt;
        float npos[3] = {xi + (nu + sx) * dt, yi + (nv + sy) * dt, zi + (nw + sz) * dt};
        float nvel[3] = {nu, nv, nw};
        for (int a = 0; a < p->dim; ++a) {
            if (npos[a] < 0.0f) { npos[a] = 0.0f; if (nvel[a] < 0.0f) nvel[a] = -p->wall_e * nvel[a]; }
            if (npos[a] > p->L[a]) { npos[a] = p->L[a]; if (nvel[a] > 0.0f) nvel[a] = -p->wall_e * nvel[a]; }
        }
        if (p->dim == 2) { npos[2] = 0.0f; nvel[2] = 0.0f; }
        pos_out[3 * (size_t)i] = npos[0]; pos_out[3 * (size_t)i + 1] = npos[1]; pos_out[3 * (size_t)i + 2] = npos[2];
        vel_out[3 * (size_t)i] = nvel[0]; vel_out[3 * (size_t)i + 1] = nvel[1]; vel_out[3 * (size_t)i + 2] = nvel[2];
    }
}

void or_sph_force_range(const or_sph_params* p, const float* p2, const float* v2, const float* rho,
                        const float* prho, const uint32_t* sk, const uint32_t* cs, int i0, int i1, float dt,
                        float t, float* pos_out, float* vel_out, int nthreads) {
    force_range_impl(p, p2, v2, rho, prho, sk, cs, i0, i1, dt, t, pos_out, vel_out, NULL, NULL, nthreads);
}

void or_sph_force_range_diag(const or_sph_params* p, const float* p2, const float* v2, const float* rho,
                             const float* prho, const uint32_t* sk, const uint32_t* cs, int i0, int i1, float dt,
                             float t, float* pos_out, float* vel_out, float* acc3, float* mag5, int nthreads) {
    force_range_impl(p, p2, v2, rho, prho, sk, cs, i0, i1, dt, t, pos_out, vel_out, acc3, mag5, nthreads);
}

int or_sph_step(const or_sph_params* p, int n, float* pos, float* vel, int32_t* id,
                float dt, float t, float* rho_out, float* prho_out, uint32_t* cs_out, int nthreads) {
    return or_sph_step_diag(p, n, pos, vel, id, dt, t, rho_out, prho_out, cs_out, NULL, NULL, nthreads);
}

int or_sph_step_diag(const or_sph_params* p, int n, float* pos, float* vel, int32_t* id, float dt, float t,
                     float* rho_out, float* prho_out, uint32_t* cs_out, float* acc3, float* mag5, int nthreads) {
    const or_grid* g = &p->grid;
    uint32_t nk = (uint32_t)g->G[0] * (uint32_t)g->xsub * (uint32_t)g->G[1] * (uint32_t)g->G[2];
    size_t nn = (size_t)(n > 0 ? n : 1);
    uint32_t* keys = (uint32_t*)malloc(sizeof(uint32_t) * nn);
    uint32_t* perm = (uint32_t*)malloc(sizeof(uint32_t) * nn);
    uint32_t* sk = (uint32_t*)malloc(sizeof(uint32_t) * nn);
    uint32_t* cs = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)nk + 1));
    float* p2 = (float*)malloc(sizeof(float) * 3 * nn);
    float* v2 = (float*)malloc(sizeof(float) * 3 * nn);
    int32_t* id2 = (int32_t*)malloc(sizeof(int32_t) * nn);
    float* rho = (float*)malloc(sizeof(float) * nn);
    float* prho = (float*)malloc(sizeof(float) * nn);
    /* hash + stable sort + reorder + cell start */
    or_keys(g, n, pos, keys);
    or_stable_sort(n, keys, nk, perm);
    for (int i = 0; i < n; ++i) {
        uint32_t s = perm[i];
        sk[i] = keys[s];
        memcpy(p2 + 3 * (size_t)i, pos + 3 * (size_t)s, 12);
        memcpy(v2 + 3 * (size_t)i, vel + 3 * (size_t)s, 12);
        id2[i] = id[s];
    }
    or_cell_start(n, sk, nk, cs);
    or_sph_density_range(p, p2, sk, cs, 0, n, rho, prho, nthreads);
    force_range_impl(p, p2, v2, rho, prho, sk, cs, 0, n, dt, t, pos, vel, acc3, mag5, nthreads);
    memcpy(id, id2, sizeof(int32_t) * (size_t)n);
    if (rho_out) memcpy(rho_out, rho, sizeof(float) * (size_t)n);
    if (prho_out) memcpy(prho_out, prho, sizeof(float) * (size_t)n);
    if (cs_out) memcpy(cs_out, cs, sizeof(uint32_t) * ((size_t)nk + 1));
    free(keys); free(perm); free(sk); free(cs); free(p2); free(v2); free(id2); free(rho); free(prho);
    return 0;
}
