/* contact_oracle.c — CPU restatement of the reference contact model (TEST INFRASTRUCTURE ONLY).
 *
 * Line-by-line restatement of /root/reference/Assets/Compute/SimulateParticles.compute:
 *   GetGridCoord/GridHash :102-109, ApplySPHForces :211-309, ApplyDragForce :311-324,
 *   UpdateMotion :326-357, quat_mul :359-365, UpdateRotation :379-408,
 * with the two semantic choices of SPEC_SPH.md §1: Jacobi reads (the reference's in-place
 * write at :308 races) and the gather form of the InterlockedAdd reaction torque (:291-294),
 * which gives the same int32 sums (integer addition is associative).
 * HLSL intrinsics: length = sqrt(dot), dot = x*x+y*y+z*z, saturate = clamp01 (NaN->0),
 * normalize(v) = v / length(v), pow(x,2.0) = x*x, (int3)(float3) = D3D ftoi (trunc, sat, NaN->0).
 * Compiled with -ffp-contract=off. PARITY UNPINNED by reference fixtures (see oracle.h).
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define GRID_DIM 32
#define TORQUE_SCALE 10000
#define ADHESION_DELTA_SCALE 1000000

/* HLSL pow / exp / sin / cos / atan2 are approximations; evaluated in double and rounded once (as the
 * GPU does, vec3.h), so the restatement and the GPU agree bit for bit. */
/* pow(x, 1.25), x >= 0 (compute:279, the model's only pow): x * sqrt(sqrt(x)) in double */
static inline float pow125r(float x) { double d = (double)x; return (float)(d * sqrt(sqrt(d))); }
static inline float expr(float x) { return (float)exp((double)x); }
static inline float sinr(float x) { return (float)sin((double)x); }
static inline float cosr(float x) { return (float)cos((double)x); }
static inline float atan2r(float y, float x) { return (float)atan2((double)y, (double)x); }

typedef struct { float x, y, z; } f3;
static inline f3 mk(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 mul(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline f3 divs(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
static inline float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float len(f3 a) { return sqrtf(dot(a, a)); }
static inline f3 cross(f3 a, f3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static inline float sat(float x) { return x > 0.0f ? (x < 1.0f ? x : 1.0f) : 0.0f; }
static inline f3 nrm(f3 a) { return divs(a, len(a)); }
static inline f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
static inline void st3(float* p, f3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }

static inline int32_t ftoi(float x) {   /* D3D10+ ftoi: truncate, saturate, NaN -> 0 */
    if (x != x) return 0;
    if (x >= 2147483648.0f) return 2147483647;
    if (x <= -2147483648.0f) return (int32_t)0x80000000;
    return (int32_t)x;
}

typedef struct { f3 force, torque; int hit; f3 react; } pair_out;

/* One pair evaluated from `self`'s thread (compute:240-296). Returns self's repulsion and
 * rolling torque A, and the rolling torque B that the reference adds to the other
 * particle (:287). */
static inline pair_out contact_pair(const or_contact_params* P, const or_particle84* self,
                                    const or_particle84* other) {
    pair_out o;
    o.hit = 0; o.force = mk(0, 0, 0); o.torque = mk(0, 0, 0); o.react = mk(0, 0, 0);
    f3 posA = ld3(self->position), velA = ld3(self->velocity), omegaA = ld3(self->angularVelocity);
    float rA = self->radius;
    float effectiveRadiusA = rA * 0.5f;                         /* :225 */
    f3 posB = ld3(other->position), velB = ld3(other->velocity), omegaB = ld3(other->angularVelocity);
    float rB = other->radius;
    float effectiveRadiusB = rB * 0.5f;                         /* :248 */
    f3 delta = sub(posA, posB);                                 /* :249 */
    float dist = len(delta);
    float overlap = (effectiveRadiusA + effectiveRadiusB) - dist;
    if (!(overlap > 0.001f)) return o;                          /* :253 */
    o.hit = 1;
    f3 dir = divs(delta, dist);
    float overlapFalloff = sat(overlap / (effectiveRadiusA + effectiveRadiusB));
    float falloff = sat(1.0f - dist / (effectiveRadiusA + effectiveRadiusB));
    o.force = mul(mul(mul(dir, falloff), P->repulsion_strength), overlapFalloff); /* :260 */
    f3 contactPointA = sub(posA, mul(dir, effectiveRadiusA));  /* :264 */
    f3 contactPointB = add(posB, mul(dir, effectiveRadiusB));
    f3 surfaceVelA = add(velA, cross(omegaA, sub(contactPointA, posA)));
    f3 surfaceVelB = add(velB, cross(omegaB, sub(contactPointB, posB)));
    f3 relSurfaceVel = sub(surfaceVelA, surfaceVelB);
    f3 tangentVel = sub(relSurfaceVel, mul(dir, dot(relSurfaceVel, dir)));  /* :271 */
    float slipSpeed = len(tangentVel);
    if (slipSpeed > 1e-4f) {                                    /* :274 */
        f3 frictionDir = divs(tangentVel, slipSpeed);
        float torqueInput = fabsf(slipSpeed * P->torque_factor);
        float frictionMag = pow125r(torqueInput);
        frictionMag = fminf(frictionMag, 10.0f);
        float torqueRadiusScale = overlapFalloff * overlapFalloff;          /* pow(x, 2.0) :282 */
        float effectiveRadiusTorqueA = torqueRadiusScale * effectiveRadiusA * P->roll_mult;
        float effectiveRadiusTorqueB = torqueRadiusScale * effectiveRadiusB * P->roll_mult;
        o.torque = cross(mul(neg(dir), effectiveRadiusTorqueA), mul(neg(frictionDir), frictionMag));
        o.react = cross(mul(dir, effectiveRadiusTorqueB), mul(frictionDir, frictionMag));
        o.hit = 2;
    }
    return o;
}

/* ---- adhesion (compute:424-584) ---- */
typedef struct { float x, y, z, w; } f4;
static inline f4 q4(const float* q) { f4 r = {q[0], q[1], q[2], q[3]}; return r; }
static inline f3 qv(f4 q) { return mk(q.x, q.y, q.z); }
static inline f4 qmul(f4 q1, f4 q2) {            /* quat_mul :359-365 */
    f3 v = add(add(mul(qv(q2), q1.w), mul(qv(q1), q2.w)), cross(qv(q1), qv(q2)));
    f4 r = {v.x, v.y, v.z, q1.w * q2.w - dot(qv(q1), qv(q2))};
    return r;
}
static inline f4 qconj(f4 q) { f4 r = {-q.x, -q.y, -q.z, q.w}; return r; }   /* :368-371 */
static inline f3 qrot(f4 q, f3 v) {                                          /* :374-377 */
    return add(v, mul(cross(qv(q), add(cross(qv(q), v), mul(v, q.w))), 2.0f));
}
/* (int)round(x * ADHESION_DELTA_SCALE): HLSL round = round half to even (rintf in the default
 * rounding mode), the cast = D3D ftoi */
static inline int32_t fixp(float x) { return ftoi(rintf(x * (float)ADHESION_DELTA_SCALE)); }
static inline void add_q(int32_t* acc, f4 d) {
    acc[0] = (int32_t)((uint32_t)acc[0] + (uint32_t)fixp(d.x));
    acc[1] = (int32_t)((uint32_t)acc[1] + (uint32_t)fixp(d.y));
    acc[2] = (int32_t)((uint32_t)acc[2] + (uint32_t)fixp(d.z));
    acc[3] = (int32_t)((uint32_t)acc[3] + (uint32_t)fixp(d.w));
}
static inline f4 qdiff(f4 a, f4 b) { f4 r = {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; return r; }

/* :474-514 (side A) / :516-540 (side B) */
static void anchor_push(float strength, f4 q, f3 anchorLocal, f3 desiredMove, int32_t* acc) {
    f3 rWorld = qrot(q, anchorLocal);
    f3 rotAxis = cross(rWorld, desiredMove);
    float rotAxisLength = len(rotAxis);
    if (!(rotAxisLength > 1e-6f)) return;
    rotAxis = nrm(rotAxis);
    float effectiveness = fabsf(dot(cross(rotAxis, rWorld), desiredMove));
    if (!(effectiveness > 1e-6f)) return;
    float rotAngle = strength * effectiveness * 5.0f;
    f4 rotQuat = {rotAxis.x * sinr(rotAngle * 0.5f), rotAxis.y * sinr(rotAngle * 0.5f),
                  rotAxis.z * sinr(rotAngle * 0.5f), cosr(rotAngle * 0.5f)};
    add_q(acc, qdiff(qmul(rotQuat, q), q));
}

/* One bond's thread of ApplyAdhesionConstraints: the 16 ints it would InterlockedAdd
 * (Δv_A xyz 0, Δv_B xyz 0, Δq_A xyzw, Δq_B xyzw). `v1` = velocities after ApplySPHForces. */
static void bond_terms(const or_adhesion84* c, int n, const or_particle84* in, const f3* v1, float dt,
                       int32_t t[16]) {
    memset(t, 0, 16 * sizeof(int32_t));
    int idxA = c->particleA, idxB = c->particleB;
    if (idxA < 0 || idxB < 0 || idxA >= n || idxB >= n) return;              /* :432 */
    const or_particle84* pA = &in[idxA];
    const or_particle84* pB = &in[idxB];
    f3 posA = ld3(pA->position), posB = ld3(pB->position);
    f4 rotA = q4(pA->rotation), rotB = q4(pB->rotation);
    /* spring :437-456 */
    f3 delta = sub(posB, posA);
    float dist = len(delta);
    if (dist > 1e-6f) {
        f3 dir = divs(delta, dist);
        float displacement = dist - c->restLength;
        float springMultiplier = 1.0f;
        f3 force = mul(dir, displacement * c->springStiffness * springMultiplier);
        f3 relVel = sub(v1[idxB], v1[idxA]);
        float dampingForce = dot(relVel, dir) * c->springDamping;
        force = add(force, mul(dir, dampingForce));
        f3 deltaVA = mul(divs(force, pA->mass), dt);
        f3 deltaVB = mul(divs(neg(force), pB->mass), dt);
        t[0] = fixp(deltaVA.x); t[1] = fixp(deltaVA.y); t[2] = fixp(deltaVA.z);
        t[4] = fixp(deltaVB.x); t[5] = fixp(deltaVB.y); t[6] = fixp(deltaVB.z);
    }
    if (c->enableAnchorConstraint != 1) return;                               /* :457 */
    float constraintStrength = c->anchorConstraintStiffness * dt;
    f3 ancA = ld3(c->anchorLocalPosA), ancB = ld3(c->anchorLocalPosB);
    f3 currentAnchorA = add(posA, qrot(rotA, ancA));
    f3 currentAnchorB = add(posB, qrot(rotB, ancB));
    f3 anchorDelta = sub(currentAnchorB, currentAnchorA);
    float anchorDist = len(anchorDelta);
    if (anchorDist > 1e-6f) {
        f3 anchorDir = divs(anchorDelta, anchorDist);
        anchor_push(constraintStrength, rotA, ancA, anchorDir, t + 8);
        anchor_push(constraintStrength, rotB, ancB, neg(anchorDir), t + 12);
    }
    /* relative orientation :541-582 */
    f4 currentRel = qmul(qconj(rotA), rotB);
    f4 correction = qmul(q4(c->initialRelOrientation), qconj(currentRel));
    float correctionAngle = 2.0f * atan2r(len(qv(correction)), fabsf(correction.w));
    if (correctionAngle > 1e-6f) {
        f3 axis = nrm(qv(correction));
        float ocs = constraintStrength * 2.0f;
        float angA = -ocs * correctionAngle * 0.5f;
        float angB = ocs * correctionAngle * 0.5f;
        f4 rqA = {axis.x * sinr(angA * 0.5f), axis.y * sinr(angA * 0.5f), axis.z * sinr(angA * 0.5f), cosr(angA * 0.5f)};
        f4 rqB = {axis.x * sinr(angB * 0.5f), axis.y * sinr(angB * 0.5f), axis.z * sinr(angB * 0.5f), cosr(angB * 0.5f)};
        add_q(t + 8, qdiff(qmul(rqA, rotA), rotA));
        add_q(t + 12, qdiff(qmul(rqB, rotB), rotB));
    }
}

static inline int32_t or_coord_r(float x, float R) {   /* compute:102-105 */
    float g = (x + R) / 4.0f;
    if (!(g > 0.0f)) return 0;
    if (g >= (float)(GRID_DIM - 1)) return GRID_DIM - 1;
    return (int32_t)g;
}

/* One frame (controller:265-331): ApplySPHForces for every particle, then (nconn > 0) the
 * adhesion pass :424-607, then drag / UpdateMotion / UpdateRotation. */
int or_contact_step_bonds(const or_contact_params* P, int n, or_particle84* parts, int32_t* torque_out,
                          const or_adhesion84* conns, int nconn, int32_t* terms_out, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    const uint32_t NK = GRID_DIM * GRID_DIM * GRID_DIM;
    size_t nn = (size_t)(n > 0 ? n : 1);
    uint32_t* keys = (uint32_t*)malloc(sizeof(uint32_t) * nn);
    uint32_t* perm = (uint32_t*)malloc(sizeof(uint32_t) * nn);
    uint32_t* sk = (uint32_t*)malloc(sizeof(uint32_t) * nn);
    uint32_t* cs = (uint32_t*)malloc(sizeof(uint32_t) * (NK + 1));
    or_particle84* in = (or_particle84*)malloc(sizeof(or_particle84) * nn);
    f3* v1 = (f3*)malloc(sizeof(f3) * nn);
    f3* w1 = (f3*)malloc(sizeof(f3) * nn);
    uint32_t* tqa = (uint32_t*)malloc(sizeof(uint32_t) * 3 * nn);
    memcpy(in, parts, sizeof(or_particle84) * (size_t)n);
    /* grid: same neighbour set as the reference's linked lists, visited in stable-sorted order */
    for (int i = 0; i < n; ++i) {
        int32_t cx = or_coord_r(in[i].position[0], P->spawn_radius);
        int32_t cy = or_coord_r(in[i].position[1], P->spawn_radius);
        int32_t cz = or_coord_r(in[i].position[2], P->spawn_radius);
        keys[i] = ((uint32_t)cx * GRID_DIM + (uint32_t)cy) * GRID_DIM + (uint32_t)cz;
    }
    or_stable_sort(n, keys, NK, perm);
    for (int i = 0; i < n; ++i) sk[i] = keys[perm[i]];
    or_cell_start(n, sk, NK, cs);

    const float dt = P->dt;
#pragma omp parallel for schedule(dynamic, 64)
    for (int a = 0; a < n; ++a) {
        const or_particle84* self = &in[a];
        uint32_t key = keys[a];
        int32_t cz = (int32_t)(key % GRID_DIM), cy = (int32_t)((key / GRID_DIM) % GRID_DIM),
                cx = (int32_t)(key / (GRID_DIM * GRID_DIM));
        f3 totalForce = mk(0, 0, 0), totalTorque = mk(0, 0, 0);
        uint32_t tq[3] = {0, 0, 0};   /* wrapping int32 sums (InterlockedAdd) */
        int32_t z0 = cz > 0 ? cz - 1 : 0, z1 = cz < GRID_DIM - 1 ? cz + 1 : GRID_DIM - 1;
        for (int ddx = -1; ddx <= 1; ++ddx) {
            int32_t x = cx + ddx;
            if (x < 0 || x >= GRID_DIM) continue;
            for (int ddy = -1; ddy <= 1; ++ddy) {
                int32_t y = cy + ddy;
                if (y < 0 || y >= GRID_DIM) continue;
                uint32_t rowk = ((uint32_t)x * GRID_DIM + (uint32_t)y) * GRID_DIM;
                for (uint32_t s = cs[rowk + (uint32_t)z0]; s < cs[rowk + (uint32_t)z1 + 1]; ++s) {
                    uint32_t b = perm[s];
                    if ((int)b == a) continue;                          /* :240 */
                    const or_particle84* other = &in[b];
                    pair_out mine = contact_pair(P, self, other);
                    if (!mine.hit) continue;
                    totalForce = add(totalForce, mine.force);           /* :261 */
                    if (mine.hit == 2) totalTorque = add(totalTorque, mine.torque); /* :289 */
                    /* reaction: what b's thread scatters into a (:291-294) */
                    pair_out theirs = contact_pair(P, other, self);
                    if (theirs.hit == 2) {
                        f3 sc = mul(mul(theirs.react, dt), (float)TORQUE_SCALE);
                        tq[0] += (uint32_t)ftoi(sc.x);
                        tq[1] += (uint32_t)ftoi(sc.y);
                        tq[2] += (uint32_t)ftoi(sc.z);
                    }
                }
            }
        }
        /* :302-306 */
        f3 linearAccel = divs(totalForce, self->mass);
        f3 angularAccel = divs(totalTorque, self->momentOfInertia);
        v1[a] = add(ld3(self->velocity), mul(linearAccel, dt));
        w1[a] = add(ld3(self->angularVelocity), mul(angularAccel, dt));
        tqa[3 * a] = tq[0]; tqa[3 * a + 1] = tq[1]; tqa[3 * a + 2] = tq[2];
    }

    /* adhesion: ApplyAdhesionConstraints :424-584 on the post-ApplySPHForces state */
    uint32_t* dv = NULL;
    uint32_t* dq = NULL;
    if (nconn > 0) {
        dv = (uint32_t*)calloc(3 * nn, sizeof(uint32_t));
        dq = (uint32_t*)calloc(4 * nn, sizeof(uint32_t));
        for (int b = 0; b < nconn; ++b) {
            int32_t t[16];
            bond_terms(&conns[b], n, in, v1, dt, t);
            if (terms_out) memcpy(terms_out + 16 * (size_t)b, t, sizeof t);
            int32_t ia = conns[b].particleA, ib = conns[b].particleB;
            if (ia < 0 || ib < 0 || ia >= n || ib >= n) continue;
            for (int k = 0; k < 3; ++k) {
                dv[3 * (size_t)ia + k] += (uint32_t)t[k];
                dv[3 * (size_t)ib + k] += (uint32_t)t[4 + k];
            }
            for (int k = 0; k < 4; ++k) {
                dq[4 * (size_t)ia + k] += (uint32_t)t[8 + k];
                dq[4 * (size_t)ib + k] += (uint32_t)t[12 + k];
            }
        }
    }

#pragma omp parallel for schedule(static)
    for (int a = 0; a < n; ++a) {
        or_particle84 p = in[a];
        f3 vel = v1[a], omg = w1[a];
        f3 pos = ld3(p.position);
        const uint32_t* tq = tqa + 3 * (size_t)a;
        if (nconn > 0) {   /* ApplyAdhesionDeltas :593-601 */
            const uint32_t* d = dv + 3 * (size_t)a;
            const uint32_t* e = dq + 4 * (size_t)a;
            vel = add(vel, divs(mk((float)(int32_t)d[0], (float)(int32_t)d[1], (float)(int32_t)d[2]),
                                (float)ADHESION_DELTA_SCALE));
            float r[4];
            for (int k = 0; k < 4; ++k) r[k] = p.rotation[k] + (float)(int32_t)e[k] / (float)ADHESION_DELTA_SCALE;
            float l = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3]);
            for (int k = 0; k < 4; ++k) p.rotation[k] = r[k] / l;
        }
        /* ApplyDragForce :316-323 */
        if (P->drag_id >= 0 && P->drag_id == a) {
            f3 toTarget = sub(ld3(P->drag_target), pos);
            f3 force = mul(mul(toTarget, P->drag_strength), dt);
            vel = add(vel, divs(force, p.mass));
        }
        /* UpdateMotion :332-354 */
        float linearDamping = expr(-p.drag * P->global_drag * dt);
        float angularDamping = expr(-P->torque_damping * dt);
        vel = mul(vel, linearDamping);
        omg = mul(omg, angularDamping);
        pos = add(pos, mul(vel, dt));
        float distFromOrigin = len(pos);
        if (distFromOrigin > P->spawn_radius) {
            f3 norm = nrm(pos);
            pos = mul(norm, P->spawn_radius);
            vel = sub(vel, mul(norm, 2.0f * dot(vel, norm)));           /* reflect */
            f3 tangentialVel = sub(vel, mul(norm, dot(vel, norm)));
            f3 frictionDir = nrm(add(tangentialVel, mk(1e-6f, 1e-6f, 1e-6f)));
            float frictionMag = len(tangentialVel) * P->boundary_friction;
            float effectiveRadius = p.radius * P->roll_mult;
            f3 torque = cross(mul(neg(norm), effectiveRadius), mul(neg(frictionDir), frictionMag));
            omg = add(omg, mul(divs(torque, p.momentOfInertia), dt));
        }
        /* UpdateRotation :385-406 */
        f3 torque = divs(mk((float)(int32_t)tq[0], (float)(int32_t)tq[1], (float)(int32_t)tq[2]),
                         (float)TORQUE_SCALE);
        f3 angAcc = divs(torque, p.momentOfInertia);
        omg = add(omg, angAcc);
        omg = mul(omg, expr(-P->torque_damping * dt));
        float angle = len(mul(omg, dt));
        if (angle > 0.00001f) {
            f3 axis = nrm(omg);
            float s = sinr(angle * 0.5f), c = cosr(angle * 0.5f);
            float dq[4] = {axis.x * s, axis.y * s, axis.z * s, c};
            const float* q = p.rotation;
            /* quat_mul(dq, q) :359-365 */
            f3 dqv = mk(dq[0], dq[1], dq[2]), qv = mk(q[0], q[1], q[2]);
            f3 xyz = add(add(mul(qv, dq[3]), mul(dqv, q[3])), cross(dqv, qv));
            float w = dq[3] * q[3] - dot(dqv, qv);
            float l = sqrtf(xyz.x * xyz.x + xyz.y * xyz.y + xyz.z * xyz.z + w * w);
            p.rotation[0] = xyz.x / l; p.rotation[1] = xyz.y / l; p.rotation[2] = xyz.z / l;
            p.rotation[3] = w / l;
        }
        st3(p.position, pos); st3(p.velocity, vel); st3(p.angularVelocity, omg);
        parts[a] = p;
        if (torque_out) {
            torque_out[3 * a] = (int32_t)tq[0]; torque_out[3 * a + 1] = (int32_t)tq[1];
            torque_out[3 * a + 2] = (int32_t)tq[2];
        }
    }
    free(keys); free(perm); free(sk); free(cs); free(in); free(v1); free(w1); free(tqa);
    free(dv); free(dq);
    return 0;
}

int or_contact_step(const or_contact_params* P, int n, or_particle84* parts, int32_t* torque_out,
                    int nthreads) {
    return or_contact_step_bonds(P, n, parts, torque_out, NULL, 0, NULL, nthreads);
}

/* ---- InitParticles (compute:118-194) ----
 * HLSL sin / pow are evaluated in double and rounded once to float: the correctly rounded float
 * value (D3D leaves their precision to the hardware; the device kernel does the same, so both
 * produce the same bits). frac(x) = x - floor(x); lerp(a, b, t) = a + t·(b − a). */
static inline float hsin(float x) { return (float)sin((double)x); }
static inline float hpow(float x, float y) { return (float)pow((double)x, (double)y); }
static inline float hfrac(float x) { return x - floorf(x); }
static inline float sgn_hash(float sf, float a, float b) { return hfrac(hsin(sf * a) * b) * 2.0f - 1.0f; }

void or_init_particles(int n, int active, float spawn_radius, float min_radius, float max_radius, float density,
                       int genome_modes, int default_mode, or_particle84* out) {
    memset(out, 0, sizeof(or_particle84) * (size_t)(n > 0 ? n : 0));   /* a fresh ComputeBuffer is zero */
    for (int i = 0; i < active && i < n; ++i) {
        or_particle84 p;
        memset(&p, 0, sizeof p);
        uint32_t seed = (uint32_t)i * 65537u + 17u;                                       /* :123 */
        float sf = (float)seed;
        if (i != 0) {
            f3 dir = nrm(mk(sgn_hash(sf, 12.9898f, 43758.5453f), sgn_hash(sf, 78.233f, 43758.5453f),
                            sgn_hash(sf, 91.934f, 43758.5453f)));                        /* :134-138 */
            float randVal = hfrac(hsin(sf * 1.2345f) * 10000.0f);                          /* :141 */
            float dist = hpow(randVal, 1.0f / 3.0f) * spawn_radius;
            f3 pos = mul(dir, dist);
            if (i > 1) {                                                                  /* :147-155 */
                float repelDist = hpow(0.5f * (float)i / (float)n, 1.0f / 3.0f) * spawn_radius * 0.1f;
                f3 e = nrm(mk(sgn_hash(sf, 45.678f, 43758.5453f), sgn_hash(sf, 67.890f, 43758.5453f),
                              sgn_hash(sf, 12.345f, 43758.5453f)));
                pos = add(pos, mul(e, repelDist));
            }
            st3(p.position, pos);
        }
        p.radius = min_radius + hfrac(hsin(sf * 3.456f) * 999.0f) * (max_radius - min_radius);   /* :160 */
        float volume = (4.0f / 3.0f) * 3.1415926f * hpow(p.radius, 3.0f);
        p.mass = density * volume;
        p.momentOfInertia = (2.0f / 5.0f) * p.mass * p.radius * p.radius;
        p.drag = 0.5f + hfrac(hsin(sf * 5.6789f) * 888.0f) * (1.0f - 0.5f);                  /* :166 */
        p.repulsionStrength = 1.0f;
        int modeIndex = -1;                                                               /* :172-186 */
        if (genome_modes > 0) {
            if (hfrac(hsin(sf * 78.123f) * 5432.1f) < 0.5f)
                modeIndex = default_mode;
            else
                modeIndex = (int)(hfrac(hsin(sf * 43.21f) * 8765.43f) * (float)genome_modes);
            modeIndex = modeIndex < 0 ? 0 : (modeIndex > genome_modes - 1 ? genome_modes - 1 : modeIndex);
        }
        p.modeIndex = modeIndex;
        p.rotation[3] = 1.0f;
        out[i] = p;
    }
}

/* The buffer half of ProcessPendingSplits (ParticleSystemController.cs:832-959) on an AoS
 * array of n_cap records; returns the new active count. */
int or_split_particles(or_particle84* parts, int active, const or_split92* sp, int count) {
    for (int k = 0; k < count; ++k) {
        or_particle84* a = &parts[sp[k].parent];
        memcpy(a->position, sp[k].posA, 12);
        memcpy(a->velocity, sp[k].velA, 12);
        memcpy(a->rotation, sp[k].rotA, 16);
        a->modeIndex = sp[k].modeA;
        or_particle84* b = &parts[active];
        *b = *a;
        memcpy(b->position, sp[k].posB, 12);
        memcpy(b->velocity, sp[k].velB, 12);
        memcpy(b->rotation, sp[k].rotB, 16);
        b->modeIndex = sp[k].modeB;
        active += 1;
    }
    return active;
}
