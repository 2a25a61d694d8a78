// adhesion.hip — Model R adhesion bonds, gfx950.
//
// The reference dispatches ApplyAdhesionConstraints (SimulateParticles.compute:424-584) with
// one thread per bond: each adds its fixed-point (×1e6) Δv and Δq terms into per-particle int
// buffers with 14 InterlockedAdds, and ApplyAdhesionDeltas (:587-607) applies and clears them
// (host clears too: ParticleSystemController.cs:292-294). Here the bond pass writes each
// bond's four int terms to its own 64-byte record (coalesced, no atomics) and the particle pass
// gathers them through a CSR incidence list (bonds.h, k_contact_finish). int32 sums are
// associative, so the totals equal the atomic ones bit for bit, in any order.
// Every rounding is the one written (no fused multiply-adds), as in the oracle: with the double-evaluated
// intrinsics (vec3.h) the Model R step is bit-identical to oracle/contact_oracle.c.
#pragma clang fp contract(off)
#include "common.h"
#include "vec3.h"

namespace sph {

constexpr int BD_BLK = 256;
constexpr float BOND_SCALE = 1000000.0f;   // ADHESION_DELTA_SCALE, compute:20

// (int3/int4)round(x * ADHESION_DELTA_SCALE): HLSL round is round-half-to-even (rint), the
// cast is D3D ftoi.
__device__ __forceinline__ int32_t fixp(float x) { return ftoi(rintf(x * BOND_SCALE)); }

__device__ __forceinline__ void add_q(int4& acc, float4 d) {
    acc.x = (int32_t)((uint32_t)acc.x + (uint32_t)fixp(d.x));
    acc.y = (int32_t)((uint32_t)acc.y + (uint32_t)fixp(d.y));
    acc.z = (int32_t)((uint32_t)acc.z + (uint32_t)fixp(d.z));
    acc.w = (int32_t)((uint32_t)acc.w + (uint32_t)fixp(d.w));
}

__device__ __forceinline__ float4 qsub(float4 a, float4 b) {
    return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}

// The anchor-to-anchor push for one side (compute:474-514 for A, :516-540 for B).
__device__ __forceinline__ void anchor_push(float strength, float4 q, f3 anchor_local, f3 desired, int4& dq) {
    const f3 r_world = quat_rotate(q, anchor_local);
    f3 axis = cross(r_world, desired);
    const float axis_len = len(axis);
    if (!(axis_len > 1e-6f)) return;
    axis = normalize(axis);
    const float effectiveness = fabsf(dot(cross(axis, r_world), desired));
    if (!(effectiveness > 1e-6f)) return;
    const float angle = strength * effectiveness * 5.0f;
    const float s = sin_r(angle * 0.5f), c = cos_r(angle * 0.5f);
    const float4 rq = make_float4(axis.x * s, axis.y * s, axis.z * s, c);
    add_q(dq, qsub(quat_mul(rq, q), q));
}

__global__ __launch_bounds__(BD_BLK) void k_bond_terms(BondSet bs, const int32_t* __restrict__ slot_of, int32_t n,
                                                      const float4* __restrict__ pos,
                                                      const float4* __restrict__ vel1,
                                                      const float4* __restrict__ rot, float dt,
                                                      int4* __restrict__ terms) {
    const int32_t b = blockIdx.x * BD_BLK + threadIdx.x;
    if (b >= bs.count) return;
    int4 dvA = make_int4(0, 0, 0, 0), dvB = dvA, dqA = dvA, dqB = dvA;
    const int2 e = bs.ends[b];
    if (e.x >= 0 && e.y >= 0 && e.x < n && e.y < n) {                     // :432
        const int32_t sa = slot_of[e.x], sb = slot_of[e.y];
        const float4 pA4 = pos[sa], pB4 = pos[sb], vA4 = vel1[sa], vB4 = vel1[sb];
        const float4 qA = rot[sa], qB = rot[sb];
        const f3 pA = xyz(pA4), pB = xyz(pB4);
        const float4 sp = bs.spring[b];   // rest, k, damping, anchor stiffness
        // --- spring (distance) constraint :436-456
        const f3 delta = pB - pA;
        const float dist = len(delta);
        if (dist > 1e-6f) {
            const f3 dir = delta / dist;
            const float displacement = dist - sp.x;
            const float springMultiplier = 1.0f;
            f3 force = dir * (displacement * sp.y * springMultiplier);
            const f3 relVel = xyz(vB4) - xyz(vA4);
            const float dampingForce = dot(relVel, dir) * sp.z;
            force = force + dir * dampingForce;
            const f3 deltaVA = force / vA4.w * dt;
            const f3 deltaVB = -force / vB4.w * dt;
            dvA = make_int4(fixp(deltaVA.x), fixp(deltaVA.y), fixp(deltaVA.z), 0);
            dvB = make_int4(fixp(deltaVB.x), fixp(deltaVB.y), fixp(deltaVB.z), 0);
        }
        const float4 ancA = bs.anc_a[b];
        if (__float_as_int(ancA.w) == 1) {                                 // :457
            const float constraintStrength = sp.w * dt;
            const f3 ancB = xyz(bs.anc_b[b]);
            // --- anchor-to-anchor distance :462-540
            const f3 anchorDelta = (pB + quat_rotate(qB, ancB)) - (pA + quat_rotate(qA, xyz(ancA)));
            const float anchorDist = len(anchorDelta);
            if (anchorDist > 1e-6f) {
                const f3 anchorDir = anchorDelta / anchorDist;
                anchor_push(constraintStrength, qA, xyz(ancA), anchorDir, dqA);
                anchor_push(constraintStrength, qB, ancB, -anchorDir, dqB);
            }
            // --- relative orientation :541-582
            const float4 currentRel = quat_mul(quat_conjugate(qA), qB);
            const float4 corr = quat_mul(bs.relq[b], quat_conjugate(currentRel));
            const float correctionAngle = 2.0f * atan2_r(len(xyz(corr)), fabsf(corr.w));
            if (correctionAngle > 1e-6f) {
                const f3 axis = normalize(xyz(corr));
                const float ocs = constraintStrength * 2.0f;
                const float angA = -ocs * correctionAngle * 0.5f;
                const float angB = ocs * correctionAngle * 0.5f;
                const float sA = sin_r(angA * 0.5f), cA = cos_r(angA * 0.5f);
                const float sB = sin_r(angB * 0.5f), cB = cos_r(angB * 0.5f);
                add_q(dqA, qsub(quat_mul(make_float4(axis.x * sA, axis.y * sA, axis.z * sA, cA), qA), qA));
                add_q(dqB, qsub(quat_mul(make_float4(axis.x * sB, axis.y * sB, axis.z * sB, cB), qB), qB));
            }
        }
    }
    int4* t = terms + 4 * (size_t)b;
    t[0] = dvA; t[1] = dvB; t[2] = dqA; t[3] = dqB;
}

void launch_bond_terms(BondSet bs, const int32_t* slot_of, int32_t n, const float4* pos, const float4* vel1,
                       const float4* rot, float dt, int4* terms, hipStream_t s) {
    if (bs.count > 0)
        k_bond_terms<<<(bs.count + BD_BLK - 1) / BD_BLK, BD_BLK, 0, s>>>(bs, slot_of, n, pos, vel1, rot, dt, terms);
}

}  // namespace sph
