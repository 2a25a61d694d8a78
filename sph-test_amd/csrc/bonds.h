// bonds.h — adhesion bonds on the device (§8f-1): the per-particle gather that replaces the
// reference's InterlockedAdd delta buffers. Included by contact.hip and adhesion.hip.
#pragma once

#include "common.h"
#include "vec3.h"

namespace sph {

constexpr float ADHESION_DELTA_SCALE = 1000000.0f;   // SimulateParticles.compute:20

// ApplyAdhesionDeltas (compute:587-607) for one particle: sum the int terms of its bonds
// (wrapping int32, as InterlockedAdd), then v += Δv/1e6 and q = normalize(q + Δq/1e6).
// The reference runs it over every active particle whenever a bond exists, so particles
// without bonds are re-normalised too.
__device__ __forceinline__ void bond_gather(const BondView& b, int32_t pid, f3& v, float4& q) {
    if (b.count == 0) return;
    uint32_t s0 = 0, s1 = 0, s2 = 0, r0 = 0, r1 = 0, r2 = 0, r3 = 0;
    if ((uint32_t)pid < (uint32_t)b.n_index) {
        const uint32_t k0 = b.off[pid], k1 = b.off[pid + 1];
        for (uint32_t k = k0; k < k1; ++k) {
            const uint32_t e = b.ent[k];
            const uint32_t base = 4u * (e >> 1) + (e & 1u);
            const int4 dv = b.terms[base], dr = b.terms[base + 2];
            s0 += (uint32_t)dv.x; s1 += (uint32_t)dv.y; s2 += (uint32_t)dv.z;
            r0 += (uint32_t)dr.x; r1 += (uint32_t)dr.y; r2 += (uint32_t)dr.z; r3 += (uint32_t)dr.w;
        }
    }
    v = v + mk((float)(int32_t)s0, (float)(int32_t)s1, (float)(int32_t)s2) / ADHESION_DELTA_SCALE;
    const float4 r = make_float4(q.x + (float)(int32_t)r0 / ADHESION_DELTA_SCALE,
                                 q.y + (float)(int32_t)r1 / ADHESION_DELTA_SCALE,
                                 q.z + (float)(int32_t)r2 / ADHESION_DELTA_SCALE,
                                 q.w + (float)(int32_t)r3 / ADHESION_DELTA_SCALE);
    const float l = sqrtf(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w);
    q = make_float4(r.x / l, r.y / l, r.z / l, r.w / l);
}

}  // namespace sph
