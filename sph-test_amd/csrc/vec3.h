// vec3.h — float3 / quaternion helpers with the HLSL intrinsic semantics the Model R kernels
// restate (SimulateParticles.compute). Device-only; shared by contact.hip and adhesion.hip.
//   length = sqrt(dot), normalize(v) = v / length(v), saturate = clamp01 (NaN -> 0),
//   quat_mul :359-365, quat_conjugate :368-371, quat_rotate :374-377.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sph {

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
// a + b that the compiler may not fuse with the multiply producing b: accumulations whose summands
// reach them by different routes (registers, cross-lane shuffles) then round identically.
__device__ __forceinline__ f3 add_exact(f3 a, f3 b) {
#pragma clang fp contract(off)
    return {a.x + b.x, a.y + b.y, a.z + b.z};
}
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ f3 operator-(f3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len(f3 a) { return sqrtf(dot(a, a)); }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float saturate(float x) { return x > 0.0f ? (x < 1.0f ? x : 1.0f) : 0.0f; }
__device__ __forceinline__ f3 normalize(f3 a) { return a / len(a); }
__device__ __forceinline__ f3 xyz(float4 v) { return {v.x, v.y, v.z}; }

// HLSL's pow / exp / sin / cos / atan2 are approximations (D3D allows a few ulp). Model R evaluates
// them in double and rounds once, exactly as the oracle does (oracle/contact_oracle.c): both are then
// correctly rounded but for results within ~1e-16 of a float tie, so GPU and oracle agree bit for bit.
// pow(x, 1.25) for x >= 0 (compute:279 is the only pow): x·sqrt(sqrt(x)) in double, every step
// correctly rounded on both sides, so it matches the oracle bit for bit at a fraction of a general
// double pow's cost (the contact pass evaluates it twice per touching pair)
__device__ __forceinline__ float pow125_r(float x) {
    const double d = (double)x;
    return (float)(d * sqrt(sqrt(d)));
}
__device__ __forceinline__ float exp_r(float x) { return (float)exp((double)x); }
__device__ __forceinline__ float sin_r(float x) { return (float)sin((double)x); }
__device__ __forceinline__ float cos_r(float x) { return (float)cos((double)x); }
// sin_r and cos_r of one argument from one double sincos (one argument reduction; the same values)
__device__ __forceinline__ void sincos_r(float x, float& s, float& c) {
    double sd, cd;
    sincos((double)x, &sd, &cd);
    s = (float)sd;
    c = (float)cd;
}
__device__ __forceinline__ float atan2_r(float y, float x) { return (float)atan2((double)y, (double)x); }

__device__ __forceinline__ int32_t ftoi(float x) {   // D3D ftoi: truncate, saturate, NaN -> 0
    if (x != x) return 0;
    if (x >= 2147483648.0f) return 2147483647;
    if (x <= -2147483648.0f) return (int32_t)0x80000000;
    return (int32_t)x;
}

// quat_mul (compute:359-365): (q1.w q2.xyz + q2.w q1.xyz + q1.xyz × q2.xyz, q1.w q2.w − q1.xyz·q2.xyz)
__device__ __forceinline__ float4 quat_mul(float4 q1, float4 q2) {
    const f3 a = xyz(q1), b = xyz(q2);
    const f3 v = b * q1.w + a * q2.w + cross(a, b);
    return make_float4(v.x, v.y, v.z, q1.w * q2.w - dot(a, b));
}
__device__ __forceinline__ float4 quat_conjugate(float4 q) { return make_float4(-q.x, -q.y, -q.z, q.w); }
// quat_rotate (compute:374-377): v + 2·(q.xyz × (q.xyz × v + q.w·v))
__device__ __forceinline__ f3 quat_rotate(float4 q, f3 v) {
    const f3 u = xyz(q);
    return v + cross(u, cross(u, v) + v * q.w) * 2.0f;
}

}  // namespace sph
