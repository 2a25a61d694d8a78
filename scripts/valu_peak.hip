// valu_peak.hip — measures the chip's VALU issue rate (profiling only, not part of the product).
// Every lane runs 8 independent f32 FMA chains (or packed-f32 pk_fma chains) for ITERS steps,
// at 1, 2, 4 and 8 waves per SIMD. Prints wave-instructions per second: the peak that
// bench.py's roofline.valu divides by.
//   hipcc -O3 --offload-arch=gfx950 scripts/valu_peak.hip -o scripts/valu_peak.bin
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_fma(float* out, float a, float b) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
#pragma unroll 16
    for (int i = 0; i < ITERS; ++i) {
        x0 = fmaf(x0, a, b); x1 = fmaf(x1, a, b); x2 = fmaf(x2, a, b); x3 = fmaf(x3, a, b);
        x4 = fmaf(x4, a, b); x5 = fmaf(x5, a, b); x6 = fmaf(x6, a, b); x7 = fmaf(x7, a, b);
    }
    out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

typedef float v2f __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_pk_fma(float* out, float a, float b) {
    v2f x0 = {(float)threadIdx.x, 1.f}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
        x6 = x0 + 6, x7 = x0 + 7;
    const v2f va = {a, a}, vb = {b, b};
#pragma unroll 16
    for (int i = 0; i < ITERS; ++i) {
        x0 = __builtin_elementwise_fma(x0, va, vb); x1 = __builtin_elementwise_fma(x1, va, vb);
        x2 = __builtin_elementwise_fma(x2, va, vb); x3 = __builtin_elementwise_fma(x3, va, vb);
        x4 = __builtin_elementwise_fma(x4, va, vb); x5 = __builtin_elementwise_fma(x5, va, vb);
        x6 = __builtin_elementwise_fma(x6, va, vb); x7 = __builtin_elementwise_fma(x7, va, vb);
    }
    const v2f s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

int main() {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    for (int wps : {1, 2, 4, 8}) {   // waves per SIMD (4 SIMDs per CU, 4 waves per block)
        const int blocks = cus * wps;
        float* out = nullptr;
        if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
        for (int pk = 0; pk < 2; ++pk) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            float ms = 0.f;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (pk)
                    k_pk_fma<<<blocks, 256>>>(out, 0.999f, 0.001f);
                else
                    k_fma<<<blocks, 256>>>(out, 0.999f, 0.001f);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms, e0, e1);
            }
            const double waves = (double)blocks * 4, instr = waves * ITERS * 8;
            const double flops = instr * 64 * 2 * (pk ? 2 : 1);
            printf("{\"cus\": %d, \"waves_per_simd\": %d, \"packed\": %d, \"us\": %.1f, \"G_wave_instr_per_s\": %.1f, "
                   "\"TFLOPs\": %.1f}\n",
                   cus, wps, pk, ms * 1e3, instr / (ms * 1e-3) / 1e9, flops / (ms * 1e-3) / 1e12);
            hipEventDestroy(e0);
            hipEventDestroy(e1);
        }
        hipFree(out);
    }
    return 0;
}
