// valu_peak.hip — measures the chip's VALU issue rate and the shader clock it holds meanwhile
// (profiling only, not part of the product).
// Every lane runs 8 independent f32 FMA chains (or packed-f32 pk_fma chains) for `iters` steps,
// at 1, 2, 4 and 8 waves per SIMD. Prints wave-instructions per second (the peak bench.py's
// roofline.valu divides by) and, from in-kernel stamps (first wave of every workgroup:
// Δs_memtime ÷ Δs_memrealtime × 100 MHz, median over workgroups; MI355X_MICROARCH.md DVFS item 6),
// the clock during the loop, so the rate can be priced against the spec issue rate at that clock:
// 256 CUs × 4 SIMDs × ½ wave64-instruction per cycle (a wave64 f32 VALU op takes 2 cycles).
//   hipcc -O3 --offload-arch=gfx950 scripts/valu_peak.hip -o scripts/valu_peak.bin
//   scripts/valu_peak.bin [iters]      (default 4096; 65536 gives ~5 ms dispatches at 8 waves/SIMD)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ void stamp(unsigned long long* clk, int slot) {
    if (threadIdx.x == 0) {
        clk[4 * blockIdx.x + 2 * slot] = __builtin_amdgcn_s_memtime();
        clk[4 * blockIdx.x + 2 * slot + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

__global__ __launch_bounds__(256) void k_fma(float* out, float a, float b, int iters, unsigned long long* clk) {
    stamp(clk, 0);
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
#pragma unroll 16
    for (int i = 0; i < iters; ++i) {
        x0 = fmaf(x0, a, b); x1 = fmaf(x1, a, b); x2 = fmaf(x2, a, b); x3 = fmaf(x3, a, b);
        x4 = fmaf(x4, a, b); x5 = fmaf(x5, a, b); x6 = fmaf(x6, a, b); x7 = fmaf(x7, a, b);
    }
    out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    stamp(clk, 1);
}

typedef float v2f __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_pk_fma(float* out, float a, float b, int iters, unsigned long long* clk) {
    stamp(clk, 0);
    v2f x0 = {(float)threadIdx.x, 1.f}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
        x6 = x0 + 6, x7 = x0 + 7;
    const v2f va = {a, a}, vb = {b, b};
#pragma unroll 16
    for (int i = 0; i < iters; ++i) {
        x0 = __builtin_elementwise_fma(x0, va, vb); x1 = __builtin_elementwise_fma(x1, va, vb);
        x2 = __builtin_elementwise_fma(x2, va, vb); x3 = __builtin_elementwise_fma(x3, va, vb);
        x4 = __builtin_elementwise_fma(x4, va, vb); x5 = __builtin_elementwise_fma(x5, va, vb);
        x6 = __builtin_elementwise_fma(x6, va, vb); x7 = __builtin_elementwise_fma(x7, va, vb);
    }
    const v2f s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
    stamp(clk, 1);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 4096;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    for (int wps : {1, 2, 4, 8}) {   // waves per SIMD (4 SIMDs per CU, 4 waves per block)
        const int blocks = cus * wps;
        float* out = nullptr;
        unsigned long long* clk = nullptr;
        if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
        if (hipMalloc(&clk, (size_t)blocks * 4 * 8) != hipSuccess) return 1;
        for (int pk = 0; pk < 2; ++pk) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            float ms = 0.f;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (pk)
                    k_pk_fma<<<blocks, 256>>>(out, 0.999f, 0.001f, iters, clk);
                else
                    k_fma<<<blocks, 256>>>(out, 0.999f, 0.001f, iters, clk);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms, e0, e1);
            }
            std::vector<unsigned long long> h((size_t)blocks * 4);
            hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
            std::vector<double> ghz;
            for (int b = 0; b < blocks; ++b) {
                const double dc = (double)(h[4 * b + 2] - h[4 * b]), dr = (double)(h[4 * b + 3] - h[4 * b + 1]);
                if (dr > 0) ghz.push_back(dc / dr * 0.1);   // s_memrealtime ticks at 100 MHz
            }
            std::sort(ghz.begin(), ghz.end());
            const double clock = ghz.empty() ? 0.0 : ghz[ghz.size() / 2];
            const double waves = (double)blocks * 4, instr = waves * (double)iters * 8;
            const double flops = instr * 64 * 2 * (pk ? 2 : 1);
            const double rate = instr / (ms * 1e-3);
            const double spec_at_clock = (double)cus * 4 * 0.5 * clock * 1e9;   // wave-instr/s
            printf("{\"cus\": %d, \"waves_per_simd\": %d, \"packed\": %d, \"iters\": %d, \"us\": %.1f, "
                   "\"G_wave_instr_per_s\": %.1f, \"TFLOPs\": %.1f, \"clock_ghz_median\": %.3f, "
                   "\"frac_of_spec_issue_at_clock\": %.3f}\n",
                   cus, wps, pk, iters, ms * 1e3, rate / 1e9, flops / (ms * 1e-3) / 1e12, clock,
                   spec_at_clock > 0 ? rate / spec_at_clock : 0.0);
            hipEventDestroy(e0);
            hipEventDestroy(e1);
        }
        hipFree(out);
        hipFree(clk);
    }
    return 0;
}
