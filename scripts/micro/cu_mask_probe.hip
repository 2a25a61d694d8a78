// Which CUs a stream CU mask bit enables on MI355X (gfx950): for a few single-bit masks (hipExtStreamCreateWithCUMask,
// 8 words = 256 CUs), every workgroup of a small launch records its XCC id and HW_ID (SE, SH, CU fields); the host
// prints the distinct placements per bit. Informs the comm-stream CU reservation experiment.
//   hipcc --offload-arch=gfx950 -O2 cu_mask_probe.hip -o cu_mask_probe && ./cu_mask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void k_where(uint32_t* out) {
    // s_getreg simm16: size - 1 in [15:11], offset in [10:6], register id in [5:0]
    const uint32_t xcc = __builtin_amdgcn_s_getreg((20u) | (0u << 6) | (15u << 11));   // HW_REG_XCC_ID
    const uint32_t hw = __builtin_amdgcn_s_getreg((4u) | (0u << 6) | (31u << 11));     // HW_REG_HW_ID
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
}

int main() {
    const int nb = 512;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, 2 * nb * sizeof(uint32_t)) != hipSuccess) return 1;
    std::vector<uint32_t> h(2 * nb);
    const int bits[] = {0, 1, 2, 3, 7, 8, 15, 31, 32, 33, 63, 64, 128, 255, -1};
    for (int b : bits) {
        uint32_t mask[8];
        for (int w = 0; w < 8; ++w) mask[w] = b < 0 ? 0xffffffffu : 0u;
        if (b >= 0) mask[b / 32] = 1u << (b % 32);
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, 8, mask) != hipSuccess) { printf("bit %d: create failed\n", b); continue; }
        hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s, d);
        if (hipStreamSynchronize(s) != hipSuccess) { printf("bit %d: run failed\n", b); return 2; }
        hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
        std::set<std::tuple<int, int, int, int>> where;   // xcc, se, sh, cu
        for (int i = 0; i < nb; ++i) {
            const uint32_t hw = h[2 * i + 1];
            where.insert({(int)(h[2 * i] & 0xf), (int)((hw >> 13) & 7), (int)((hw >> 12) & 1), (int)((hw >> 8) & 0xf)});
        }
        printf("bit %4d: %zu placements:", b, where.size());
        int k = 0;
        for (auto& t : where) {
            if (k++ < 12) printf(" (x%d se%d sh%d cu%d)", std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t));
        }
        printf("\n");
        hipStreamDestroy(s);
    }
    hipFree(d);
    return 0;
}
