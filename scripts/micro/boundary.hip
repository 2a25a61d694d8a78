// Back-to-back dependent launches on one stream: wall time per launch for kernel shapes like the small-N step's
// (grid size, static LDS, kernarg size, a store into host-mapped memory). Measurement tool, not product code.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Big { uint32_t w[120]; };   // 480-byte kernarg

__global__ void k_empty(uint32_t* p) { if (p && blockIdx.x == 0 && threadIdx.x == 0) p[1] = 1u; }
__global__ void k_lds(uint32_t* p) {
    __shared__ uint32_t s[36864];   // 144 KB
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (p && blockIdx.x == 0 && threadIdx.x == 0) p[1] = s[5];
}
__global__ void k_big(Big b, uint32_t* p) { if (p && blockIdx.x == 0 && threadIdx.x == 0) p[1] = b.w[7]; }
__global__ void k_store(uint32_t* p, int n) {   // each thread stores one word
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (uint32_t)i;
}

template <typename F>
double per_launch(const char* name, int reps, F launch, hipStream_t s) {
    for (int i = 0; i < 50; ++i) launch();
    (void)hipStreamSynchronize(s);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) launch();
    const auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(s);
    const auto t2 = std::chrono::steady_clock::now();
    const double host = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
    const double wall = std::chrono::duration<double, std::micro>(t2 - t0).count() / reps;
    printf("{\"case\": \"%s\", \"us_per_launch\": %.2f, \"host_us_per_launch\": %.2f}\n", name, wall, host);
    fflush(stdout);
    return wall;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *d = nullptr, *hm = nullptr, *hmd = nullptr;
    CK(hipMalloc(&d, 64 << 20));
    CK(hipHostMalloc(&hm, 4096, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)&hmd, hm, 0));
    const int R = 2000;
    Big b;
    memset(&b, 0, sizeof b);
    per_launch("empty 1 WG", R, [&] { k_empty<<<1, 256, 0, s>>>(d); }, s);
    per_launch("empty 16 WG", R, [&] { k_empty<<<16, 256, 0, s>>>(d); }, s);
    per_launch("empty 256 WG", R, [&] { k_empty<<<256, 256, 0, s>>>(d); }, s);
    per_launch("empty 1024 WG", R, [&] { k_empty<<<1024, 256, 0, s>>>(d); }, s);
    per_launch("empty 4096 WG", R, [&] { k_empty<<<4096, 256, 0, s>>>(d); }, s);
    per_launch("lds144k 16 WG", R, [&] { k_lds<<<16, 256, 0, s>>>(d); }, s);
    per_launch("lds144k 256 WG", R, [&] { k_lds<<<256, 256, 0, s>>>(d); }, s);
    per_launch("kernarg480 1024 WG", R, [&] { k_big<<<1024, 256, 0, s>>>(b, d); }, s);
    per_launch("host-mapped store 1 WG", R, [&] { k_empty<<<1, 256, 0, s>>>(hmd); }, s);
    per_launch("host-mapped store 256 WG", R, [&] { k_empty<<<256, 256, 0, s>>>(hmd); }, s);
    per_launch("store 400KB 400 WG", R, [&] { k_store<<<400, 256, 0, s>>>(d, 102400); }, s);
    per_launch("store 4MB 4096 WG", R, [&] { k_store<<<4096, 256, 0, s>>>(d, 1 << 20); }, s);
    // alternating pairs: empty then host-mapped (one boundary each)
    per_launch("pair empty+mapped 256 WG (per pair)", R, [&] { k_empty<<<256, 256, 0, s>>>(d); k_empty<<<256, 256, 0, s>>>(hmd); }, s);
    CK(hipStreamDestroy(s));
    return 0;
}
