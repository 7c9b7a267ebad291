// Experiment (not product): random 4-byte gather rate vs table size on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <random>
#include <vector>
__global__ void gather4(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ tab, int64_t n, uint32_t* __restrict__ out) {
    int64_t r0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (r0 + 4 > n) return;
    uint4 c = *reinterpret_cast<const uint4*>(idx + r0);
    uint4 o = make_uint4(tab[c.x], tab[c.y], tab[c.z], tab[c.w]);
    *reinterpret_cast<uint4*>(out + r0) = o;
}
int main() {
    const int64_t n = 10000000;
    std::vector<uint32_t> h(n);
    uint32_t *di, *dt, *dout;
    hipMalloc(&di, n * 4); hipMalloc(&dout, n * 4); hipMalloc(&dt, 1ull << 30);
    hipMemset(dt, 1, 1ull << 30);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    std::mt19937_64 r(1);
    for (int lg : {20, 22, 24, 26, 28}) {  // table entries: 1M (4MB) .. 256M (1GB)
        const uint32_t mask = (1u << lg) - 1;
        for (auto& x : h) x = r() & mask;
        hipMemcpy(di, h.data(), n * 4, hipMemcpyHostToDevice);
        float best = 1e9;
        for (int it = 0; it < 5; ++it) {
            hipEventRecord(a);
            hipLaunchKernelGGL(gather4, dim3((n / 4 + 255) / 256), dim3(256), 0, 0, di, dt, n, dout);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); best = ms < best ? ms : best;
        }
        printf("table %5lld MB: %.1f us  -> %.1f G gathers/s\n", (4ll << lg) >> 20, best * 1000, n / (best * 1e-3) / 1e9);
    }
    return 0;
}
