// Experiment (not product): presence-marking variants for 10M 24-bit codes.
//  V0 byte stores into a 16 MB byte table (current)
//  V1 agent-scope atomicOr into one 2 MB bitmap
//  V2 workgroup-scope atomicOr into a per-XCD 2 MB bitmap (8 copies, s_getreg XCC_ID)
//  V3 like V2 but agent-scope atomics
// Reports time per variant and checks the merged bitmap against the host truth.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr uint32_t NB = 1u << 24;  // 4^12 codes
constexpr uint32_t WORDS32 = NB / 32;

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v & 7u;
}

__global__ void v0(const uint32_t* c, int64_t n, uint8_t* pres) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) pres[c[i]] = 1;
}
__global__ void v1(const uint32_t* c, int64_t n, uint32_t* bm) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) __hip_atomic_fetch_or(bm + (c[i] >> 5), 1u << (c[i] & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int SCOPE>
__global__ void v2(const uint32_t* c, int64_t n, uint32_t* bm8) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t* bm = bm8 + (size_t)xcc_id() * WORDS32;
    if (i < n) __hip_atomic_fetch_or(bm + (c[i] >> 5), 1u << (c[i] & 31), __ATOMIC_RELAXED, SCOPE);
}
__global__ void merge8(const uint32_t* bm8, uint32_t* out) {
    int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= WORDS32) return;
    uint32_t v = 0;
    for (int x = 0; x < 8; ++x) v |= bm8[(size_t)x * WORDS32 + w];
    out[w] = v;
}
__global__ void bytes_to_bits(const uint8_t* pres, uint32_t* out) {
    int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= WORDS32) return;
    uint32_t v = 0;
    for (int b = 0; b < 32; ++b) v |= (pres[w * 32 + b] ? 1u : 0u) << b;
    out[w] = v;
}
__global__ void xcc_census(uint32_t* hist) {
    if (threadIdx.x == 0) atomicAdd(hist + xcc_id(), 1u);
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 10000000;
    const int only = argc > 2 ? atoi(argv[2]) : -1;
    std::vector<uint32_t> h(n);
    std::mt19937_64 r(7);
    const uint64_t M = n / 10;
    std::vector<uint32_t> parent(M);
    for (auto& p : parent) p = r() & (NB - 1);
    for (int64_t i = 0; i < n; ++i) {
        uint32_t c = parent[r() % M];
        if ((r() % 1000) == 0) c ^= 1u << (2 * (r() % 12));
        h[i] = c;
    }
    std::vector<uint32_t> truth(WORDS32, 0);
    for (auto c : h) truth[c >> 5] |= 1u << (c & 31);
    uint32_t *dc, *bm, *bm8, *out, *hist;
    uint8_t* pres;
    CK(hipMalloc(&dc, n * 4));
    CK(hipMalloc(&bm, WORDS32 * 4));
    CK(hipMalloc(&bm8, 8ull * WORDS32 * 4));
    CK(hipMalloc(&out, WORDS32 * 4));
    CK(hipMalloc(&pres, NB));
    CK(hipMalloc(&hist, 64));
    CK(hipMemcpy(dc, h.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(hist, 0, 64));
    hipLaunchKernelGGL(xcc_census, dim3(4096), dim3(64), 0, 0, hist);
    uint32_t hh[8];
    CK(hipMemcpy(hh, hist, 32, hipMemcpyDeviceToHost));
    printf("xcc census:");
    for (int x = 0; x < 8; ++x) printf(" %u", hh[x]);
    printf("\n");
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const dim3 g((unsigned)((n + 255) / 256)), blk(256), gw((WORDS32 + 255) / 256);
    std::vector<uint32_t> got(WORDS32);
    for (int v = 0; v < 4; ++v) {
        if (only >= 0 && v != only) continue;
        float best = 1e9;
        for (int it = 0; it < 6; ++it) {
            CK(hipMemset(pres, 0, NB));
            CK(hipMemset(bm, 0, WORDS32 * 4));
            CK(hipMemset(bm8, 0, 8ull * WORDS32 * 4));
            CK(hipDeviceSynchronize());
            hipEventRecord(a);
            if (v == 0) { hipLaunchKernelGGL(v0, g, blk, 0, 0, dc, n, pres); hipLaunchKernelGGL(bytes_to_bits, gw, blk, 0, 0, pres, out); }
            if (v == 1) { hipLaunchKernelGGL(v1, g, blk, 0, 0, dc, n, bm); }
            if (v == 2) { hipLaunchKernelGGL(v2<__HIP_MEMORY_SCOPE_WORKGROUP>, g, blk, 0, 0, dc, n, bm8); hipLaunchKernelGGL(merge8, gw, blk, 0, 0, bm8, out); }
            if (v == 3) { hipLaunchKernelGGL(v2<__HIP_MEMORY_SCOPE_AGENT>, g, blk, 0, 0, dc, n, bm8); hipLaunchKernelGGL(merge8, gw, blk, 0, 0, bm8, out); }
            hipEventRecord(b);
            CK(hipEventSynchronize(b));
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
            CK(hipMemcpy(got.data(), v == 1 ? bm : out, WORDS32 * 4, hipMemcpyDeviceToHost));
            int64_t bad = 0;
            for (uint32_t w = 0; w < WORDS32; ++w) bad += got[w] != truth[w];
            if (bad) printf("  V%d iter %d: %lld words differ\n", v, it, (long long)bad);
        }
        printf("V%d best %.1f us\n", v, best * 1000);
    }
    return 0;
}
