// Experiment (not product): where does the XCD-partitioned presence mark spend its time?
//  A  partitioned by blockIdx % 8, reads + partition test only (no stores)
//  B  partitioned by blockIdx % 8 + byte stores (the product kernel's scheme)
//  C  partitioned by the hardware XCC id (timing only: coverage not exact) + byte stores
//  D  unpartitioned, uint4 loads + byte stores
//  E  B with 16 partitions (two per XCD)
//  F  B with non-temporal code loads;  G  F with non-temporal byte stores;  H  A with nt loads
// Also prints the blockIdx % 8 -> XCC id histogram.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr uint32_t NB = 1u << 24;

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v & 7u;
}

template <int MODE, int PARTS, bool NT = false>
__global__ __launch_bounds__(256) void mark(const uint32_t* __restrict__ codes, int64_t n, int64_t chunk,
                                            uint8_t* __restrict__ pres, uint32_t* cnt) {
    const uint32_t part = MODE == 2 ? xcc_id() : blockIdx.x % PARTS;
    const int64_t c0 = (int64_t)(blockIdx.x / PARTS) * chunk;
    const int64_t c1 = c0 + chunk < n ? c0 + chunk : n;
    uint32_t hits = 0;
    for (int64_t r = c0 + 4 * (int64_t)threadIdx.x; r < c1; r += 4 * 256) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        u32x4 v;
        if (NT) v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(codes + r));
        else v = *reinterpret_cast<const u32x4*>(codes + r);
        const uint32_t c[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (MODE == 3 || (uint32_t)(((uint64_t)c[k] * PARTS) >> 24) == part) {
                if (MODE == 0) hits++;
                else if (MODE == 4) __builtin_nontemporal_store((uint8_t)1, pres + c[k]);
                else pres[c[k]] = 1;
            }
        }
    }
    if (MODE == 0 && hits == 0xFFFFFFFFu) cnt[0] = hits;
}

__global__ void census(uint32_t* hist) {
    if (threadIdx.x == 0) atomicAdd(hist + (blockIdx.x % 8) * 8 + xcc_id(), 1u);
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 10000000;
    std::vector<uint32_t> h(n);
    std::mt19937_64 r(7);
    const uint64_t M = n / 10;
    std::vector<uint32_t> parent(M);
    for (auto& p : parent) p = r() & (NB - 1);
    for (int64_t i = 0; i < n; ++i) h[i] = parent[r() % M];
    uint32_t *dc, *cnt, *hist;
    uint8_t* pres;
    CK(hipMalloc(&dc, n * 4 + 4096));
    CK(hipMalloc(&pres, NB));
    CK(hipMalloc(&cnt, 64));
    CK(hipMalloc(&hist, 256));
    CK(hipMemcpy(dc, h.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(hist, 0, 256));
    hipLaunchKernelGGL(census, dim3(2048), dim3(64), 0, 0, hist);
    uint32_t hh[64];
    CK(hipMemcpy(hh, hist, 256, hipMemcpyDeviceToHost));
    printf("blockIdx%%8 -> xcc histogram:\n");
    for (int b = 0; b < 8; ++b) {
        for (int x = 0; x < 8; ++x) printf(" %4u", hh[b * 8 + x]);
        printf("\n");
    }
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int chunks : {64, 256, 1024}) {
        int64_t chunk = (n + chunks - 1) / chunks;
        chunk = (chunk + 1023) / 1024 * 1024;
        const int64_t nch = (n + chunk - 1) / chunk;
        for (int v = 0; v < 8; ++v) {
            float best = 1e9;
            for (int it = 0; it < 8; ++it) {
                CK(hipMemset(pres, 0, NB));
                CK(hipDeviceSynchronize());
                hipEventRecord(a);
                if (v == 0) hipLaunchKernelGGL((mark<0, 8>), dim3(nch * 8), dim3(256), 0, 0, dc, n, chunk, pres, cnt);
                if (v == 1) hipLaunchKernelGGL((mark<1, 8>), dim3(nch * 8), dim3(256), 0, 0, dc, n, chunk, pres, cnt);
                if (v == 2) hipLaunchKernelGGL((mark<2, 8>), dim3(nch * 8), dim3(256), 0, 0, dc, n, chunk, pres, cnt);
                if (v == 3) hipLaunchKernelGGL((mark<3, 1>), dim3(nch), dim3(256), 0, 0, dc, n, chunk, pres, cnt);
                if (v == 4) hipLaunchKernelGGL((mark<1, 16>), dim3(nch * 16), dim3(256), 0, 0, dc, n, chunk, pres, cnt);
                if (v == 5) hipLaunchKernelGGL((mark<1, 8, true>), dim3(nch * 8), dim3(256), 0, 0, dc, n, chunk, pres, cnt);
                if (v == 6) hipLaunchKernelGGL((mark<4, 8, true>), dim3(nch * 8), dim3(256), 0, 0, dc, n, chunk, pres, cnt);
                if (v == 7) hipLaunchKernelGGL((mark<0, 8, true>), dim3(nch * 8), dim3(256), 0, 0, dc, n, chunk, pres, cnt);
                hipEventRecord(b);
                CK(hipEventSynchronize(b));
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            printf("chunks %4d variant %c: %.1f us\n", chunks, "ABCDEFGH"[v], best * 1000);
        }
    }
    return 0;
}
