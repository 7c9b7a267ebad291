// Experiment (not product): cost of a phase boundary on gfx950 — K dependent kernel
// launches on one stream vs one persistent kernel whose K phases are separated by grid
// barriers (device-scope counter + generation word; variants with / without the
// agent-scope fences that make the phases' global writes visible across XCDs).
// Each phase: every thread reads one u32 written by another workgroup in the previous
// phase (so the fences matter) and writes one. Prints us per phase boundary.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                        \
        }                                                                    \
    } while (0)

constexpr int kT = 256;

__global__ __launch_bounds__(kT) void k_phase(uint32_t* a, int phase, int n) {
    const int i = blockIdx.x * kT + threadIdx.x;
    const int j = (i + 7919 * kT) % n;  // another workgroup's element
    a[i + ((phase + 1) & 1) * n] = a[j + (phase & 1) * n] + 1;
}

// mode 0: fences (release before arrive, acquire after); 1: no fences; 2: per-XCD
// counters (blockIdx % 8), then one XCD leader per group arrives globally, with fences
__device__ __forceinline__ bool grid_barrier(unsigned* bar, unsigned nblocks, int mode, unsigned* err) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        unsigned* count = bar;
        unsigned* gen = bar + 64;
        const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (mode != 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        bool last;
        if (mode == 2) {
            const unsigned x = blockIdx.x & 7u;
            const unsigned per = (nblocks - x + 7u) / 8u;  // blocks of this XCD group
            unsigned* xc = bar + 128 + 64 * x;
            const unsigned a = __hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = false;
            if (a == per - 1) {
                __hip_atomic_store(xc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned groups = nblocks < 8 ? nblocks : 8u;
                last = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1;
            }
        } else {
            last = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblocks - 1;
        }
        if (last) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            int polls = 0;
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (++polls > (1 << 22)) {
                    atomicAdd(err, 1u);
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (mode != 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return ok;
}

__global__ __launch_bounds__(kT) void k_persistent(uint32_t* a, int phases, int n, unsigned* bar, int mode,
                                                   unsigned* err) {
    const int i = blockIdx.x * kT + threadIdx.x;
    const int j = (i + 7919 * kT) % n;
    for (int ph = 0; ph < phases; ++ph) {
        a[i + ((ph + 1) & 1) * n] = a[j + (ph & 1) * n] + 1;
        if (ph + 1 < phases && !grid_barrier(bar, gridDim.x, mode, err)) return;
    }
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int K = 64;
    for (int blocks : {256, 512, 1024}) {
        const int n = blocks * kT;
        uint32_t* a;
        unsigned *bar, *err;
        CK(hipMalloc(&a, 2 * n * 4));
        CK(hipMalloc(&bar, 4096 * 4));
        CK(hipMalloc(&err, 4));
        CK(hipMemset(a, 0, 2 * n * 4));
        CK(hipMemset(bar, 0, 4096 * 4));
        CK(hipMemset(err, 0, 4));
        // launches
        float best_l = 1e30f;
        for (int it = 0; it < 5; ++it) {
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_phase, dim3(blocks), dim3(kT), 0, s, a, k, n);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best_l = std::min(best_l, ms);
        }
        uint32_t chk_l;
        CK(hipMemcpy(&chk_l, a + ((K) & 1) * n, 4, hipMemcpyDeviceToHost));
        printf("blocks %5d  %d launches: %7.2f us per phase (value %u)\n", blocks, K, 1000.f * best_l / K, chk_l);
        for (int mode = 0; mode < 3; ++mode) {
            float best = 1e30f;
            for (int it = 0; it < 5; ++it) {
                CK(hipMemset(a, 0, 2 * n * 4));
                CK(hipEventRecord(e0, s));
                hipLaunchKernelGGL(k_persistent, dim3(blocks), dim3(kT), 0, s, a, K, n, bar, mode, err);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms);
            }
            unsigned herr;
            uint32_t chk;
            CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&chk, a + ((K) & 1) * n, 4, hipMemcpyDeviceToHost));
            printf("blocks %5d  persistent %d phases, barrier mode %d (%s): %7.2f us per phase (value %u, err %u)\n",
                   blocks, K, mode, mode == 0 ? "fences" : mode == 1 ? "no fences" : "per-XCD + fences",
                   1000.f * best / K, chk, herr);
        }
        CK(hipFree(a));
        CK(hipFree(bar));
        CK(hipFree(err));
    }
    return 0;
}
