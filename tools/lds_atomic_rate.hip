// Experiment (round 6): LDS operation rates for a wave-private 8 KB hash table, the shape of
// k_kmer_wave's inserts. Each wave owns 1024 u64 slots and issues ITERS operations per lane at
// pseudo-random slots; printed: lane-operations per CU clock for each form.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_rate.hip -o tools/lds_atomic_rate
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kSlots = 1024;
constexpr int kWG = 2;  // waves per workgroup
constexpr int ITERS = 4096;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(64 * kWG) void k_rate(unsigned long long* out) {
    __shared__ unsigned long long T[kWG][kSlots];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long* t = T[wv];
    for (int i = lane; i < kSlots; i += 64) t[i] = ~0ull;
    __builtin_amdgcn_wave_barrier();
    uint32_t s = mix(blockIdx.x * 131 + threadIdx.x * 7 + 1);
    unsigned long long acc = 0;
    for (int it = 0; it < ITERS; ++it) {
        s = s * 1664525u + 1013904223u;
        const uint32_t h = (s >> 12) & (kSlots - 1);
        const unsigned long long key = (unsigned long long)(s >> 20) << 32 | 0x100;
        if (MODE == 0) {  // returning 64-bit CAS (claim or find), dependent chain
            const unsigned long long v = atomicCAS(&t[h], ~0ull, key);
            acc += v;
            s ^= (uint32_t)v;  // dependency on the returned value
        } else if (MODE == 1) {  // non-returning 64-bit add
            atomicAdd(&t[h], 0x100ull);
        } else if (MODE == 2) {  // plain read + write (read-modify-write, not atomic)
            const unsigned long long v = t[h];
            t[h] = v + 0x100;
            s ^= (uint32_t)v;
        } else if (MODE == 3) {  // returning 32-bit add
            const uint32_t v = atomicAdd(reinterpret_cast<uint32_t*>(&t[h]), 1u);
            s ^= v;
        } else if (MODE == 4) {  // independent returning CAS: 4 per trip, no dependency between them
            unsigned long long v0 = atomicCAS(&t[h], ~0ull, key);
            unsigned long long v1 = atomicCAS(&t[(h + 257) & (kSlots - 1)], ~0ull, key);
            unsigned long long v2 = atomicCAS(&t[(h + 513) & (kSlots - 1)], ~0ull, key);
            unsigned long long v3 = atomicCAS(&t[(h + 771) & (kSlots - 1)], ~0ull, key);
            acc += v0 + v1 + v2 + v3;
            s ^= (uint32_t)(v0 ^ v1 ^ v2 ^ v3);
        } else if (MODE == 5) {  // plain dependent read only
            const unsigned long long v = t[h];
            s ^= (uint32_t)v;
            acc += v;
        }
    }
    if (acc == 12345) out[0] = acc;
}

template <int MODE>
float run(int blocks, unsigned long long* out) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_rate<MODE><<<blocks, 64 * kWG>>>(out);
    hipEventRecord(a);
    k_rate<MODE><<<blocks, 64 * kWG>>>(out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    unsigned long long* out;
    hipMalloc(&out, 64);
    const char* names[] = {"CAS rtn b64 (dependent)", "add b64 no-rtn", "read+write b64", "add rtn u32 (dependent)",
                           "4 independent CAS rtn b64", "read b64 (dependent)"};
    for (int wpc : {4, 8, 12, 16}) {  // waves per CU
        const int blocks = 256 * wpc / kWG;
        float ms[6] = {run<0>(blocks, out), run<1>(blocks, out), run<2>(blocks, out), run<3>(blocks, out),
                       run<4>(blocks, out), run<5>(blocks, out)};
        for (int m = 0; m < 6; ++m) {
            const double ops = (double)blocks * 64 * kWG * ITERS * (m == 4 ? 4 : 1);
            printf("waves/CU %2d  %-28s %8.3f ms  %6.2f lane-ops per CU clock\n", wpc, names[m], ms[m],
                   ops / 256.0 / (ms[m] * 1e-3 * 2.4e9));
        }
    }
    return 0;
}
