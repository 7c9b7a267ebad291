// Experiment (not product): can bucketing reads by code make H3's mark + assign cheaper?
//  S  hipcub SortPairs (code -> row) on the top 9 bits only (one pass, stable)
//  M  mark from buckets: one block per 2^15-code bucket, LDS bitmap -> bitmap words
//  A  assign from buckets: LDS copy of the bucket's label slice (128 KB), out[row] = label
//  B  baseline assign: out[i] = labelcode[code[i]] (64 MB table, random gather)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr uint32_t NB = 1u << 24;
constexpr int BBITS = 9;                       // buckets
constexpr uint32_t BCODES = NB >> BBITS;       // 32768 codes per bucket

__global__ void iota(uint32_t* v, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

// bucket starts from the sorted keys
__global__ void bucket_bounds(const uint32_t* k, int64_t n, uint32_t* start) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t b = k[i] >> (24 - BBITS);
    if (i == 0 || (k[i - 1] >> (24 - BBITS)) != b) start[b] = (uint32_t)i;
    if (i == n - 1) start[1 << BBITS] = (uint32_t)n;
}

__global__ __launch_bounds__(1024) void mark_b(const uint32_t* k, const uint32_t* start, uint64_t* bitmap) {
    __shared__ uint32_t bm[BCODES / 32];
    const uint32_t b = blockIdx.x;
    for (int i = threadIdx.x; i < (int)(BCODES / 32); i += 1024) bm[i] = 0;
    __syncthreads();
    for (uint32_t i = start[b] + threadIdx.x; i < start[b + 1]; i += 1024) {
        const uint32_t c = k[i] & (BCODES - 1);
        atomicOr(&bm[c >> 5], 1u << (c & 31));
    }
    __syncthreads();
    uint64_t* out = bitmap + (uint64_t)b * (BCODES / 64);
    for (int i = threadIdx.x; i < (int)(BCODES / 64); i += 1024) out[i] = (uint64_t)bm[2 * i] | ((uint64_t)bm[2 * i + 1] << 32);
}

__global__ __launch_bounds__(1024) void assign_b(const uint32_t* k, const uint32_t* rows, const uint32_t* start,
                                                 const uint32_t* labelcode, uint32_t* out) {
    __shared__ uint32_t lab[BCODES];  // 128 KB
    const uint32_t b = blockIdx.x;
    const uint4* src = reinterpret_cast<const uint4*>(labelcode + (uint64_t)b * BCODES);
    for (int i = threadIdx.x; i < (int)(BCODES / 4); i += 1024) reinterpret_cast<uint4*>(lab)[i] = src[i];
    __syncthreads();
    for (uint32_t i = start[b] + threadIdx.x; i < start[b + 1]; i += 1024) out[rows[i]] = lab[k[i] & (BCODES - 1)];
}

__global__ void assign_base(const uint32_t* codes, int64_t n, const uint32_t* labelcode, uint32_t* out) {
    int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i + 4 > n) return;
    const uint4 v = *reinterpret_cast<const uint4*>(codes + i);
    *reinterpret_cast<uint4*>(out + i) = make_uint4(labelcode[v.x], labelcode[v.y], labelcode[v.z], labelcode[v.w]);
}

int main() {
    const int64_t n = 10000000;
    std::vector<uint32_t> h(n);
    std::mt19937_64 r(7);
    const uint64_t M = n / 10;
    std::vector<uint32_t> parent(M);
    for (auto& p : parent) p = r() & (NB - 1);
    for (int64_t i = 0; i < n; ++i) h[i] = parent[r() % M];
    uint32_t *codes, *rows, *k2, *r2, *start, *lab, *out;
    uint64_t* bitmap;
    CK(hipMalloc(&codes, n * 4));
    CK(hipMalloc(&rows, n * 4));
    CK(hipMalloc(&k2, n * 4));
    CK(hipMalloc(&r2, n * 4));
    CK(hipMalloc(&start, ((1 << BBITS) + 1) * 4));
    CK(hipMalloc(&lab, (size_t)NB * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&bitmap, NB / 8));
    CK(hipMemcpy(codes, h.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(lab, 1, (size_t)NB * 4));
    hipLaunchKernelGGL(iota, dim3((n + 255) / 256), dim3(256), 0, 0, rows, n);
    size_t tb = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, codes, k2, rows, r2, (int)n, 24 - BBITS, 24));
    void* tmp;
    CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char* name, auto fn) {
        float best = 1e9;
        for (int it = 0; it < 6; ++it) {
            CK(hipDeviceSynchronize());
            hipEventRecord(a);
            fn();
            hipEventRecord(b);
            CK(hipEventSynchronize(b));
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        printf("%-28s %8.1f us\n", name, best * 1000);
    };
    timeit("S sort 9-bit (code,row)", [&] {
        hipcub::DeviceRadixSort::SortPairs(tmp, tb, codes, k2, rows, r2, (int)n, 24 - BBITS, 24);
    });
    timeit("  bucket bounds", [&] { hipLaunchKernelGGL(bucket_bounds, dim3((n + 255) / 256), dim3(256), 0, 0, k2, n, start); });
    timeit("M mark from buckets", [&] { hipLaunchKernelGGL(mark_b, dim3(1 << BBITS), dim3(1024), 0, 0, k2, start, bitmap); });
    timeit("A assign from buckets", [&] {
        hipLaunchKernelGGL(assign_b, dim3(1 << BBITS), dim3(1024), 0, 0, k2, r2, start, lab, out);
    });
    timeit("B baseline assign", [&] {
        hipLaunchKernelGGL(assign_base, dim3((n / 4 + 255) / 256), dim3(256), 0, 0, codes, n, lab, out);
    });
    return 0;
}
