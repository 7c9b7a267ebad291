// Experiment (not product code): HBM write ceilings for the score kernel's output
// pattern on gfx950. n rows; outputs 6 x f64 + 1 x u32 columns (52 B/row) + 4 B/row read.
//   fill1   one f64 column, 16-B stores (the single-stream write ceiling)
//   cols7   the score kernel's pattern: a wave owns rows {2l, 2l+1, 128+2l, 129+2l} of a
//           256-row tile and writes all 7 columns for them (double2 / uint2 stores)
//   cols7nt same with nontemporal stores
//   colseq  each workgroup writes its 1024 rows column after column, with a barrier
//           between columns (fewer concurrent write streams per workgroup)
// Build: hipcc -O3 --offload-arch=gfx950 tools/store_pattern.hip -o tools/store_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void fill1(double* a, long n) {
    long i = ((long)blockIdx.x * 256 + threadIdx.x) * 2;
    if (i + 1 < n) *reinterpret_cast<f64x2*>(a + i) = f64x2{1.0, 2.0};
}

template <bool NT>
__global__ __launch_bounds__(256) void cols7(const unsigned* codes, double* o0, double* o1, double* o2, double* o3,
                                            double* o4, double* o5, unsigned* o6, long n) {
    const int lane = threadIdx.x & 63;
    const long base = ((long)blockIdx.x * 256 + (threadIdx.x & ~63)) * 4;
    const long rA = base + 2 * lane, rB = rA + 128;
    if (base + 256 > n) return;
    const u32x2 va = *reinterpret_cast<const u32x2*>(codes + rA);
    const u32x2 vb = *reinterpret_cast<const u32x2*>(codes + rB);
    double* outs[6] = {o0, o1, o2, o3, o4, o5};
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        const f64x2 a{(double)(va.x + c), (double)(va.y + c)}, b{(double)(vb.x + c), (double)(vb.y + c)};
        if (NT) {
            __builtin_nontemporal_store(a, reinterpret_cast<f64x2*>(outs[c] + rA));
            __builtin_nontemporal_store(b, reinterpret_cast<f64x2*>(outs[c] + rB));
        } else {
            *reinterpret_cast<f64x2*>(outs[c] + rA) = a;
            *reinterpret_cast<f64x2*>(outs[c] + rB) = b;
        }
    }
    if (NT) {
        __builtin_nontemporal_store(va, reinterpret_cast<u32x2*>(o6 + rA));
        __builtin_nontemporal_store(vb, reinterpret_cast<u32x2*>(o6 + rB));
    } else {
        *reinterpret_cast<u32x2*>(o6 + rA) = va;
        *reinterpret_cast<u32x2*>(o6 + rB) = vb;
    }
}

// each workgroup: 1024 rows, one column at a time over the whole workgroup (thread t
// writes rows 2t, 2t+1 of the tile as one double2 per column)
__global__ __launch_bounds__(256) void colseq(const unsigned* codes, double* o0, double* o1, double* o2, double* o3,
                                             double* o4, double* o5, unsigned* o6, long n) {
    const long r0 = (long)blockIdx.x * 1024;
    if (r0 + 1024 > n) return;
    const int t = threadIdx.x;
    const u32x2 va = *reinterpret_cast<const u32x2*>(codes + r0 + 2 * t);
    const u32x2 vb = *reinterpret_cast<const u32x2*>(codes + r0 + 512 + 2 * t);
    double* outs[6] = {o0, o1, o2, o3, o4, o5};
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        __builtin_nontemporal_store(f64x2{(double)(va.x + c), (double)(va.y + c)},
                                    reinterpret_cast<f64x2*>(outs[c] + r0 + 2 * t));
        __builtin_nontemporal_store(f64x2{(double)(vb.x + c), (double)(vb.y + c)},
                                    reinterpret_cast<f64x2*>(outs[c] + r0 + 512 + 2 * t));
    }
    __builtin_nontemporal_store(va, reinterpret_cast<u32x2*>(o6 + r0 + 2 * t));
    __builtin_nontemporal_store(vb, reinterpret_cast<u32x2*>(o6 + r0 + 512 + 2 * t));
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 10000000L / 1024 * 1024;
    unsigned *codes, *o6;
    double* o[6];
    CK(hipMalloc(&codes, n * 4));
    CK(hipMemset(codes, 1, n * 4));
    for (int c = 0; c < 6; ++c) CK(hipMalloc(&o[c], n * 8));
    CK(hipMalloc(&o6, n * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(a));
        for (int i = 0; i < it; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = 1000.0 * ms / it;
        printf("%-8s %8.1f us  %7.1f GB/s\n", name, us, bytes / us / 1e3);
    };
    const int g = (int)(n / 1024);
    timeit("fill1", n * 8.0, [&] { hipLaunchKernelGGL(fill1, dim3((n / 2 + 255) / 256), dim3(256), 0, 0, o[0], n); });
    timeit("fill6", n * 48.0, [&] {
        for (int c = 0; c < 6; ++c) hipLaunchKernelGGL(fill1, dim3((n / 2 + 255) / 256), dim3(256), 0, 0, o[c], n);
    });
    timeit("cols7", n * 56.0, [&] {
        hipLaunchKernelGGL(cols7<false>, dim3(g), dim3(256), 0, 0, codes, o[0], o[1], o[2], o[3], o[4], o[5], o6, n);
    });
    timeit("cols7nt", n * 56.0, [&] {
        hipLaunchKernelGGL(cols7<true>, dim3(g), dim3(256), 0, 0, codes, o[0], o[1], o[2], o[3], o[4], o[5], o6, n);
    });
    timeit("colseq", n * 56.0, [&] {
        hipLaunchKernelGGL(colseq, dim3(g), dim3(256), 0, 0, codes, o[0], o[1], o[2], o[3], o[4], o[5], o6, n);
    });
    CK(hipDeviceSynchronize());
    return 0;
}
