// Experiment (not product): GPU idle time between two back-to-back kernels on one stream
// when the host puts an event record / a cross-stream wait between them (gfx950).
// Kernel A stamps its last wave's exit, kernel B its first wave's entry (wall_clock64);
// the gap is B.entry - A.exit in device ticks (100 MHz), median over 200 pairs.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void k_a(uint64_t* t, int spin) {
    uint64_t t0 = wall_clock64();
    while ((int64_t)(wall_clock64() - t0) < spin) {
    }
    __syncthreads();
    if (threadIdx.x == 0) atomicMax((unsigned long long*)t, (unsigned long long)wall_clock64());
}
__global__ void k_b(uint64_t* t) {
    if (threadIdx.x == 0) atomicMin((unsigned long long*)(t + 1), (unsigned long long)wall_clock64());
}

#define CK(x)                                                            \
    do {                                                                 \
        hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                          \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                    \
        }                                                                \
    } while (0)

int main() {
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    hipStream_t s, s2;
    CK(hipStreamCreate(&s));
    CK(hipStreamCreate(&s2));
    uint64_t* t;
    CK(hipMalloc(&t, 16 * 256));
    hipEvent_t e_def, e_nf, e_nt, e_ntnf, e_other, e_x;
    CK(hipEventCreate(&e_def));
    CK(hipEventCreateWithFlags(&e_nf, hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&e_nt, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e_ntnf, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&e_other, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&e_x, hipEventDisableSystemFence));
    const char* names[] = {"none",
                           "record(default event)",
                           "record(DisableSystemFence)",
                           "record(DisableTiming)",
                           "record(DisableTiming|DisableSystemFence)",
                           "wait(other stream, done, no-fence event)",
                           "record(nt|nf) + wait(other, done)",
                           "A launched with hipExt stop event (nf)",
                           "wait(other stream, done, default event)"};
    const int nv = 9, reps = 200;
    std::vector<uint64_t> h(2 * reps);
    // the other stream's events fire long before they are waited on
    CK(hipEventRecord(e_other, s2));
    hipEvent_t e_other_def;
    CK(hipEventCreate(&e_other_def));
    CK(hipEventRecord(e_other_def, s2));
    CK(hipStreamSynchronize(s2));
    for (int v = 0; v < nv; ++v) {
        std::vector<double> gaps;
        for (int r = 0; r < reps; ++r) {
            uint64_t* tr = t + 2 * (r % 128);
            uint64_t init[2] = {0, ~0ull};
            CK(hipMemcpyAsync(tr, init, 16, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            if (v == 7)
                hipExtLaunchKernelGGL(k_a, dim3(1024), dim3(256), 0, s, nullptr, e_x, 0, tr, 20000);
            else
                hipLaunchKernelGGL(k_a, dim3(1024), dim3(256), 0, s, tr, 20000);
            if (v == 1) CK(hipEventRecord(e_def, s));
            if (v == 2) CK(hipEventRecord(e_nf, s));
            if (v == 3) CK(hipEventRecord(e_nt, s));
            if (v == 4) CK(hipEventRecord(e_ntnf, s));
            if (v == 5) CK(hipStreamWaitEvent(s, e_other, 0));
            if (v == 6) {
                CK(hipEventRecord(e_ntnf, s));
                CK(hipStreamWaitEvent(s, e_other, 0));
            }
            if (v == 8) CK(hipStreamWaitEvent(s, e_other_def, 0));
            hipLaunchKernelGGL(k_b, dim3(1), dim3(64), 0, s, tr);
            CK(hipStreamSynchronize(s));
            uint64_t hh[2];
            CK(hipMemcpy(hh, tr, 16, hipMemcpyDeviceToHost));
            gaps.push_back((double)(int64_t)(hh[1] - hh[0]) * 1000.0 / khz);
        }
        std::sort(gaps.begin(), gaps.end());
        printf("%-45s gap median %7.2f us  p10 %7.2f  p90 %7.2f\n", names[v], gaps[reps / 2], gaps[reps / 10],
               gaps[reps * 9 / 10]);
    }
    // throughput form: 400 pairs of 20-us kernels back to back on the stream, the host
    // enqueue far ahead; total device time per pair with each variant between the kernels
    {
        hipEvent_t t0, t1;
        CK(hipEventCreate(&t0));
        CK(hipEventCreate(&t1));
        const int pairs = 400;
        for (int v = 0; v < nv; ++v) {
            float best = 1e30f;
            for (int it = 0; it < 3; ++it) {
                CK(hipEventRecord(t0, s));
                for (int r = 0; r < pairs; ++r) {
                    uint64_t* tr = t + 2 * (r % 128);
                    if (v == 7)
                        hipExtLaunchKernelGGL(k_a, dim3(1024), dim3(256), 0, s, nullptr, e_x, 0, tr, 2000);
                    else
                        hipLaunchKernelGGL(k_a, dim3(1024), dim3(256), 0, s, tr, 2000);
                    if (v == 1) CK(hipEventRecord(e_def, s));
                    if (v == 2) CK(hipEventRecord(e_nf, s));
                    if (v == 3) CK(hipEventRecord(e_nt, s));
                    if (v == 4) CK(hipEventRecord(e_ntnf, s));
                    if (v == 5) CK(hipStreamWaitEvent(s, e_other, 0));
                    if (v == 6) {
                        CK(hipEventRecord(e_ntnf, s));
                        CK(hipStreamWaitEvent(s, e_other, 0));
                    }
                    if (v == 8) CK(hipStreamWaitEvent(s, e_other_def, 0));
                    hipLaunchKernelGGL(k_a, dim3(1024), dim3(256), 0, s, tr, 2000);
                }
                CK(hipEventRecord(t1, s));
                CK(hipEventSynchronize(t1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, t0, t1));
                best = ms < best ? ms : best;
            }
            printf("%-45s per pair of 20-us kernels: %7.2f us (overhead vs 40 us: %6.2f)\n", names[v],
                   best * 1000 / pairs, best * 1000 / pairs - 40.0);
        }
    }
    return 0;
}
