// Experiment (not product): k_local_cc on random code bitmaps of given density, timed
// and checked against a CPU union-find of the same LDS-local components.
// Includes the product kernels; links librogtk_hip.so for the host helpers they reference.
#define ROGTK_LCC_TIMING 1
#include "../rogtk_amd/csrc/cluster_kernels.hip"

#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <vector>

using namespace rogtk;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
    const int L = 12;
    ClusterLayout cl;
    cluster_layout(L, 1ll << 24, &cl);
    uint8_t* ws;
    CK(hipMalloc(&ws, cl.total));
    WsPtrs p = ws_ptrs(cl, ws);
    uint64_t* bm;
    CK(hipMalloc(&bm, cl.words * 8));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::mt19937_64 rng(5);
    for (double d : {0.065, 0.25, 0.42, 0.9}) {
        std::vector<uint64_t> h(cl.words);
        const uint64_t thr = (uint64_t)(d * 18446744073709551615.0);
        for (auto& w : h) {
            w = 0;
            for (int k = 0; k < 64; ++k) w |= (uint64_t)(rng() < thr) << k;
        }
        CK(hipMemcpy(bm, h.data(), cl.words * 8, hipMemcpyHostToDevice));
        CK(hipMemset(p.stats, 0, 64));
        hipLaunchKernelGGL(k_scan_words, dim3((unsigned)cl.blocks), dim3(kBlock), 0, 0, bm, 1, cl.words,
                           (const unsigned long long*)nullptr, p.G, p.wpref, p.blksum);
        hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kBlock), 0, 0, p.blksum, cl.blocks, p.blkoff, p.stats, 0, -1, 1,
                           (int64_t)0, getenv("LCC_P0_7") ? 0 : L);
        hipLaunchKernelGGL(k_rt, dim3(grid_for(cl.words)), dim3(kBlock), 0, 0, p.G, cl.words, p.wpref, p.blkoff, p.RT, p.lroot, cl.rwords);
        const int64_t lblocks = (cl.words + kLocalWords - 1) / kLocalWords;
        float best = 1e9;
        for (int it = 0; it < 8; ++it) {
            CK(hipDeviceSynchronize());
            hipEventRecord(a);
            launch_local_cc(p.RT, cl.words, L, p.f, p.D, p.UR, p.lroot, cl.rwords, cl.max_distinct, p.stats, 0);
            hipEventRecord(b);
            CK(hipEventSynchronize(b));
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        unsigned long long clk[8] = {0};
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_lcc_clk), clk, sizeof(clk)));
        launch_local_cc(p.RT, cl.words, L, p.f, p.D, p.UR, p.lroot, cl.rwords, cl.max_distinct, p.stats, 0);
        CK(hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_lcc_clk), sizeof(clk)));
        printf("  per-block us: phase1 %.2f union %.2f compress %.2f out %.2f\n", clk[0] / 100.0 / lblocks,
               clk[1] / 100.0 / lblocks, clk[2] / 100.0 / lblocks, clk[3] / 100.0 / lblocks);
        std::vector<uint32_t> f(1 << 24), ur(cl.words);
        std::vector<uint64_t> lr(cl.rwords);
        CK(hipMemcpy(f.data(), p.f, 4u << 24, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ur.data(), p.UR, cl.words * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(lr.data(), p.lroot, cl.rwords * 8, hipMemcpyDeviceToHost));
        // CPU truth: components over positions 0..6 inside each 4^7-code block; root = min code
        std::vector<uint32_t> rank(1u << 24), par(1u << 24);
        auto present = [&](uint32_t c) { return (h[c >> 6] >> (c & 63)) & 1; };
        uint32_t nd = 0;
        for (uint32_t c = 0; c < (1u << 24); ++c) {
            rank[c] = nd;
            par[c] = c;
            nd += present(c);
        }
        auto find = [&](uint32_t x) {
            while (par[x] != x) { par[x] = par[par[x]]; x = par[x]; }
            return x;
        };
        for (uint32_t c = 0; c < (1u << 24); ++c) {
            if (!present(c)) continue;
            for (int pos = 0; pos < 7; ++pos)
                for (uint32_t k = 1; k < 4; ++k) {
                    const uint32_t c2 = c ^ (k << (2 * pos));
                    if (c2 < c && present(c2)) {
                        uint32_t x = find(c), y = find(c2);
                        if (x != y) { if (x < y) std::swap(x, y); par[x] = y; }
                    }
                }
        }
        long bad_root = 0, bad_lr = 0, bad_self = 0;
        for (uint32_t c = 0; c < (1u << 24); ++c) {
            if (!present(c)) continue;
            const uint32_t want = rank[find(c)];
            const uint32_t got = ur[c >> 6] != 0xFFFFFFFFu ? ur[c >> 6] : f[rank[c]];
            bad_root += got != want;
            const bool is_root = find(c) == c;
            const bool live = is_root || ur[c >> 6] == 0xFFFFFFFFu;
            bad_lr += live != (bool)((lr[rank[c] >> 6] >> (rank[c] & 63)) & 1);
            if (is_root) bad_self += f[rank[c]] != rank[c];
        }
        printf("d=%.3f nd=%u local_cc %8.1f us  wrong: root %ld lroot %ld self %ld\n", d, nd, best * 1000, bad_root,
               bad_lr, bad_self);
    }
    return 0;
}
