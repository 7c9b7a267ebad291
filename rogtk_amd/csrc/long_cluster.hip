// long_cluster.hip — H3 for UMIs of 17..32 bases, where the 4^L presence
// bitmap of the packed engine (cluster_kernels.hip, L <= 16) stops being affordable.
//
// Same specification and ids as the packed engine and the oracle
// (oracle/rogtk_oracle.cpp: oracle_umi_cluster packs L <= 32):
//   * regular rows (valid, byte length L, pure ACGT) -> 2-bit codes in a u64;
//   * max_distance 0: one cluster per distinct code; 1: connected components of the
//     distinct codes under Hamming distance 1;
//   * ids dense in order of each cluster's smallest code; irregular rows grouped by
//     exact bytes after them (irregular.hip); null rows 0xFFFFFFFF.
//
// Sort-based, no code-space tables:
//   1. compact the regular rows as (code, row); radix-sort by code; run heads -> the
//      sorted distinct codes D and each row's distinct index;
//   2. one record (code with digit p zeroed, p, code) per distinct code and position,
//      sorted by masked code then stably by p: equal (p, key) runs are the codes that
//      differ only at p (a clique); consecutive members give edges (dist_cluster.hip);
//   3. hook-to-min + pointer-jump rounds over the edges until nothing changes (f[x] <= x,
//      so every root is its component's smallest index = smallest code);
//   4. roots -> scan -> dense labels -> rows.
#include <hipcub/hipcub.hpp>

#include <vector>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

constexpr int kB = 256;
// (code, position) records per edge-finding batch; ROGTK_LONG_REC_BATCH overrides (read
// per call: tests lower it to cover the batching)
inline int64_t rec_batch() {
    const char* e = getenv("ROGTK_LONG_REC_BATCH");
    const long long v = e ? atoll(e) : 0;
    return v > 0 ? (int64_t)v : (int64_t)1 << 28;
}

inline dim3 grid(int64_t n) { return dim3((unsigned)std::max<int64_t>(1, (n + kB - 1) / kB)); }

__device__ __forceinline__ int base2(uint8_t c) {
    return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1;
}

template <int OW>
__global__ __launch_bounds__(kB) void k_stage64(const void* __restrict__ offs, const uint8_t* __restrict__ vals,
                                                const uint8_t* __restrict__ validity, int64_t voff, int64_t n, int L,
                                                uint64_t* __restrict__ rkey, int64_t* __restrict__ rrow,
                                                unsigned long long* __restrict__ nreg, int64_t* __restrict__ irr,
                                                unsigned long long* __restrict__ nirr, uint32_t* __restrict__ cid) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    bool valid = false, regular = false;
    uint64_t code = 0;
    if (i < n) {
        valid = true;
        if (validity) {
            const int64_t b = voff + i;
            valid = (validity[b >> 3] >> (b & 7)) & 1;
        }
        if (valid) {
            int64_t st, len;
            if (OW == 4) {
                st = ((const int32_t*)offs)[i];
                len = (int64_t)((const int32_t*)offs)[i + 1] - st;
            } else {
                st = ((const int64_t*)offs)[i];
                len = ((const int64_t*)offs)[i + 1] - st;
            }
            regular = len == L;
            for (int j = 0; regular && j < L; ++j) {
                const int b = base2(vals[st + j]);
                regular = b >= 0;
                code = (code << 2) | (uint64_t)(b & 3);
            }
        } else {
            cid[i] = 0xFFFFFFFFu;
        }
    }
    const int lane = threadIdx.x & 63;
    const uint64_t rmask = __ballot(regular), imask = __ballot(valid && !regular);
    if (rmask) {
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(nreg, (unsigned long long)__popcll(rmask));
        base = __shfl(base, 0);
        if (regular) {
            const int64_t k = (int64_t)base + __popcll(rmask & ((1ull << lane) - 1ull));
            rkey[k] = code;
            rrow[k] = i;
        }
    }
    if (imask) {
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(nirr, (unsigned long long)__popcll(imask));
        base = __shfl(base, 0);
        if (valid && !regular) irr[base + __popcll(imask & ((1ull << lane) - 1ull))] = i;
    }
}

__global__ __launch_bounds__(kB) void k_heads(const uint64_t* __restrict__ k, int64_t n, uint32_t* __restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i < n) flag[i] = (i == 0 || k[i] != k[i - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(kB) void k_distinct(const uint64_t* __restrict__ k, const uint32_t* __restrict__ flag,
                                                 const uint32_t* __restrict__ ex, int64_t n, uint64_t* __restrict__ D,
                                                 unsigned long long* __restrict__ nd) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    if (flag[i]) D[ex[i]] = k[i];
    if (i == n - 1) *nd = (unsigned long long)ex[i] + flag[i];
}

// exclusive head count -> the row's distinct index (heads keep theirs)
__global__ __launch_bounds__(kB) void k_didx(const uint32_t* __restrict__ flag, int64_t n, uint32_t* __restrict__ ex) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i < n) ex[i] = ex[i] + flag[i] - 1u;
}

__global__ __launch_bounds__(kB) void k_iota32(uint32_t* p, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i < n) p[i] = (uint32_t)i;
}

__device__ __forceinline__ uint32_t find_root(const uint32_t* f, uint32_t x) {
    for (uint32_t p = f[x]; p != x; p = f[x]) x = p;
    return x;
}

__global__ __launch_bounds__(kB) void k_union(const uint2* __restrict__ E, int64_t m, uint32_t* f,
                                              unsigned int* __restrict__ changed) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    bool ch = false;
    if (i < m) {
        const uint32_t a = find_root(f, E[i].x), b = find_root(f, E[i].y);
        if (a != b) {
            atomicMin(f + (a > b ? a : b), a < b ? a : b);
            ch = true;
        }
    }
    if (__any(ch) && (threadIdx.x & 63) == 0) *changed = 1u;
}

__global__ __launch_bounds__(kB) void k_compress(uint32_t* f, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i < n) f[i] = find_root(f, (uint32_t)i);
}

__global__ __launch_bounds__(kB) void k_rootflags(const uint32_t* __restrict__ f, int64_t n, uint32_t* __restrict__ r) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i < n) r[i] = f[i] == (uint32_t)i ? 1u : 0u;
}

__global__ __launch_bounds__(kB) void k_assign_long(const int64_t* __restrict__ srow, const uint32_t* __restrict__ ex,
                                                    int64_t n, const uint32_t* __restrict__ f,
                                                    const uint32_t* __restrict__ rlab, int md,
                                                    uint32_t* __restrict__ cid) {
    const int64_t k = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    const uint32_t d = ex[k];
    cid[srow[k]] = md ? rlab[f[d]] : d;
}

__global__ void k_put_count(int64_t* stats, int64_t v) { stats[1] = v; }

// label of every distinct code (the irregular merge's lookup table)
__global__ __launch_bounds__(kB) void k_dlab(const uint32_t* __restrict__ f, const uint32_t* __restrict__ rlab,
                                             int64_t nd, uint32_t* __restrict__ dlab) {
    const int64_t d = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (d < nd) dlab[d] = rlab[f[d]];
}

struct Arena {
    uint8_t* base = nullptr;
    size_t off = 0, cap = 0;
    hipStream_t s;
    ~Arena() {
        if (base) (void)hipFreeAsync(base, s);
    }
    template <class T>
    T* take(int64_t count) {
        uint8_t* p = base + off;
        off += ((size_t)std::max<int64_t>(count, 1) * sizeof(T) + 255) / 256 * 256;
        return (T*)p;
    }
};

}  // namespace

int long_cluster(const void* offsets, int ow, const uint8_t* values, const uint8_t* validity, int64_t voff,
                 int64_t n, int L, int max_distance, int64_t max_len, uint32_t* cid, int64_t* n_clusters,
                 hipStream_t s) {
    ROGTK_REQUIRE(L > kMaxPackedLen && L <= 32, ROGTK_E_UNSUPPORTED, "long_cluster: umi_len %d outside 17..32", L);
    ROGTK_REQUIRE(n < (1ll << 31), ROGTK_E_UNSUPPORTED, "long_cluster: more than 2^31 rows");
    if (n_clusters) *n_clusters = 0;
    if (n <= 0) return ROGTK_OK;
    ProfScope prof(K_UNION, s);
    // scratch sizes (the sort temp is sized for the largest sort)
    size_t sort_b = 0, scan_b = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                       (int64_t*)nullptr, (int64_t*)nullptr, (int)n, 0, 64, s));
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                                     (int)n, s));
    const size_t tmp_b = std::max({sort_b, scan_b});
    Arena A;
    A.s = s;
    A.cap = (size_t)n * (8 * 8 + 4 * 6) + (size_t)n * L * 8 + tmp_b + 64 * 256;
    ROGTK_HIP_CHECK(hipMallocAsync((void**)&A.base, A.cap, s));
    uint64_t* rkey = A.take<uint64_t>(n);
    uint64_t* skey = A.take<uint64_t>(n);
    int64_t* rrow = A.take<int64_t>(n);
    int64_t* srow = A.take<int64_t>(n);
    int64_t* irr = A.take<int64_t>(n);
    uint32_t* flag = A.take<uint32_t>(n);
    uint32_t* ex = A.take<uint32_t>(n);
    uint64_t* D = A.take<uint64_t>(n);
    uint32_t* f = A.take<uint32_t>(n);
    uint32_t* rlab = A.take<uint32_t>(n);
    uint2* E = A.take<uint2>(n * (int64_t)L);
    unsigned long long* cnt = A.take<unsigned long long>(8);  // nreg, nirr, nd, ne, changed
    int64_t* stats = A.take<int64_t>(2);
    void* tmp = A.take<uint8_t>((int64_t)tmp_b);
    ROGTK_HIP_CHECK(hipMemsetAsync(cnt, 0, 8 * 8, s));
    if (ow == 4)
        hipLaunchKernelGGL(k_stage64<4>, grid(n), dim3(kB), 0, s, offsets, values, validity, voff, n, L, rkey, rrow,
                           cnt, irr, cnt + 1, cid);
    else
        hipLaunchKernelGGL(k_stage64<8>, grid(n), dim3(kB), 0, s, offsets, values, validity, voff, n, L, rkey, rrow,
                           cnt, irr, cnt + 1, cid);
    ROGTK_HIP_CHECK(hipGetLastError());
    unsigned long long h[2];
    ROGTK_HIP_CHECK(hipMemcpyAsync(h, cnt, 16, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    const int64_t nreg = (int64_t)h[0], nirr = (int64_t)h[1];
    int64_t n_reg_clusters = 0;
    int64_t nd_all = 0;  // distinct regular codes
    if (nreg > 0) {
        size_t tb = tmp_b;
        ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, rkey, skey, rrow, srow, (int)nreg, 0, 2 * L, s));
        hipLaunchKernelGGL(k_heads, grid(nreg), dim3(kB), 0, s, skey, nreg, flag);
        tb = tmp_b;
        ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, flag, ex, (int)nreg, s));
        hipLaunchKernelGGL(k_distinct, grid(nreg), dim3(kB), 0, s, skey, flag, ex, nreg, D, cnt + 2);
        hipLaunchKernelGGL(k_didx, grid(nreg), dim3(kB), 0, s, flag, nreg, ex);
        ROGTK_HIP_CHECK(hipGetLastError());
        unsigned long long hnd = 0;
        ROGTK_HIP_CHECK(hipMemcpyAsync(&hnd, cnt + 2, 8, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipStreamSynchronize(s));
        const int64_t nd = (int64_t)hnd;
        nd_all = nd;
        if (max_distance == 1) {
            hipLaunchKernelGGL(k_iota32, grid(nd), dim3(kB), 0, s, f, nd);
            // edges: one record (code with digit p zeroed, p, code) per distinct code and
            // position, grouped by (p, masked code) with two sorts (dist_cluster.hip, the
            // steps of the sharded engine at world 1) instead of one sort per position:
            // 1.7x faster at L = 20 (10M reads)
            // positions in batches of <= rec_batch() records (nd * L may pass 2^31, the
            // sorts' limit; the batch also bounds the 20 B/record scratch)
            int64_t ne = 0;
            {
                const int64_t per = std::max<int64_t>(1, std::min<int64_t>(L, rec_batch() / std::max<int64_t>(nd, 1)));
                ROGTK_REQUIRE(nd < (1ll << 31), ROGTK_E_UNSUPPORTED, "long_cluster: 2^31 distinct UMIs");
                const int64_t nrec_max = nd * per;
                Arena R;
                R.s = s;
                R.cap = (size_t)nrec_max * 20 + 3 * 256;
                ROGTK_HIP_CHECK(hipMallocAsync((void**)&R.base, R.cap, s));
                uint64_t* rmk = R.take<uint64_t>(nrec_max);
                uint32_t* rpos = R.take<uint32_t>(nrec_max);
                uint64_t* rcode = R.take<uint64_t>(nrec_max);
                for (int p0 = 0; p0 < L; p0 += (int)per) {
                    const int np = (int)std::min<int64_t>(per, L - p0);
                    if (int rc = masked_records_range(D, nd, p0, np, rmk, rpos, rcode, s)) return rc;
                    int64_t got = 0;
                    if (int rc = rogtk_clique_edges(rmk, rpos, rcode, nd * np, L, D, nd, (uint32_t*)(E + ne), &got, s))
                        return rc;
                    ne += got;
                }
            }
            for (int round = 0; ne > 0; ++round) {
                ROGTK_REQUIRE(round < 4096, ROGTK_E_HIP, "long_cluster: union rounds did not converge");
                ROGTK_HIP_CHECK(hipMemsetAsync(cnt + 4, 0, 8, s));
                hipLaunchKernelGGL(k_union, grid(ne), dim3(kB), 0, s, E, ne, f, (unsigned int*)(cnt + 4));
                hipLaunchKernelGGL(k_compress, grid(nd), dim3(kB), 0, s, f, nd);
                unsigned long long ch = 0;
                ROGTK_HIP_CHECK(hipMemcpyAsync(&ch, cnt + 4, 8, hipMemcpyDeviceToHost, s));
                ROGTK_HIP_CHECK(hipStreamSynchronize(s));
                if (!ch) break;
            }
            hipLaunchKernelGGL(k_rootflags, grid(nd), dim3(kB), 0, s, f, nd, flag);
            tb = tmp_b;
            ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, flag, rlab, (int)nd, s));
            uint32_t last[2];
            ROGTK_HIP_CHECK(hipMemcpyAsync(&last[0], rlab + nd - 1, 4, hipMemcpyDeviceToHost, s));
            ROGTK_HIP_CHECK(hipMemcpyAsync(&last[1], flag + nd - 1, 4, hipMemcpyDeviceToHost, s));
            ROGTK_HIP_CHECK(hipStreamSynchronize(s));
            n_reg_clusters = (int64_t)last[0] + last[1];
        } else {
            n_reg_clusters = nd;
        }
        hipLaunchKernelGGL(k_assign_long, grid(nreg), dim3(kB), 0, s, srow, ex, nreg, f, rlab, max_distance, cid);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    int64_t total = n_reg_clusters;
    if (nirr > 0 && max_distance == 1) {
        // Hamming-1 edges of the irregular rows, merged with the regular clusters
        // (irregular.hip); the lookup binary-searches the sorted distinct codes
        const int64_t nd = n_reg_clusters > 0 ? nd_all : 0;
        uint32_t* dlab = flag;  // free after the labels: one label per distinct code
        if (nd > 0) {
            hipLaunchKernelGGL(k_dlab, grid(nd), dim3(kB), 0, s, f, rlab, nd, dlab);
            ROGTK_HIP_CHECK(hipGetLastError());
        }
        CodeLookup lk = [&](const uint64_t* q, int64_t nq, uint32_t* lab, hipStream_t st) {
            return sorted_code_lookup(D, nd, dlab, q, nq, lab, st);
        };
        if (int rc = irregular_merge(offsets, ow, values, irr, nirr, max_len, L, n_reg_clusters, nd > 0 ? &lk : nullptr,
                                     cid, n, cid, &total, s))
            return rc;
    } else if (nirr > 0) {
        int64_t n_irr_clusters = 0;
        hipLaunchKernelGGL(k_put_count, dim3(1), dim3(1), 0, s, stats, n_reg_clusters);
        if (int rc = irregular_cluster(offsets, ow, values, irr, nirr, max_len, stats, cid, &n_irr_clusters, s))
            return rc;
        total += n_irr_clusters;
    }
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    if (n_clusters) *n_clusters = total;
    return ROGTK_OK;
}

}  // namespace rogtk
