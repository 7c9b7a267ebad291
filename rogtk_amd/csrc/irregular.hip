// irregular.hip — exact grouping of irregular UMIs on gfx950.
//
// Irregular rows (valid, but not byte length L of pure A/C/G/T: 'N', lowercase,
// other lengths, empty, any UTF-8) are grouped by exact byte equality — the
// semantics of polars group_by('umi') used by the reference's callers
// (rogtk/__init__.py:206-214) — and numbered after the regular clusters in
// byte-lexicographic order (a proper prefix sorts first).
//
// Sort: LSD radix over the rows' bytes — one stable pass on the byte length, then
// one stable pass per 8-byte chunk (big-endian, zero padded) from the last chunk
// to the first. Zero padding + the length pass make the order exactly
// lexicographic. Equal neighbours are found by comparing bytes; a flag + scan
// numbers the distinct strings.
#include <hipcub/hipcub.hpp>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

constexpr int kBlock = 256;

template <int OW>
__device__ __forceinline__ void span(const void* offs, int64_t row, int64_t& st, int64_t& len) {
    if (OW == 4) {
        const int32_t* o = (const int32_t*)offs;
        st = o[row];
        len = (int64_t)o[row + 1] - o[row];
    } else {
        const int64_t* o = (const int64_t*)offs;
        st = o[row];
        len = o[row + 1] - o[row];
    }
}

template <int OW>
__global__ void k_len_keys(const void* __restrict__ offs, const int64_t* __restrict__ rows, int64_t n,
                           uint64_t* __restrict__ key, uint32_t* __restrict__ perm) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    int64_t st, len;
    span<OW>(offs, rows[k], st, len);
    key[k] = (uint64_t)len;
    perm[k] = (uint32_t)k;
}

template <int OW>
__global__ void k_chunk_keys(const void* __restrict__ offs, const uint8_t* __restrict__ vals,
                             const int64_t* __restrict__ rows, const uint32_t* __restrict__ perm,
                             int64_t n, int64_t chunk, uint64_t* __restrict__ key) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    int64_t st, len;
    span<OW>(offs, rows[perm[k]], st, len);
    uint64_t v = 0;
    const int64_t b0 = chunk * 8;
    for (int j = 0; j < 8; ++j) v = (v << 8) | (b0 + j < len ? vals[st + b0 + j] : 0u);
    key[k] = v;
}

template <int OW>
__global__ void k_eq_flags(const void* __restrict__ offs, const uint8_t* __restrict__ vals,
                           const int64_t* __restrict__ rows, const uint32_t* __restrict__ perm,
                           int64_t n, uint32_t* __restrict__ flag) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    uint32_t f = 1;
    if (k > 0) {
        int64_t sa, la, sb, lb;
        span<OW>(offs, rows[perm[k]], sa, la);
        span<OW>(offs, rows[perm[k - 1]], sb, lb);
        if (la == lb) {
            bool eq = true;
            for (int64_t j = 0; j < la && eq; ++j) eq = vals[sa + j] == vals[sb + j];
            f = eq ? 0u : 1u;
        }
    }
    flag[k] = f;
}

__global__ void k_irr_assign(const int64_t* __restrict__ rows, const uint32_t* __restrict__ perm,
                             const uint32_t* __restrict__ rank, const uint32_t* __restrict__ flag,
                             int64_t n, const int64_t* __restrict__ stats, uint32_t* __restrict__ out,
                             uint32_t* __restrict__ total) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    const uint32_t base = stats ? (uint32_t)stats[1] : 0u;  // regular clusters come first
    // id = (inclusive scan of "new string" flags) - 1, so every copy of a string
    // gets the id of its first copy in sorted order.
    out[rows[perm[k]]] = base + rank[k] + flag[k] - 1u;
    if (k == n - 1) *total = rank[k] + flag[k];
}

inline int grid_for(int64_t n) { return (int)std::max<int64_t>(1, (n + kBlock - 1) / kBlock); }

template <int OW>
int run(const void* offs, const uint8_t* vals, const int64_t* rows, int64_t n, int64_t max_len,
        const int64_t* stats_dev, uint32_t* cluster_id, int64_t* n_out, hipStream_t s) {
    const size_t n8 = (size_t)n * 8, n4 = (size_t)n * 4;
    size_t sort_bytes = 0, scan_bytes = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (uint64_t*)nullptr,
                                                       (uint64_t*)nullptr, (uint32_t*)nullptr,
                                                       (uint32_t*)nullptr, (int)n, 0, 64, s));
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint32_t*)nullptr,
                                                     (uint32_t*)nullptr, (int)n, s));
    const size_t tmp_bytes = std::max(sort_bytes, scan_bytes);
    const size_t total_bytes = 2 * n8 + 4 * n4 + tmp_bytes + 16 * 256;
    uint8_t* base = nullptr;
    ROGTK_HIP_CHECK(hipMallocAsync((void**)&base, total_bytes, s));
    size_t off = 0;
    auto take = [&](size_t b) {
        uint8_t* p = base + off;
        off += (b + 255) / 256 * 256;
        return p;
    };
    uint64_t* key = (uint64_t*)take(n8);
    uint64_t* key2 = (uint64_t*)take(n8);
    uint32_t* perm = (uint32_t*)take(n4);
    uint32_t* perm2 = (uint32_t*)take(n4);
    uint32_t* flag = (uint32_t*)take(n4);
    uint32_t* rank = (uint32_t*)take(n4);
    uint32_t* misc = (uint32_t*)take(256);
    void* tmp = take(tmp_bytes);
    const dim3 g(grid_for(n)), b(kBlock);
    bool ok = true;
    uint32_t total = 0;
    auto sort = [&]() {
        size_t tb = tmp_bytes;
        ok = ok && hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, key2, perm, perm2, (int)n, 0, 64, s) ==
                       hipSuccess;
        std::swap(perm, perm2);
    };
    hipLaunchKernelGGL(k_len_keys<OW>, g, b, 0, s, offs, rows, n, key, perm);
    sort();
    for (int64_t c = (max_len + 7) / 8 - 1; c >= 0 && ok; --c) {
        hipLaunchKernelGGL(k_chunk_keys<OW>, g, b, 0, s, offs, vals, rows, perm, n, c, key);
        sort();
    }
    if (ok) {
        hipLaunchKernelGGL(k_eq_flags<OW>, g, b, 0, s, offs, vals, rows, perm, n, flag);
        size_t tb = tmp_bytes;
        ok = hipcub::DeviceScan::ExclusiveSum(tmp, tb, flag, rank, (int)n, s) == hipSuccess;
    }
    if (ok) {
        hipLaunchKernelGGL(k_irr_assign, g, b, 0, s, rows, perm, rank, flag, n, stats_dev, cluster_id,
                           misc);
        ok = hipGetLastError() == hipSuccess &&
             hipMemcpyAsync(&total, misc, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
    }
    hipFreeAsync(base, s);
    ROGTK_REQUIRE(ok, ROGTK_E_HIP, "irregular_cluster: HIP failure");
    *n_out = total;
    return ROGTK_OK;
}

}  // namespace

int irregular_cluster(const void* offsets, int offset_width, const uint8_t* values,
                      const int64_t* rows, int64_t n_rows, int64_t max_len, const int64_t* stats_dev,
                      uint32_t* cluster_id, int64_t* n_irregular_clusters, hipStream_t s) {
    *n_irregular_clusters = 0;
    if (n_rows <= 0) return ROGTK_OK;
    ROGTK_REQUIRE(n_rows < (1ll << 31), ROGTK_E_UNSUPPORTED, "irregular rows: more than 2^31");
    ProfScope prof(K_IRREGULAR, s);
    if (offset_width == 4)
        return run<4>(offsets, values, rows, n_rows, max_len, stats_dev, cluster_id, n_irregular_clusters, s);
    return run<8>(offsets, values, rows, n_rows, max_len, stats_dev, cluster_id, n_irregular_clusters, s);
}

}  // namespace rogtk
