// route.hip — rows of a string column packed by destination rank for one all-to-all
// ("groups must be co-located: route reads by hash(cluster id) with
// one alltoallv"). The exchange itself is torch.distributed (RCCL over xGMI); this is
// the device-side pack that makes each destination's rows one contiguous byte range.
//
//   1. stable radix sort of the destination ranks (hipcub) -> perm (rows by dest)
//   2. per-destination row and byte counts
//   3. lengths in perm order -> exclusive scan -> packed offsets
//   4. one wave per row copies its bytes to the packed buffer
#include <hipcub/hipcub.hpp>

#include <vector>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

constexpr int kMaxWorld = 1024;

__global__ __launch_bounds__(256) void k_iota(int64_t* p, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = i;
}

__global__ __launch_bounds__(256) void k_route_hist(const int32_t* __restrict__ dest, const int64_t* __restrict__ off,
                                                    int64_t n, int world, unsigned long long* rows,
                                                    unsigned long long* bytes, unsigned long long* bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int d = dest[i];
    if (d < 0 || d >= world) {
        atomicAdd(bad, 1ull);
        return;
    }
    atomicAdd(rows + d, 1ull);
    atomicAdd(bytes + d, (unsigned long long)(off[i + 1] - off[i]));
}

__global__ __launch_bounds__(256) void k_perm_lens(const int64_t* __restrict__ perm, const int64_t* __restrict__ off,
                                                   int64_t n, int64_t* __restrict__ lens) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const int64_t r = perm[i];
        lens[i] = off[r + 1] - off[r];
    } else if (i == n) {
        lens[n] = 0;
    }
}

__global__ __launch_bounds__(256) void k_copy_rows(const int64_t* __restrict__ perm, const int64_t* __restrict__ off,
                                                   const uint8_t* __restrict__ values,
                                                   const int64_t* __restrict__ poff, int64_t n,
                                                   uint8_t* __restrict__ out) {
    const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (w >= n) return;
    const int64_t r = perm[w];
    const int64_t a = off[r], len = off[r + 1] - a, o = poff[w];
    for (int64_t k = lane; k < len; k += 64) out[o + k] = values[a + k];
}

}  // namespace
}  // namespace rogtk

using namespace rogtk;

extern "C" int rogtk_route_pack(const int64_t* offsets, const uint8_t* values, const int32_t* dest, int64_t n,
                                int world, int64_t* perm, int64_t* counts, int64_t* byte_counts,
                                int64_t* packed_offsets, uint8_t* packed_values, int64_t values_cap, void* stream) {
    ROGTK_REQUIRE(world >= 1 && world <= kMaxWorld, ROGTK_E_INVALID, "route: world %d outside 1..%d", world,
                  kMaxWorld);
    ROGTK_REQUIRE(n >= 0 && (n == 0 || (offsets && values && dest && perm && packed_offsets && packed_values)),
                  ROGTK_E_INVALID, "route: NULL argument");
    ROGTK_REQUIRE(counts && byte_counts, ROGTK_E_INVALID, "route: NULL counts");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    thread_local DevBuf keys_out, iota, tmp, lens, hist;
    if (hist.ensure((size_t)(2 * world + 1) * 8) != ROGTK_OK) return ROGTK_E_HIP;
    ROGTK_HIP_CHECK(hipMemsetAsync(hist.p, 0, (size_t)(2 * world + 1) * 8, s));
    unsigned long long* h = hist.as<unsigned long long>();
    if (n > 0) {
        const dim3 g((unsigned)((n + 255) / 256));
        hipLaunchKernelGGL(k_route_hist, g, dim3(256), 0, s, dest, offsets, n, world, h, h + world, h + 2 * world);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    std::vector<unsigned long long> hh(2 * world + 1);
    ROGTK_HIP_CHECK(hipMemcpyAsync(hh.data(), hist.p, hh.size() * 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    ROGTK_REQUIRE(hh[2 * world] == 0, ROGTK_E_INVALID, "route: %llu destinations outside 0..%d",
                  hh[2 * world], world - 1);
    int64_t total = 0;
    for (int d = 0; d < world; ++d) {
        counts[d] = (int64_t)hh[d];
        byte_counts[d] = (int64_t)hh[world + d];
        total += byte_counts[d];
    }
    ROGTK_REQUIRE(total <= values_cap, ROGTK_E_OVERFLOW, "route: %lld bytes exceed values_cap %lld",
                  (long long)total, (long long)values_cap);
    if (n == 0) {
        ROGTK_HIP_CHECK(hipMemsetAsync(packed_offsets, 0, 8, s));
        return ROGTK_OK;
    }
    // stable sort of (dest, row) on the destination bits only
    int bits = 1;
    while ((1 << bits) < world) ++bits;
    if (keys_out.ensure((size_t)n * 4) != ROGTK_OK || iota.ensure((size_t)n * 8) != ROGTK_OK ||
        lens.ensure((size_t)(n + 1) * 8) != ROGTK_OK)
        return ROGTK_E_HIP;
    const dim3 g((unsigned)((n + 255) / 256));
    hipLaunchKernelGGL(k_iota, g, dim3(256), 0, s, iota.as<int64_t>(), n);
    size_t tb = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, dest, keys_out.as<int32_t>(), iota.as<int64_t>(),
                                                       perm, (int)n, 0, bits, s));
    if (tmp.ensure(tb) != ROGTK_OK) return ROGTK_E_HIP;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, dest, keys_out.as<int32_t>(), iota.as<int64_t>(),
                                                       perm, (int)n, 0, bits, s));
    hipLaunchKernelGGL(k_perm_lens, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, s, perm, offsets, n,
                       lens.as<int64_t>());
    tb = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, lens.as<int64_t>(), packed_offsets, (int)(n + 1), s));
    if (tmp.ensure(tb) != ROGTK_OK) return ROGTK_E_HIP;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, lens.as<int64_t>(), packed_offsets, (int)(n + 1), s));
    hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, s, perm, offsets, values,
                       packed_offsets, n, packed_values);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}
