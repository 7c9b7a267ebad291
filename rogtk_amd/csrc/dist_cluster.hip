// dist_cluster.hip — device steps of the sharded H3 (rogtk_amd/dist.py
// umi_cluster_sharded): UMI clusters over rows spread across ranks, merged with RCCL
// all-to-alls instead of the 4^L presence bitmap, so it covers every UMI length up to 32
// ("variant for L > 14"). Same spec and ids as the single-GPU engines
// (oracle/rogtk_oracle.cpp oracle_umi_cluster).
//
// Per rank (host orchestration in dist.py):
//   1. rogtk_long_codes       rows -> u64 2-bit codes + kind (null / regular / irregular)
//   2. rogtk_unique_codes     sorted distinct regular codes of the shard
//   3. rogtk_owner_counts     owner rank = code range (the sorted array is already
//                             grouped by owner) -> all-to-all -> unique again: the rank's
//                             owned distinct codes; all-gather -> the global sorted set G
//   4. rogtk_masked_records   per owned code and position p, (code with digit p zeroed, p,
//                             code), packed by destination rank = hash(masked key, p)
//                             -> all-to-all: every clique (codes equal but at p) meets on one rank
//   5. rogtk_clique_edges     group the received records by (p, masked key); consecutive
//                             members of a group are Hamming-1 neighbours -> edges as
//                             indices into G -> all-gather the edges
//   6. rogtk_cc_labels        hook-to-min + compress rounds over all edges on |G| vertices
//                             (redundant on every rank, deterministic): dense labels in
//                             order of each component's smallest code
//   7. rogtk_assign_codes     row -> its code's index in G (binary search) -> label
//   8. rogtk_irregular_merge  irregular rows (all-gathered strings): exact-bytes groups, or
//                             for max_distance 1 their Hamming-1 edges to each other and
//                             to G's codes merged with the regular clusters (irregular.hip;
//                             the G labels are remapped in place when clusters merge)
//   (7 runs after 8, so rows see the final labels)
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

constexpr int kB = 256;

inline dim3 grid(int64_t n, int64_t cap = 1 << 20) {
    return dim3((unsigned)std::min<int64_t>(cap, std::max<int64_t>(1, (n + kB - 1) / kB)));
}

__device__ __forceinline__ int base2(uint8_t c) {
    return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1;
}

template <int OW>
__global__ __launch_bounds__(kB) void k_long_codes(const void* __restrict__ offs, const uint8_t* __restrict__ vals,
                                                   const uint8_t* __restrict__ validity, int64_t voff, int64_t n, int L,
                                                   uint64_t* __restrict__ codes, uint8_t* __restrict__ kind) {
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) {
        bool valid = true;
        if (validity) {
            const int64_t b = voff + i;
            valid = (validity[b >> 3] >> (b & 7)) & 1;
        }
        uint64_t code = 0;
        uint8_t k = 0;
        if (valid) {
            int64_t st, len;
            if (OW == 4) {
                st = ((const int32_t*)offs)[i];
                len = (int64_t)((const int32_t*)offs)[i + 1] - st;
            } else {
                st = ((const int64_t*)offs)[i];
                len = ((const int64_t*)offs)[i + 1] - st;
            }
            bool regular = len == L;
            for (int j = 0; regular && j < L; ++j) {
                const int b = base2(vals[st + j]);
                regular = b >= 0;
                code = (code << 2) | (uint64_t)(b & 3);
            }
            k = regular ? 1 : 2;
            if (!regular) code = 0;
        }
        codes[i] = code;
        kind[i] = k;
    }
}

__global__ __launch_bounds__(kB) void k_regular_flags(const uint8_t* __restrict__ kind, int64_t n,
                                                      uint8_t* __restrict__ flags) {
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB)
        flags[i] = kind[i] == 1 ? 1 : 0;
}

// first index of sorted[] >= v
__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t* a, int64_t n, uint64_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// owner(code) = floor(code * world / 4^L): a contiguous code range per rank
__host__ __device__ __forceinline__ uint64_t owner_start(int r, int world, int L) {
    const unsigned __int128 space = (unsigned __int128)1 << (2 * L);
    return (uint64_t)((space * (unsigned)r + (unsigned)world - 1) / (unsigned)world);
}

__global__ void k_owner_bounds(const uint64_t* __restrict__ sorted, int64_t n, int L, int world,
                               int64_t* __restrict__ bounds) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r > world) return;
    bounds[r] = r == world ? n : lower_bound_u64(sorted, n, owner_start(r, world, L));
}

__device__ __forceinline__ uint64_t mask_digit(uint64_t c, int p) { return c & ~(3ull << (2 * p)); }

__device__ __forceinline__ uint32_t clique_dest(uint64_t mk, int p, int world) {
    uint64_t h = (mk ^ ((uint64_t)p << 58)) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    return (uint32_t)((h * 0xBF58476D1CE4E5B9ull) >> 33) % (uint32_t)world;
}

// record k = (code index k / L, position k % L): its destination rank
__global__ __launch_bounds__(kB) void k_record_dest(const uint64_t* __restrict__ D, int64_t n, int L, int world,
                                                    uint32_t* __restrict__ dest, uint32_t* __restrict__ rid) {
    const int64_t total = n * L;
    for (int64_t k = (int64_t)blockIdx.x * kB + threadIdx.x; k < total; k += (int64_t)gridDim.x * kB) {
        const int p = (int)(k % L);
        dest[k] = clique_dest(mask_digit(D[k / L], p), p, world);
        rid[k] = (uint32_t)k;
    }
}

__global__ __launch_bounds__(kB) void k_record_fill(const uint64_t* __restrict__ D, const uint32_t* __restrict__ rid,
                                                    int64_t total, int L, uint64_t* __restrict__ mk,
                                                    uint32_t* __restrict__ pos, uint64_t* __restrict__ code) {
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < total; i += (int64_t)gridDim.x * kB) {
        const uint32_t k = rid[i];
        const int p = (int)(k % (uint32_t)L);
        const uint64_t c = D[k / (uint32_t)L];
        mk[i] = mask_digit(c, p);
        pos[i] = (uint32_t)p;
        code[i] = c;
    }
}

__global__ void k_dest_counts(const uint32_t* __restrict__ sdest, int64_t total, int world,
                              int64_t* __restrict__ counts) {
    // sdest is sorted: rank r's count = upper_bound(r) - lower_bound(r)
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= world) return;
    int64_t lo = 0, hi = total;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (sdest[mid] < (uint32_t)r) lo = mid + 1;
        else hi = mid;
    }
    int64_t a = lo;
    lo = a;
    hi = total;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (sdest[mid] <= (uint32_t)r) lo = mid + 1;
        else hi = mid;
    }
    counts[r] = lo - a;
}

__global__ __launch_bounds__(kB) void k_iota(uint32_t* __restrict__ v, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) v[i] = (uint32_t)i;
}

__global__ __launch_bounds__(kB) void k_iota64(int64_t* __restrict__ v, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) v[i] = i;
}

__global__ __launch_bounds__(kB) void k_gather_pos(const uint32_t* __restrict__ pos, const uint32_t* __restrict__ perm,
                                                   int64_t n, uint32_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) out[i] = pos[perm[i]];
}

// consecutive records of one (p, masked key) group -> an edge between their codes' indices
// in G. Grid-stride over whole workgroup tiles (the wave append needs every lane in step),
// so any record count is covered by a capped grid.
__global__ __launch_bounds__(kB) void k_group_edges(const uint64_t* __restrict__ mk, const uint32_t* __restrict__ pos,
                                                    const uint64_t* __restrict__ code, const uint32_t* __restrict__ perm,
                                                    int64_t n, const uint64_t* __restrict__ G, int64_t ng,
                                                    uint2* __restrict__ E, unsigned long long* __restrict__ ne) {
    const int lane = threadIdx.x & 63;
    for (int64_t i0 = (int64_t)blockIdx.x * kB; i0 < n; i0 += (int64_t)gridDim.x * kB) {
        const int64_t i = i0 + threadIdx.x;
        bool e = false;
        uint32_t a = 0, b = 0;
        if (i > 0 && i < n) {
            const uint32_t x = perm[i - 1], y = perm[i];
            if (pos[x] == pos[y] && mk[x] == mk[y] && code[x] != code[y]) {
                e = true;
                a = (uint32_t)lower_bound_u64(G, ng, code[x]);
                b = (uint32_t)lower_bound_u64(G, ng, code[y]);
            }
        }
        const uint64_t m = __ballot(e);
        if (!m) continue;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(ne, (unsigned long long)__popcll(m));
        base = __shfl(base, 0);
        if (e) E[base + __popcll(m & ((1ull << lane) - 1ull))] = make_uint2(a, b);
    }
}

// records of positions p0 .. p0 + np - 1 of every distinct code (world 1, long engine)
__global__ __launch_bounds__(kB) void k_record_range(const uint64_t* __restrict__ D, int64_t nd, int p0, int np,
                                                     uint64_t* __restrict__ mk, uint32_t* __restrict__ pos,
                                                     uint64_t* __restrict__ code) {
    const int64_t total = nd * np;
    for (int64_t k = (int64_t)blockIdx.x * kB + threadIdx.x; k < total; k += (int64_t)gridDim.x * kB) {
        const int p = p0 + (int)(k % np);
        const uint64_t c = D[k / np];
        mk[k] = mask_digit(c, p);
        pos[k] = (uint32_t)p;
        code[k] = c;
    }
}

__device__ __forceinline__ uint32_t find_root(const uint32_t* f, uint32_t x) {
    for (uint32_t p = f[x]; p != x; p = f[x]) x = p;
    return x;
}

__global__ __launch_bounds__(kB) void k_hook_edges(const uint2* __restrict__ E, int64_t m, uint32_t* f,
                                                   unsigned int* __restrict__ changed) {
    bool ch = false;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < m; i += (int64_t)gridDim.x * kB) {
        const uint32_t a = find_root(f, E[i].x), b = find_root(f, E[i].y);
        if (a != b) {
            atomicMin(f + (a > b ? a : b), a < b ? a : b);
            ch = true;
        }
    }
    if (__any(ch) && (threadIdx.x & 63) == 0) *changed = 1u;
}

__global__ __launch_bounds__(kB) void k_compress_all(uint32_t* f, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB)
        f[i] = find_root(f, (uint32_t)i);
}

__global__ __launch_bounds__(kB) void k_root_flags(const uint32_t* __restrict__ f, int64_t n, uint32_t* __restrict__ r) {
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB)
        r[i] = f[i] == (uint32_t)i ? 1u : 0u;
}

__global__ __launch_bounds__(kB) void k_labels(const uint32_t* __restrict__ f, const uint32_t* __restrict__ rlab,
                                               int64_t n, uint32_t* __restrict__ lab) {
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) lab[i] = rlab[f[i]];
}

__global__ __launch_bounds__(kB) void k_assign_codes(const uint64_t* __restrict__ codes, const uint8_t* __restrict__ kind,
                                                     int64_t n, const uint64_t* __restrict__ G, int64_t ng,
                                                     const uint32_t* __restrict__ labels, uint32_t* __restrict__ cid,
                                                     unsigned int* __restrict__ missing) {
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) {
        const uint8_t k = kind[i];
        if (k == 0) {
            cid[i] = 0xFFFFFFFFu;
        } else if (k == 1) {
            const int64_t j = lower_bound_u64(G, ng, codes[i]);
            if (j < ng && G[j] == codes[i]) {
                cid[i] = labels[j];
            } else {
                cid[i] = 0xFFFFFFFFu;
                *missing = 1u;  // G must hold every regular code of every shard
            }
        }
    }
}

struct Scratch {
    void* p = nullptr;
    hipStream_t s = nullptr;
    ~Scratch() {
        if (p) (void)hipFreeAsync(p, s);
    }
    int get(size_t bytes, hipStream_t st) {
        s = st;
        ROGTK_HIP_CHECK(hipMallocAsync(&p, std::max<size_t>(bytes, 256), st));
        return ROGTK_OK;
    }
};

int check_len(int L) {
    ROGTK_REQUIRE(L >= 1 && L <= 32, ROGTK_E_UNSUPPORTED, "sharded cluster: umi_len %d outside 1..32", L);
    return ROGTK_OK;
}

}  // namespace

int masked_records_range(const uint64_t* D, int64_t nd, int p0, int np, uint64_t* mk, uint32_t* pos, uint64_t* code,
                         hipStream_t s) {
    if (nd <= 0 || np <= 0) return ROGTK_OK;
    hipLaunchKernelGGL(k_record_range, grid(nd * np, 16384), dim3(kB), 0, s, D, nd, p0, np, mk, pos, code);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

}  // namespace rogtk

using namespace rogtk;

extern "C" {

int rogtk_long_codes(const void* offsets, int offset_width, const uint8_t* values, const uint8_t* validity,
                     int64_t validity_offset, int64_t n, int umi_len, uint64_t* codes, uint8_t* kind, void* stream) {
    if (int rc = check_len(umi_len)) return rc;
    ROGTK_REQUIRE(offset_width == 4 || offset_width == 8, ROGTK_E_INVALID, "offset_width must be 4 or 8");
    ROGTK_REQUIRE(n >= 0 && (n == 0 || (offsets && codes && kind)), ROGTK_E_INVALID, "long_codes: NULL buffer");
    if (n == 0) return ROGTK_OK;
    hipStream_t s = (hipStream_t)stream;
    if (offset_width == 4)
        hipLaunchKernelGGL(k_long_codes<4>, grid(n, 16384), dim3(kB), 0, s, offsets, values, validity,
                           validity_offset, n, umi_len, codes, kind);
    else
        hipLaunchKernelGGL(k_long_codes<8>, grid(n, 16384), dim3(kB), 0, s, offsets, values, validity,
                           validity_offset, n, umi_len, codes, kind);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

int rogtk_unique_codes(const uint64_t* codes, const uint8_t* kind, int64_t n, int umi_len, uint64_t* out,
                       int64_t* n_out, void* stream) {
    if (int rc = check_len(umi_len)) return rc;
    ROGTK_REQUIRE(n_out && n >= 0 && n < (1ll << 31), ROGTK_E_INVALID, "unique_codes: bad n / NULL n_out");
    *n_out = 0;
    if (n == 0) return ROGTK_OK;
    ROGTK_REQUIRE(codes && out, ROGTK_E_INVALID, "unique_codes: NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    size_t sel_b = 0, sort_b = 0, uniq_b = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceSelect::Flagged(nullptr, sel_b, (uint64_t*)nullptr, (uint8_t*)nullptr,
                                                  (uint64_t*)nullptr, (int*)nullptr, (int)n, s));
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, sort_b, (uint64_t*)nullptr, (uint64_t*)nullptr, (int)n,
                                                      0, 64, s));
    ROGTK_HIP_CHECK(hipcub::DeviceSelect::Unique(nullptr, uniq_b, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                 (int*)nullptr, (int)n, s));
    const size_t tb = std::max({sel_b, sort_b, uniq_b});
    Scratch S;
    const size_t a8 = ((size_t)n * 8 + 255) / 256 * 256, a1 = ((size_t)n + 255) / 256 * 256;
    if (int rc = S.get(2 * a8 + a1 + 256 + tb, s)) return rc;
    uint64_t* reg = (uint64_t*)S.p;
    uint64_t* sorted = (uint64_t*)((uint8_t*)S.p + a8);
    uint8_t* flags = (uint8_t*)S.p + 2 * a8;
    int* cnt = (int*)((uint8_t*)S.p + 2 * a8 + a1);
    void* tmp = (uint8_t*)S.p + 2 * a8 + a1 + 256;
    const uint64_t* src = codes;
    int nreg = (int)n;
    if (kind) {  // the regular rows' codes only
        hipLaunchKernelGGL(k_regular_flags, grid(n, 16384), dim3(kB), 0, s, kind, n, flags);
        size_t b = tb;
        ROGTK_HIP_CHECK(hipcub::DeviceSelect::Flagged(tmp, b, codes, flags, reg, cnt, (int)n, s));
        ROGTK_HIP_CHECK(hipMemcpyAsync(&nreg, cnt, 4, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipStreamSynchronize(s));
        src = reg;
    }
    if (nreg == 0) return ROGTK_OK;
    size_t b = tb;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(tmp, b, src, sorted, nreg, 0, 2 * umi_len, s));
    b = tb;
    ROGTK_HIP_CHECK(hipcub::DeviceSelect::Unique(tmp, b, sorted, out, cnt, nreg, s));
    int h = 0;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&h, cnt, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    *n_out = h;
    return ROGTK_OK;
}

int rogtk_owner_counts(const uint64_t* sorted, int64_t n, int umi_len, int world, int64_t* counts, void* stream) {
    if (int rc = check_len(umi_len)) return rc;
    ROGTK_REQUIRE(world >= 1 && world <= 4096 && counts, ROGTK_E_INVALID, "owner_counts: bad world / NULL counts");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        for (int r = 0; r < world; ++r) counts[r] = 0;
        return ROGTK_OK;
    }
    Scratch S;
    if (int rc = S.get((size_t)(world + 1) * 8, s)) return rc;
    int64_t* bounds = (int64_t*)S.p;
    hipLaunchKernelGGL(k_owner_bounds, dim3((unsigned)((world + 1 + 255) / 256)), dim3(256), 0, s, sorted, n, umi_len,
                       world, bounds);
    ROGTK_HIP_CHECK(hipGetLastError());
    std::vector<int64_t> h((size_t)world + 1);
    ROGTK_HIP_CHECK(hipMemcpyAsync(h.data(), bounds, (size_t)(world + 1) * 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    for (int r = 0; r < world; ++r) counts[r] = h[(size_t)r + 1] - h[(size_t)r];
    return ROGTK_OK;
}

int rogtk_masked_records(const uint64_t* D, int64_t n, int umi_len, int world, uint64_t* mk, uint32_t* pos,
                         uint64_t* code, int64_t* counts, void* stream) {
    if (int rc = check_len(umi_len)) return rc;
    ROGTK_REQUIRE(world >= 1 && world <= 4096 && counts, ROGTK_E_INVALID, "masked_records: bad world / NULL counts");
    const int64_t total = n * umi_len;
    ROGTK_REQUIRE(total < (1ll << 31), ROGTK_E_UNSUPPORTED, "masked_records: n * umi_len >= 2^31");
    for (int r = 0; r < world; ++r) counts[r] = 0;
    if (n == 0) return ROGTK_OK;
    ROGTK_REQUIRE(D && mk && pos && code, ROGTK_E_INVALID, "masked_records: NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    if (world == 1) {  // one destination: records in (code, position) order, no packing sort
        Scratch S1;
        if (int rc = S1.get((size_t)total * 4, s)) return rc;
        hipLaunchKernelGGL(k_iota, grid(total, 16384), dim3(kB), 0, s, (uint32_t*)S1.p, total);
        hipLaunchKernelGGL(k_record_fill, grid(total, 16384), dim3(kB), 0, s, D, (const uint32_t*)S1.p, total,
                           umi_len, mk, pos, code);
        ROGTK_HIP_CHECK(hipGetLastError());
        counts[0] = total;
        return ROGTK_OK;
    }
    size_t sort_b = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                                       (uint32_t*)nullptr, (uint32_t*)nullptr, (int)total, 0, 32, s));
    const size_t a4 = ((size_t)total * 4 + 255) / 256 * 256;
    Scratch S;
    if (int rc = S.get(4 * a4 + (size_t)world * 8 + 256 + sort_b, s)) return rc;
    uint32_t* dest = (uint32_t*)S.p;
    uint32_t* rid = (uint32_t*)((uint8_t*)S.p + a4);
    uint32_t* sdest = (uint32_t*)((uint8_t*)S.p + 2 * a4);
    uint32_t* srid = (uint32_t*)((uint8_t*)S.p + 3 * a4);
    int64_t* dcnt = (int64_t*)((uint8_t*)S.p + 4 * a4);
    void* tmp = (uint8_t*)S.p + 4 * a4 + (size_t)world * 8 + 256;
    hipLaunchKernelGGL(k_record_dest, grid(total, 16384), dim3(kB), 0, s, D, n, umi_len, world, dest, rid);
    int dbits = 1;
    while ((1 << dbits) < world) ++dbits;
    size_t b = sort_b;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, b, dest, sdest, rid, srid, (int)total, 0, dbits, s));
    hipLaunchKernelGGL(k_record_fill, grid(total, 16384), dim3(kB), 0, s, D, srid, total, umi_len, mk, pos, code);
    hipLaunchKernelGGL(k_dest_counts, dim3((unsigned)((world + 255) / 256)), dim3(256), 0, s, sdest, total, world, dcnt);
    ROGTK_HIP_CHECK(hipGetLastError());
    ROGTK_HIP_CHECK(hipMemcpyAsync(counts, dcnt, (size_t)world * 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    return ROGTK_OK;
}

int rogtk_clique_edges(const uint64_t* mk, const uint32_t* pos, const uint64_t* code, int64_t n, int umi_len,
                       const uint64_t* G, int64_t ng, uint32_t* edges, int64_t* n_edges, void* stream) {
    if (int rc = check_len(umi_len)) return rc;
    ROGTK_REQUIRE(n_edges && n >= 0 && n < (1ll << 31), ROGTK_E_INVALID, "clique_edges: bad n / NULL n_edges");
    *n_edges = 0;
    if (n < 2) return ROGTK_OK;
    ROGTK_REQUIRE(mk && pos && code && G && edges, ROGTK_E_INVALID, "clique_edges: NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    size_t b1 = 0, b2 = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                       (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 64, s));
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, b2, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                                       (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 8, s));
    const size_t tb = std::max(b1, b2);
    const size_t a8 = ((size_t)n * 8 + 255) / 256 * 256, a4 = ((size_t)n * 4 + 255) / 256 * 256;
    Scratch S;
    if (int rc = S.get(a8 + 5 * a4 + 256 + tb, s)) return rc;
    uint64_t* smk = (uint64_t*)S.p;
    uint32_t* idx = (uint32_t*)((uint8_t*)S.p + a8);
    uint32_t* perm1 = (uint32_t*)((uint8_t*)S.p + a8 + a4);
    uint32_t* p1 = (uint32_t*)((uint8_t*)S.p + a8 + 2 * a4);
    uint32_t* sp = (uint32_t*)((uint8_t*)S.p + a8 + 3 * a4);
    uint32_t* perm = (uint32_t*)((uint8_t*)S.p + a8 + 4 * a4);
    unsigned long long* ne = (unsigned long long*)((uint8_t*)S.p + a8 + 5 * a4);
    void* tmp = (uint8_t*)S.p + a8 + 5 * a4 + 256;
    // LSD order: by masked key, then stably by position -> groups contiguous by (p, key)
    hipLaunchKernelGGL(k_iota, grid(n, 16384), dim3(kB), 0, s, idx, n);
    size_t b = tb;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, b, mk, smk, idx, perm1, (int)n, 0, 2 * umi_len, s));
    hipLaunchKernelGGL(k_gather_pos, grid(n, 16384), dim3(kB), 0, s, pos, perm1, n, p1);
    b = tb;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, b, p1, sp, perm1, perm, (int)n, 0, 8, s));
    ROGTK_HIP_CHECK(hipMemsetAsync(ne, 0, 8, s));
    hipLaunchKernelGGL(k_group_edges, grid(n, 16384), dim3(kB), 0, s, mk, pos, code, perm, n, G, ng, (uint2*)edges, ne);
    ROGTK_HIP_CHECK(hipGetLastError());
    unsigned long long h = 0;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&h, ne, 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    *n_edges = (int64_t)h;
    return ROGTK_OK;
}

int rogtk_cc_labels(int64_t nv, const uint32_t* edges, int64_t m, uint32_t* labels, int64_t* n_clusters,
                    void* stream) {
    ROGTK_REQUIRE(n_clusters && nv >= 0 && nv < (1ll << 32) && m >= 0, ROGTK_E_INVALID, "cc_labels: bad sizes");
    *n_clusters = 0;
    if (nv == 0) return ROGTK_OK;
    ROGTK_REQUIRE(labels && (m == 0 || edges), ROGTK_E_INVALID, "cc_labels: NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    size_t scan_b = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)nv,
                                                     s));
    const size_t a4 = ((size_t)nv * 4 + 255) / 256 * 256;
    Scratch S;
    if (int rc = S.get(3 * a4 + 256 + scan_b, s)) return rc;
    uint32_t* f = (uint32_t*)S.p;
    uint32_t* rflag = (uint32_t*)((uint8_t*)S.p + a4);
    uint32_t* rlab = (uint32_t*)((uint8_t*)S.p + 2 * a4);
    unsigned int* changed = (unsigned int*)((uint8_t*)S.p + 3 * a4);
    void* tmp = (uint8_t*)S.p + 3 * a4 + 256;
    hipLaunchKernelGGL(k_iota, grid(nv, 16384), dim3(kB), 0, s, f, nv);
    // hook-to-min + compress until no edge crosses two trees (f[x] <= x: roots are the
    // components' smallest indices = smallest codes)
    for (int round = 0; m > 0; ++round) {
        ROGTK_REQUIRE(round < 4096, ROGTK_E_HIP, "cc_labels: rounds did not converge");
        ROGTK_HIP_CHECK(hipMemsetAsync(changed, 0, 4, s));
        hipLaunchKernelGGL(k_hook_edges, grid(m, 16384), dim3(kB), 0, s, (const uint2*)edges, m, f, changed);
        hipLaunchKernelGGL(k_compress_all, grid(nv, 16384), dim3(kB), 0, s, f, nv);
        ROGTK_HIP_CHECK(hipGetLastError());
        unsigned int h = 0;
        ROGTK_HIP_CHECK(hipMemcpyAsync(&h, changed, 4, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipStreamSynchronize(s));
        if (!h) break;
    }
    hipLaunchKernelGGL(k_root_flags, grid(nv, 16384), dim3(kB), 0, s, f, nv, rflag);
    size_t b = scan_b;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, b, rflag, rlab, (int)nv, s));
    hipLaunchKernelGGL(k_labels, grid(nv, 16384), dim3(kB), 0, s, f, rlab, nv, labels);
    ROGTK_HIP_CHECK(hipGetLastError());
    uint32_t last[2];
    ROGTK_HIP_CHECK(hipMemcpyAsync(&last[0], rlab + nv - 1, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(&last[1], rflag + nv - 1, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    *n_clusters = (int64_t)last[0] + last[1];
    return ROGTK_OK;
}

int rogtk_assign_codes(const uint64_t* codes, const uint8_t* kind, int64_t n, const uint64_t* G, int64_t ng,
                       const uint32_t* labels, uint32_t* cluster_id, void* stream) {
    ROGTK_REQUIRE(n >= 0 && ng >= 0, ROGTK_E_INVALID, "assign_codes: negative size");
    if (n == 0) return ROGTK_OK;
    ROGTK_REQUIRE(codes && kind && cluster_id && (ng == 0 || (G && labels)), ROGTK_E_INVALID,
                  "assign_codes: NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    Scratch S;
    if (int rc = S.get(256, s)) return rc;
    unsigned int* missing = (unsigned int*)S.p;
    ROGTK_HIP_CHECK(hipMemsetAsync(missing, 0, 4, s));
    hipLaunchKernelGGL(k_assign_codes, grid(n, 16384), dim3(kB), 0, s, codes, kind, n, G, ng, labels, cluster_id,
                       missing);
    ROGTK_HIP_CHECK(hipGetLastError());
    unsigned int h = 0;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&h, missing, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    ROGTK_REQUIRE(!h, ROGTK_E_INVALID, "assign_codes: a regular code is missing from the global distinct set");
    return ROGTK_OK;
}

int rogtk_group_strings(const int64_t* offsets, const uint8_t* values, int64_t n, int64_t max_len, uint32_t id_base,
                        uint32_t* ids, int64_t* n_groups, void* stream) {
    ROGTK_REQUIRE(n_groups && n >= 0, ROGTK_E_INVALID, "group_strings: bad n / NULL n_groups");
    *n_groups = 0;
    if (n == 0) return ROGTK_OK;
    ROGTK_REQUIRE(offsets && ids, ROGTK_E_INVALID, "group_strings: NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    Scratch S;
    const size_t a8 = ((size_t)n * 8 + 255) / 256 * 256;
    if (int rc = S.get(a8 + 256, s)) return rc;
    int64_t* rows = (int64_t*)S.p;
    int64_t* base = (int64_t*)((uint8_t*)S.p + a8);  // stats block: [1] = the id base
    std::vector<int64_t> hrows((size_t)n);
    for (int64_t i = 0; i < n; ++i) hrows[(size_t)i] = i;
    const int64_t hb[2] = {0, (int64_t)id_base};
    ROGTK_HIP_CHECK(hipMemcpyAsync(rows, hrows.data(), (size_t)n * 8, hipMemcpyHostToDevice, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(base, hb, 16, hipMemcpyHostToDevice, s));
    int64_t groups = 0;
    if (int rc = irregular_cluster(offsets, 8, values, rows, n, std::max<int64_t>(max_len, 1), base, ids, &groups, s))
        return rc;
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    *n_groups = groups;
    return ROGTK_OK;
}

int rogtk_irregular_merge(const int64_t* offsets, const uint8_t* values, int64_t n, int64_t max_len, int umi_len,
                          int max_distance, const uint64_t* G, int64_t ng, uint32_t* labels, int64_t n_reg,
                          uint32_t* ids, int64_t* n_clusters, void* stream) {
    ROGTK_REQUIRE(n_clusters && n >= 0 && ng >= 0 && n_reg >= 0, ROGTK_E_INVALID, "irregular_merge: bad sizes");
    ROGTK_REQUIRE(max_distance == 0 || max_distance == 1, ROGTK_E_UNSUPPORTED,
                  "max_distance %d: only 0 and 1 are supported", max_distance);
    *n_clusters = n_reg;
    if (n == 0) return ROGTK_OK;
    if (max_distance == 0) {
        int64_t groups = 0;
        if (int rc = rogtk_group_strings(offsets, values, n, max_len, (uint32_t)n_reg, ids, &groups, stream))
            return rc;
        *n_clusters = n_reg + groups;
        return ROGTK_OK;
    }
    ROGTK_REQUIRE(offsets && ids && (ng == 0 || (G && labels)), ROGTK_E_INVALID, "irregular_merge: NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    Scratch S;
    if (int rc = S.get((size_t)n * 8, s)) return rc;
    int64_t* rows = (int64_t*)S.p;
    hipLaunchKernelGGL(k_iota64, grid(n, 16384), dim3(kB), 0, s, rows, n);
    ROGTK_HIP_CHECK(hipGetLastError());
    CodeLookup lk = [&](const uint64_t* q, int64_t nq, uint32_t* lab, hipStream_t st) {
        return sorted_code_lookup(G, ng, labels, q, nq, lab, st);
    };
    return irregular_merge(offsets, 8, values, rows, n, std::max<int64_t>(max_len, 1), umi_len, n_reg,
                           ng > 0 ? &lk : nullptr, labels, ng, ids, n_clusters, s);
}

}  // extern "C"
