// irregular.hip — H3 for irregular UMIs on gfx950.
//
// Irregular rows are valid rows that are not byte length L of pure A/C/G/T ('N',
// lowercase, other lengths, empty, any UTF-8). Their distinct strings are numbered after
// the regular clusters in byte-lexicographic order (a proper prefix sorts first).
//
// max_distance 0 (irregular_cluster): groups of exactly equal bytes — the semantics of
// polars group_by('umi') used by the reference's callers (rogtk/__init__.py:206-214).
//
// max_distance 1 (irregular_merge): SURVEY.md §8a H3.2 — connected components over ALL
// distinct strings with an edge wherever the H2.1 distance (expressions.rs:1054-1069:
// equal byte length, then mismatches) is 1, byte-wise. Besides the regular-regular edges
// the regular engines find, that adds
//   * irregular ~ irregular: equal length, equal except at one position p. One record per
//     (distinct string, position) keyed by a hash of (length, p, the string without byte
//     p), radix-sorted; every record links to the nearest earlier record of its key run
//     whose masked bytes really are equal (the hash only groups; bytes decide);
//   * irregular ~ regular: a string of length L with exactly one non-ACGT byte, at p, is
//     1 byte from the <= 4 codes with A/C/G/T at p. Those codes are pairwise Hamming-1, so
//     the present ones already share one regular component: one edge to its label.
// Vertices are the regular clusters (0..n_reg-1, in order of their smallest code) and the
// distinct irregular strings (n_reg + j, byte-lexicographic); hook-to-min connected
// components keep every root the smallest vertex, so dense ids come out as the spec wants:
// components with a regular UMI first (by smallest regular code), then the rest (by
// smallest string). Regular clusters bridged by irregular strings merge: the caller's
// regular ids are then remapped in place.
//
// Sort: LSD radix over the rows' bytes — one stable pass on the byte length, then one
// stable pass per 8-byte chunk (big-endian, zero padded) from the last chunk to the first.
// Zero padding + the length pass make the order exactly lexicographic. Equal neighbours
// are found by comparing bytes; a flag + scan numbers the distinct strings.
#include <hipcub/hipcub.hpp>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

constexpr int kBlock = 256;
constexpr uint32_t kNoLabel = 0xFFFFFFFFu;
constexpr uint64_t kNoCode = ~0ull;
constexpr int kMaxRunWalk = 4096;  // masked-key run members compared per record (bytes decide)

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

// ------------------------------------------------------------ Hamming-1 merge
__device__ __forceinline__ uint64_t fmix64(uint64_t h) {
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 33;
    return h;
}
// per-position multiplier of the string hash h = sum_i b_i * R(i) (mod 2^64)
__device__ __forceinline__ uint64_t pos_mult(int64_t i) { return fmix64((uint64_t)i + 0x9E3779B97F4A7C15ull) | 1ull; }

__device__ __forceinline__ int base2(uint8_t c) {
    return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1;
}

// distinct string d (sorted order) -> its first row and length
template <int OW>
__global__ void k_distinct_rep(const void* __restrict__ offs, const int64_t* __restrict__ rows,
                               const uint32_t* __restrict__ perm, const uint32_t* __restrict__ rank,
                               const uint32_t* __restrict__ flag, int64_t n, int64_t* __restrict__ rep,
                               int64_t* __restrict__ dlen) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n || !flag[k]) return;
    const int64_t row = rows[perm[k]];
    int64_t st, len;
    span<OW>(offs, row, st, len);
    rep[rank[k]] = row;
    dlen[rank[k]] = len;
}

// Per distinct string d: its records (masked-key hash, (d << 32) | p) for every position,
// and, when it has length L <= 32 with exactly one non-ACGT byte, the 4 regular codes 1
// byte away (kNoCode otherwise).
template <int OW>
__global__ void k_records(const void* __restrict__ offs, const uint8_t* __restrict__ vals,
                          const int64_t* __restrict__ rep, const int64_t* __restrict__ roff, int64_t nd, int L,
                          uint64_t* __restrict__ key, uint64_t* __restrict__ val, uint64_t* __restrict__ q) {
    const int64_t d = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (d >= nd) return;
    int64_t st, len;
    span<OW>(offs, rep[d], st, len);
    const uint8_t* s = vals + st;
    uint64_t h = 0;
    for (int64_t i = 0; i < len; ++i) h += (uint64_t)s[i] * pos_mult(i);
    const int64_t r0 = roff[d];
    for (int64_t p = 0; p < len; ++p) {
        const uint64_t hm = h - (uint64_t)s[p] * pos_mult(p);
        key[r0 + p] = fmix64(hm ^ fmix64(((uint64_t)len << 32) ^ (uint64_t)p ^ 0x5A5A5A5A00000000ull));
        val[r0 + p] = ((uint64_t)d << 32) | (uint64_t)p;
    }
    if (q) {
        uint64_t c = 0;
        int bad = -1, nbad = 0;
        if (L >= 1 && L <= 32 && len == L) {
            for (int i = 0; i < L; ++i) {
                int b = base2(s[i]);
                if (b < 0) {
                    ++nbad;
                    bad = i;
                    b = 0;
                }
                c = (c << 2) | (uint64_t)b;
            }
        }
        const int sh = 2 * (L - 1 - bad);
        for (int x = 0; x < 4; ++x)
            q[4 * d + x] = nbad == 1 ? ((c & ~(3ull << sh)) | ((uint64_t)x << sh)) : kNoCode;
    }
}

// wave-aggregated append of one edge per flagged lane
__device__ __forceinline__ void append_edge(bool e, uint32_t a, uint32_t b, uint2* __restrict__ E,
                                            unsigned long long* __restrict__ ne) {
    const uint64_t m = __ballot(e);
    if (!m) return;
    const int lane = threadIdx.x & 63;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(ne, (unsigned long long)__popcll(m));
    base = __shfl(base, 0);
    if (e) E[base + __popcll(m & ((1ull << lane) - 1ull))] = make_uint2(a, b);
}

// sorted record k -> an edge to the nearest earlier record of its key run whose string
// equals its own except at the same position p (same length)
template <int OW>
__global__ void k_masked_edges(const void* __restrict__ offs, const uint8_t* __restrict__ vals,
                               const int64_t* __restrict__ rep, const uint64_t* __restrict__ skey,
                               const uint64_t* __restrict__ sval, int64_t nr, uint32_t vbase,
                               uint2* __restrict__ E, unsigned long long* __restrict__ ne,
                               unsigned int* __restrict__ overflow) {
    for (int64_t k0 = (int64_t)blockIdx.x * kBlock; k0 < nr; k0 += (int64_t)gridDim.x * kBlock) {
        const int64_t k = k0 + threadIdx.x;
        bool e = false;
        uint32_t a = 0, b = 0;
        if (k > 0 && k < nr && skey[k] == skey[k - 1]) {
            const uint64_t vk = sval[k];
            const uint32_t dk = (uint32_t)(vk >> 32), pk = (uint32_t)vk;
            int64_t sk, lk;
            span<OW>(offs, rep[dk], sk, lk);
            int walked = 0;
            for (int64_t j = k - 1; j >= 0 && skey[j] == skey[k]; --j) {
                if (++walked > kMaxRunWalk) {
                    *overflow = 1u;
                    break;
                }
                const uint64_t vj = sval[j];
                const uint32_t dj = (uint32_t)(vj >> 32), pj = (uint32_t)vj;
                if (pj != pk) continue;
                int64_t sj, lj;
                span<OW>(offs, rep[dj], sj, lj);
                if (lj != lk) continue;
                bool eq = true;
                for (int64_t i = 0; i < lk && eq; ++i) eq = i == (int64_t)pk || vals[sj + i] == vals[sk + i];
                if (eq) {
                    e = true;
                    a = vbase + dj;
                    b = vbase + dk;
                    break;
                }
            }
        }
        append_edge(e, a, b, E, ne);
    }
}

// distinct string d -> an edge to the regular cluster of any present neighbour code
__global__ void k_regular_edges(const uint32_t* __restrict__ lab4, int64_t nd, uint32_t vbase,
                                uint2* __restrict__ E, unsigned long long* __restrict__ ne) {
    for (int64_t d0 = (int64_t)blockIdx.x * kBlock; d0 < nd; d0 += (int64_t)gridDim.x * kBlock) {
        const int64_t d = d0 + threadIdx.x;
        bool e = false;
        uint32_t a = 0;
        if (d < nd)
            for (int x = 0; x < 4 && !e; ++x) {
                const uint32_t l = lab4[4 * d + x];
                if (l != kNoLabel) {
                    e = true;
                    a = l;
                }
            }
        append_edge(e, a, vbase + (uint32_t)d, E, ne);
    }
}

// ids of regular clusters after a merge: v < n_reg -> labels[v]
__global__ void k_relabel(uint32_t* __restrict__ ids, int64_t n, const uint32_t* __restrict__ labels, uint32_t n_reg) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const uint32_t v = ids[i];
        if (v < n_reg) ids[i] = labels[v];
    }
}

__global__ void k_irr_write(const int64_t* __restrict__ rows, const uint32_t* __restrict__ perm,
                            const uint32_t* __restrict__ rank, const uint32_t* __restrict__ flag, int64_t n,
                            const uint32_t* __restrict__ labels, uint32_t vbase, uint32_t* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    out[rows[perm[k]]] = labels[vbase + rank[k] + flag[k] - 1u];
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

__global__ void k_sorted_lookup(const uint64_t* __restrict__ G, int64_t ng, const uint32_t* __restrict__ labels,
                                const uint64_t* __restrict__ q, int64_t nq, uint32_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nq; i += (int64_t)gridDim.x * kBlock) {
        const uint64_t c = q[i];
        uint32_t l = kNoLabel;
        if (c != kNoCode) {
            const int64_t j = lower_bound_u64(G, ng, c);
            if (j < ng && G[j] == c) l = labels[j];
        }
        out[i] = l;
    }
}

inline int grid_for(int64_t n, int64_t cap = 1 << 20) {
    return (int)std::min<int64_t>(cap, std::max<int64_t>(1, (n + kBlock - 1) / kBlock));
}

struct Arena {
    uint8_t* base = nullptr;
    size_t off = 0;
    hipStream_t s = nullptr;
    ~Arena() {
        if (base) (void)hipFreeAsync(base, s);
    }
    int get(size_t bytes, hipStream_t st) {
        s = st;
        ROGTK_HIP_CHECK(hipMallocAsync((void**)&base, std::max<size_t>(bytes, 256), st));
        return ROGTK_OK;
    }
    template <class T>
    T* take(int64_t count) {
        uint8_t* p = base + off;
        off += ((size_t)std::max<int64_t>(count, 1) * sizeof(T) + 255) / 256 * 256;
        return (T*)p;
    }
};
inline size_t al(size_t b) { return (std::max<size_t>(b, 1) + 255) / 256 * 256; }

// The sorted order of the irregular rows: perm (sorted position -> index into rows),
// flag (first copy of a string), rank (exclusive scan of flag = distinct index - [!flag]).
struct StringSort {
    Arena A;
    uint32_t *perm = nullptr, *flag = nullptr, *rank = nullptr;
    int64_t distinct = 0;
};

template <int OW>
int sort_strings(const void* offs, const uint8_t* vals, const int64_t* rows, int64_t n, int64_t max_len,
                 StringSort& S, hipStream_t s) {
    const size_t n8 = (size_t)n * 8, n4 = (size_t)n * 4;
    size_t sort_bytes = 0, scan_bytes = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (uint64_t*)nullptr,
                                                       (uint64_t*)nullptr, (uint32_t*)nullptr,
                                                       (uint32_t*)nullptr, (int)n, 0, 64, s));
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint32_t*)nullptr,
                                                     (uint32_t*)nullptr, (int)n, s));
    const size_t tmp_bytes = std::max(sort_bytes, scan_bytes);
    if (int rc = S.A.get(2 * al(n8) + 4 * al(n4) + al(tmp_bytes) + 256, s)) return rc;
    uint64_t* key = S.A.take<uint64_t>(n);
    uint64_t* key2 = S.A.take<uint64_t>(n);
    uint32_t* perm = S.A.take<uint32_t>(n);
    uint32_t* perm2 = S.A.take<uint32_t>(n);
    uint32_t* flag = S.A.take<uint32_t>(n);
    uint32_t* rank = S.A.take<uint32_t>(n);
    void* tmp = S.A.take<uint8_t>((int64_t)tmp_bytes);
    const dim3 g(grid_for(n, 1ll << 31)), b(kBlock);
    auto sort = [&]() -> int {
        size_t tb = tmp_bytes;
        ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, key2, perm, perm2, (int)n, 0, 64, s));
        std::swap(perm, perm2);
        return ROGTK_OK;
    };
    hipLaunchKernelGGL(k_len_keys<OW>, g, b, 0, s, offs, rows, n, key, perm);
    if (int rc = sort()) return rc;
    for (int64_t c = (max_len + 7) / 8 - 1; c >= 0; --c) {
        hipLaunchKernelGGL(k_chunk_keys<OW>, g, b, 0, s, offs, vals, rows, perm, n, c, key);
        if (int rc = sort()) return rc;
    }
    hipLaunchKernelGGL(k_eq_flags<OW>, g, b, 0, s, offs, vals, rows, perm, n, flag);
    size_t tb = tmp_bytes;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, flag, rank, (int)n, s));
    ROGTK_HIP_CHECK(hipGetLastError());
    uint32_t last[2];
    ROGTK_HIP_CHECK(hipMemcpyAsync(&last[0], rank + n - 1, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(&last[1], flag + n - 1, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    S.perm = perm;
    S.flag = flag;
    S.rank = rank;
    S.distinct = (int64_t)last[0] + last[1];
    return ROGTK_OK;
}

template <int OW>
int run_exact(const void* offs, const uint8_t* vals, const int64_t* rows, int64_t n, int64_t max_len,
              const int64_t* stats_dev, uint32_t* cluster_id, int64_t* n_out, hipStream_t s) {
    StringSort S;
    if (int rc = sort_strings<OW>(offs, vals, rows, n, max_len, S, s)) return rc;
    Arena M;
    if (int rc = M.get(256, s)) return rc;
    hipLaunchKernelGGL(k_irr_assign, dim3(grid_for(n, 1ll << 31)), dim3(kBlock), 0, s, rows, S.perm, S.rank, S.flag,
                       n, stats_dev, cluster_id, M.take<uint32_t>(1));
    ROGTK_HIP_CHECK(hipGetLastError());
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    *n_out = S.distinct;
    return ROGTK_OK;
}

template <int OW>
int run_merge(const void* offs, const uint8_t* vals, const int64_t* rows, int64_t n, int64_t max_len, int L,
              int64_t n_reg, const CodeLookup* lookup, uint32_t* relabel, int64_t relabel_n, uint32_t* cluster_id,
              int64_t* n_clusters, hipStream_t s) {
    StringSort S;
    if (int rc = sort_strings<OW>(offs, vals, rows, n, max_len, S, s)) return rc;
    const int64_t nd = S.distinct;
    ROGTK_REQUIRE(n_reg + nd < (1ll << 32) - 1, ROGTK_E_UNSUPPORTED, "irregular merge: more than 2^32 vertices");
    // distinct strings: representative rows, lengths -> record offsets
    size_t scan_b = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (int64_t*)nullptr, (int64_t*)nullptr, (int)nd, s));
    Arena D;
    if (int rc = D.get(3 * al((size_t)(nd + 1) * 8) + al(scan_b) + 256, s)) return rc;
    int64_t* rep = D.take<int64_t>(nd);
    int64_t* dlen = D.take<int64_t>(nd + 1);
    int64_t* roff = D.take<int64_t>(nd + 1);
    unsigned long long* cnt = D.take<unsigned long long>(4);  // edges, overflow
    void* stmp = D.take<uint8_t>((int64_t)scan_b);
    ROGTK_HIP_CHECK(hipMemsetAsync(dlen + nd, 0, 8, s));
    ROGTK_HIP_CHECK(hipMemsetAsync(cnt, 0, 32, s));
    hipLaunchKernelGGL(k_distinct_rep<OW>, dim3(grid_for(n, 1ll << 31)), dim3(kBlock), 0, s, offs, rows, S.perm,
                       S.rank, S.flag, n, rep, dlen);
    size_t tb = scan_b;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(stmp, tb, dlen, roff, (int)(nd + 1), s));
    int64_t nr = 0;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&nr, roff + nd, 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    ROGTK_REQUIRE(nr < (1ll << 31), ROGTK_E_UNSUPPORTED, "irregular merge: more than 2^31 (string, position) records");
    const bool want_regular = lookup && L >= 1 && L <= 32 && n_reg > 0;
    size_t sort_b = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                       (uint64_t*)nullptr, (uint64_t*)nullptr, (int)std::max<int64_t>(nr, 1),
                                                       0, 64, s));
    const int64_t max_edges = nr + nd;
    Arena R;
    if (int rc = R.get(4 * al((size_t)nr * 8) + al(sort_b) + al((size_t)max_edges * 8) +
                           (want_regular ? al((size_t)nd * 32) + al((size_t)nd * 16) : 0) +
                           al((size_t)(n_reg + nd) * 4) + 256,
                       s))
        return rc;
    uint64_t* key = R.take<uint64_t>(nr);
    uint64_t* val = R.take<uint64_t>(nr);
    uint64_t* skey = R.take<uint64_t>(nr);
    uint64_t* sval = R.take<uint64_t>(nr);
    void* tmp = R.take<uint8_t>((int64_t)sort_b);
    uint2* E = R.take<uint2>(max_edges);
    uint64_t* q = want_regular ? R.take<uint64_t>(4 * nd) : nullptr;
    uint32_t* lab4 = want_regular ? R.take<uint32_t>(4 * nd) : nullptr;
    uint32_t* labels = R.take<uint32_t>(n_reg + nd);
    const uint32_t vbase = (uint32_t)n_reg;
    hipLaunchKernelGGL(k_records<OW>, dim3(grid_for(nd, 1ll << 31)), dim3(kBlock), 0, s, offs, vals, rep, roff, nd, L,
                       key, val, q);
    ROGTK_HIP_CHECK(hipGetLastError());
    if (nr > 1) {
        size_t b = sort_b;
        ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, b, key, skey, val, sval, (int)nr, 0, 64, s));
        hipLaunchKernelGGL(k_masked_edges<OW>, dim3(grid_for(nr, 16384)), dim3(kBlock), 0, s, offs, vals, rep, skey,
                           sval, nr, vbase, E, cnt, (unsigned int*)(cnt + 1));
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    if (want_regular) {
        if (int rc = (*lookup)(q, 4 * nd, lab4, s)) return rc;
        hipLaunchKernelGGL(k_regular_edges, dim3(grid_for(nd, 16384)), dim3(kBlock), 0, s, lab4, nd, vbase, E, cnt);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    unsigned long long h[2];
    ROGTK_HIP_CHECK(hipMemcpyAsync(h, cnt, 16, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    ROGTK_REQUIRE(!(h[1] & 0xFFFFFFFFull), ROGTK_E_UNSUPPORTED,
                  "irregular merge: a masked-key run longer than %d records (hash collisions)", kMaxRunWalk);
    const int64_t m = (int64_t)h[0];
    int64_t k = 0;
    if (int rc = rogtk_cc_labels(n_reg + nd, (const uint32_t*)E, m, labels, &k, s)) return rc;
    if (n_reg > 0 && relabel && relabel_n > 0) {
        uint32_t lastreg = 0;
        ROGTK_HIP_CHECK(hipMemcpyAsync(&lastreg, labels + n_reg - 1, 4, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipStreamSynchronize(s));
        if (lastreg != (uint32_t)(n_reg - 1))  // some regular clusters merged: remap their ids
            hipLaunchKernelGGL(k_relabel, dim3(grid_for(relabel_n, 16384)), dim3(kBlock), 0, s, relabel, relabel_n,
                               labels, (uint32_t)n_reg);
    }
    hipLaunchKernelGGL(k_irr_write, dim3(grid_for(n, 1ll << 31)), dim3(kBlock), 0, s, rows, S.perm, S.rank, S.flag, n,
                       labels, vbase, cluster_id);
    ROGTK_HIP_CHECK(hipGetLastError());
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    *n_clusters = k;
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
        return run_exact<4>(offsets, values, rows, n_rows, max_len, stats_dev, cluster_id, n_irregular_clusters, s);
    return run_exact<8>(offsets, values, rows, n_rows, max_len, stats_dev, cluster_id, n_irregular_clusters, s);
}

int irregular_merge(const void* offsets, int offset_width, const uint8_t* values, const int64_t* rows,
                    int64_t n_rows, int64_t max_len, int L, int64_t n_reg, const CodeLookup* lookup,
                    uint32_t* relabel, int64_t relabel_n, uint32_t* cluster_id, int64_t* n_clusters, hipStream_t s) {
    *n_clusters = n_reg;
    if (n_rows <= 0) return ROGTK_OK;
    ROGTK_REQUIRE(n_rows < (1ll << 31), ROGTK_E_UNSUPPORTED, "irregular rows: more than 2^31");
    ROGTK_REQUIRE(n_reg >= 0 && n_reg < (1ll << 32), ROGTK_E_INVALID, "irregular merge: bad regular cluster count");
    ProfScope prof(K_IRREGULAR, s);
    if (offset_width == 4)
        return run_merge<4>(offsets, values, rows, n_rows, max_len, L, n_reg, lookup, relabel, relabel_n, cluster_id,
                            n_clusters, s);
    return run_merge<8>(offsets, values, rows, n_rows, max_len, L, n_reg, lookup, relabel, relabel_n, cluster_id,
                        n_clusters, s);
}

int sorted_code_lookup(const uint64_t* G, int64_t ng, const uint32_t* labels, const uint64_t* q, int64_t nq,
                       uint32_t* lab, hipStream_t s) {
    if (nq <= 0) return ROGTK_OK;
    hipLaunchKernelGGL(k_sorted_lookup, dim3(grid_for(nq, 16384)), dim3(kBlock), 0, s, G, ng, labels, q, nq, lab);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

}  // namespace rogtk
