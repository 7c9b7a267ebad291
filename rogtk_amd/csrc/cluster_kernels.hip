// cluster_kernels.hip — H3 UMI cluster assignment on gfx950 (spec: DESIGN.md §H3).
//
// The reference has no clustering of its own: exact grouping is the caller's
// polars group_by('umi') (rogtk/__init__.py:206-214). This build assigns dense
// cluster ids over the packed SoA, exactly (max_distance 0) or as connected
// components of the Hamming<=1 graph (max_distance 1), deterministically and
// identically for any number of shards.
//
// Pipeline (all tables indexed by the 2-bit code, 4^L entries, L <= 16):
//   mark      presence[code] = 1 (plain byte stores; fused into k_score_packed)
//   bitmap    presence bytes -> 64-bit words (+ clears presence for the next batch)
//   scan      OR of n shard bitmaps -> global bitmap G, per-word in-block prefix
//             popcounts + block totals; second kernel scans block totals
//             => rank(code) = blkoff[w>>10] + wpref[w] + popc(G[w] & below(code))
//   compact   D[rank] = code (sorted distinct UMIs), parent[rank] = rank
//   union     per distinct UMI: probe its 3L single-substitution neighbours that
//             are smaller codes, lock-free union-find (agent-scope atomicCAS,
//             larger root hooked under smaller => root = smallest code)
//   flatten   parent[i] = find(i); ballot root flags into an index-space bitmap
//   scan      rank of roots (dense cluster ids in smallest-code order)
//   label     label_by_code[D[i]] (L <= 13) or parent[i] := dense id
//   assign    cluster_id[row] = label(code[row])
#include "rogtk_internal.h"

namespace rogtk {
namespace {

constexpr int kBlock = 256;
constexpr int kScanWords = 1024;  // words per scan block (4 per thread)

enum StatSlot { S_NDISTINCT = 0, S_NCLUSTERS = 1, S_OVERFLOW = 2, S_ERROR = 3 };

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Path-halving find. Every parent pointer is <= its index (we only ever hook a
// larger root under a smaller one), so stale reads still name an ancestor.
__device__ __forceinline__ uint32_t uf_find(uint32_t* parent, uint32_t x) {
    for (;;) {
        const uint32_t p = ld_agent(parent + x);
        if (p == x) return x;
        const uint32_t gp = ld_agent(parent + p);
        if (gp == p) return p;
        st_agent(parent + x, gp);
        x = gp;
    }
}

__device__ __forceinline__ void uf_unite(uint32_t* parent, uint32_t a, uint32_t b) {
    for (;;) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a < b) {
            const uint32_t t = a;
            a = b;
            b = t;
        }
        uint32_t expected = a;
        if (__hip_atomic_compare_exchange_strong(parent + a, &expected, b, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return;
        // `a` was hooked by someone else meanwhile: retry from the new roots.
    }
}

__device__ __forceinline__ uint32_t rank_of(const uint64_t* __restrict__ G,
                                            const uint32_t* __restrict__ wpref,
                                            const uint32_t* __restrict__ blkoff, uint64_t code) {
    const uint64_t w = code >> 6;
    const uint64_t below = (1ull << (code & 63)) - 1ull;
    return blkoff[w / kScanWords] + wpref[w] + (uint32_t)__popcll(G[w] & below);
}

// presence bytes -> bitmap words; one lane loads 16 contiguous bytes, 4 lanes make a word.
__global__ __launch_bounds__(kBlock) void k_bitmap_wide(uint8_t* __restrict__ pres, int64_t words,
                                                        uint64_t* __restrict__ out) {
    const int64_t lane_g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t w = lane_g >> 2;
    uint32_t m16 = 0;
    if (w < words) {
        uint4* p = reinterpret_cast<uint4*>(pres) + lane_g;
        const uint4 v = *p;
        const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t b = x[q] & 0x01010101u;  // presence bytes are 0 or 1
            m16 |= ((b | (b >> 7) | (b >> 14) | (b >> 21)) & 0xFu) << (4 * q);
        }
        if (v.x | v.y | v.z | v.w) *p = make_uint4(0, 0, 0, 0);
    }
    uint64_t word = (uint64_t)m16 << (16 * (threadIdx.x & 3));
    word |= __shfl_xor(word, 1);
    word |= __shfl_xor(word, 2);
    if ((threadIdx.x & 3) == 0 && w < words) out[w] = word;
}

__global__ void k_bitmap_small(uint8_t* __restrict__ pres, uint64_t nbits, uint64_t* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t m = 0;
    for (uint64_t b = 0; b < nbits; ++b) {
        if (pres[b]) m |= 1ull << b;
        pres[b] = 0;
    }
    out[0] = m;
}

// Block-wide exclusive scan of one value per thread (256 threads = 4 waves).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_wave, uint32_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(incl, off);
        if (lane >= off) incl += t;
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) {
        const uint32_t s = s_wave[k];
        if (k < wave) before += s;
        total += s;
    }
    __syncthreads();
    return before + incl - v;
}

// OR n_bitmaps shard bitmaps, write G (optional), per-word in-block prefix + block sums.
// words_dev != nullptr: the live word count is ceil(*words_dev / 64) (index space).
__global__ __launch_bounds__(kBlock) void k_scan_words(const uint64_t* __restrict__ bitmaps,
                                                       int n_bitmaps, int64_t words,
                                                       const unsigned long long* __restrict__ count_dev,
                                                       uint64_t* __restrict__ G,
                                                       uint32_t* __restrict__ wpref,
                                                       uint32_t* __restrict__ blksum) {
    __shared__ uint32_t s_wave[kBlock / 64];
    int64_t live = words;
    if (count_dev) live = min<int64_t>(words, (int64_t)((*count_dev + 63) / 64));
    const int64_t w0 = (int64_t)blockIdx.x * kScanWords + 4 * threadIdx.x;
    uint32_t c[4];
    uint32_t tsum = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t w = w0 + k;
        uint64_t v = 0;
        if (w < live)
            for (int r = 0; r < n_bitmaps; ++r) v |= bitmaps[(int64_t)r * words + w];
        if (G && w < words) G[w] = v;
        c[k] = (uint32_t)__popcll(v);
        tsum += c[k];
    }
    uint32_t total;
    uint32_t ex = block_excl_scan(tsum, s_wave, total);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t w = w0 + k;
        if (w < words) wpref[w] = ex;
        ex += c[k];
    }
    if (threadIdx.x == 0) blksum[blockIdx.x] = total;
}

// Single-block exclusive scan of block sums -> blkoff[0..nblocks], total -> stats.
__global__ __launch_bounds__(kBlock) void k_scan_blocks(const uint32_t* __restrict__ blksum,
                                                        int64_t nblocks, uint32_t* __restrict__ blkoff,
                                                        unsigned long long* __restrict__ stats,
                                                        int slot, int copy_slot) {
    __shared__ uint32_t s_wave[kBlock / 64];
    uint32_t carry = 0;
    for (int64_t base = 0; base < nblocks; base += kBlock) {
        const int64_t b = base + threadIdx.x;
        const uint32_t v = b < nblocks ? blksum[b] : 0u;
        uint32_t total;
        const uint32_t ex = block_excl_scan(v, s_wave, total);
        if (b < nblocks) blkoff[b] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) {
        blkoff[nblocks] = carry;
        stats[slot] = carry;
        if (copy_slot >= 0) stats[copy_slot] = carry;
    }
}

__global__ __launch_bounds__(kBlock) void k_compact(const uint64_t* __restrict__ G, int64_t words,
                                                    const uint32_t* __restrict__ wpref,
                                                    const uint32_t* __restrict__ blkoff,
                                                    uint32_t* __restrict__ D, uint32_t* __restrict__ parent,
                                                    uint32_t* __restrict__ labelcode, int64_t max_distinct,
                                                    unsigned long long* __restrict__ stats) {
    const int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (w >= words) return;
    uint64_t m = G[w];
    if (!m) return;
    uint32_t idx = blkoff[w / kScanWords] + wpref[w];
    while (m) {
        const int b = __ffsll((long long)m) - 1;
        m &= m - 1;
        const uint32_t code = (uint32_t)((w << 6) + b);
        if ((int64_t)idx < max_distinct) {
            D[idx] = code;
            parent[idx] = idx;
            if (labelcode) labelcode[code] = idx;  // exact mode: label = rank
        } else {
            stats[S_OVERFLOW] = 1;
        }
        ++idx;
    }
}

__global__ __launch_bounds__(kBlock) void k_union(const uint64_t* __restrict__ G,
                                                  const uint32_t* __restrict__ wpref,
                                                  const uint32_t* __restrict__ blkoff,
                                                  const uint32_t* __restrict__ D, uint32_t* parent,
                                                  int64_t max_distinct, int L,
                                                  const unsigned long long* __restrict__ stats) {
    const int64_t nd = min<int64_t>((int64_t)stats[S_NDISTINCT], max_distinct);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nd;
         i += (int64_t)gridDim.x * kBlock) {
        const uint32_t c = D[i];
        for (int p = 0; p < L; ++p) {
            const uint32_t sh = 2 * p;
#pragma unroll
            for (uint32_t d = 1; d <= 3; ++d) {
                const uint32_t nb = c ^ (d << sh);
                if (nb >= c) continue;  // each edge once, from its larger end
                if (!((G[nb >> 6] >> (nb & 63)) & 1ull)) continue;
                uf_unite(parent, (uint32_t)i, rank_of(G, wpref, blkoff, nb));
            }
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_flatten(uint32_t* parent, int64_t max_distinct,
                                                    uint64_t* __restrict__ rbits,
                                                    const unsigned long long* __restrict__ stats) {
    const int64_t nd = min<int64_t>((int64_t)stats[S_NDISTINCT], max_distinct);
    const int lane = threadIdx.x & 63;
    const int64_t wave_g = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t nwaves = (int64_t)gridDim.x * (kBlock / 64);
    for (int64_t base = wave_g * 64; base < nd; base += nwaves * 64) {
        const int64_t i = base + lane;
        bool root = false;
        if (i < nd) {
            const uint32_t r = uf_find(parent, (uint32_t)i);
            parent[i] = r;
            root = r == (uint32_t)i;
        }
        const uint64_t m = __ballot(root);
        if (lane == 0) rbits[base >> 6] = m;
    }
}

__global__ __launch_bounds__(kBlock) void k_label(uint32_t* __restrict__ parent,
                                                  const uint32_t* __restrict__ D,
                                                  const uint64_t* __restrict__ rbits,
                                                  const uint32_t* __restrict__ rpref,
                                                  const uint32_t* __restrict__ rblkoff,
                                                  uint32_t* __restrict__ labelcode, int64_t max_distinct,
                                                  const unsigned long long* __restrict__ stats) {
    const int64_t nd = min<int64_t>((int64_t)stats[S_NDISTINCT], max_distinct);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nd;
         i += (int64_t)gridDim.x * kBlock) {
        const uint32_t lab = rank_of(rbits, rpref, rblkoff, parent[i]);
        if (labelcode) labelcode[D[i]] = lab;
        else parent[i] = lab;
    }
}

// mode 0: labelcode[code]; 1: parent[rank(code)] (labels by index; exact mode leaves
// parent[i] == i, so the same lookup serves both distances)
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_assign(const uint32_t* __restrict__ codes,
                                                   const uint64_t* __restrict__ regbits, int64_t n,
                                                   const uint32_t* __restrict__ labelcode,
                                                   const uint32_t* __restrict__ parent,
                                                   const uint64_t* __restrict__ G,
                                                   const uint32_t* __restrict__ wpref,
                                                   const uint32_t* __restrict__ blkoff,
                                                   uint32_t* __restrict__ out) {
    const int64_t row0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    if (row0 >= n) return;
    const bool full = row0 + 4 <= n;
    uint32_t c[4] = {0, 0, 0, 0};
    if (full) {
        const uint4 v = *reinterpret_cast<const uint4*>(codes + row0);
        c[0] = v.x; c[1] = v.y; c[2] = v.z; c[3] = v.w;
    } else {
        for (int k = 0; k < 4; ++k)
            if (row0 + k < n) c[k] = codes[row0 + k];
    }
    uint32_t reg = regbits ? (uint32_t)(regbits[row0 >> 6] >> (row0 & 63)) & 0xFu : 0xFu;
    uint32_t id[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        id[k] = 0xFFFFFFFFu;
        if ((reg >> k) & 1u) {
            if (MODE == 0) id[k] = labelcode[c[k]];
            else id[k] = parent[rank_of(G, wpref, blkoff, c[k])];
        }
    }
    if (full) {
        *reinterpret_cast<uint4*>(out + row0) = make_uint4(id[0], id[1], id[2], id[3]);
    } else {
        for (int k = 0; k < 4; ++k)
            if (row0 + k < n) out[row0 + k] = id[k];
    }
}

inline int grid_for(int64_t lanes, int64_t cap = 0) {
    int64_t g = (lanes + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (cap && g > cap) g = cap;
    return (int)g;
}

struct WsPtrs {
    unsigned long long* stats;
    uint8_t* presence;
    uint64_t* G;
    uint32_t *wpref, *blksum, *blkoff, *D, *parent;
    uint64_t* rbits;
    uint32_t *rpref, *rblksum, *rblkoff, *labelcode;
};

inline WsPtrs ws_ptrs(const ClusterLayout& cl, uint8_t* ws) {
    WsPtrs p;
    p.stats = (unsigned long long*)(ws + cl.off_stats);
    p.presence = ws + cl.off_presence;
    p.G = (uint64_t*)(ws + cl.off_bitmap);
    p.wpref = (uint32_t*)(ws + cl.off_wpref);
    p.blksum = (uint32_t*)(ws + cl.off_blksum);
    p.blkoff = (uint32_t*)(ws + cl.off_blkoff);
    p.D = (uint32_t*)(ws + cl.off_D);
    p.parent = (uint32_t*)(ws + cl.off_parent);
    p.rbits = (uint64_t*)(ws + cl.off_rbits);
    p.rpref = (uint32_t*)(ws + cl.off_rpref);
    p.rblksum = (uint32_t*)(ws + cl.off_rblksum);
    p.rblkoff = (uint32_t*)(ws + cl.off_rblkoff);
    p.labelcode = cl.label_by_code ? (uint32_t*)(ws + cl.off_labelcode) : nullptr;
    return p;
}

constexpr int64_t kPersistentGrid = 2048;  // 256 CUs x 8 blocks

}  // namespace

int cluster_layout(int L, int64_t max_distinct, ClusterLayout* o) {
    ROGTK_REQUIRE(L >= 1 && L <= kMaxPackedLen, ROGTK_E_UNSUPPORTED,
                  "cluster: umi_len %d outside 1..%d", L, kMaxPackedLen);
    ROGTK_REQUIRE(max_distinct >= 1 && max_distinct <= 0xFFFFFFFFll, ROGTK_E_INVALID,
                  "cluster: max_distinct %lld outside 1..2^32-1", (long long)max_distinct);
    ClusterLayout c{};
    c.L = L;
    c.nbits = 1ull << (2 * L);
    if ((uint64_t)max_distinct > c.nbits) max_distinct = (int64_t)c.nbits;
    c.max_distinct = max_distinct;
    c.words = (int64_t)((c.nbits + 63) / 64);
    c.blocks = (c.words + kScanWords - 1) / kScanWords;
    c.rwords = (max_distinct + 63) / 64;
    c.rblocks = (c.rwords + kScanWords - 1) / kScanWords;
    c.label_by_code = L <= 13;
    int64_t off = 0;
    auto take = [&](int64_t bytes) {
        const int64_t at = off;
        off += (bytes + 255) / 256 * 256;
        return at;
    };
    c.off_stats = take(64);
    c.off_presence = take((int64_t)(c.nbits < 64 ? 64 : c.nbits));
    c.off_bitmap = take(c.words * 8);
    c.off_wpref = take(c.words * 4);
    c.off_blksum = take(c.blocks * 4);
    c.off_blkoff = take((c.blocks + 1) * 4);
    c.off_D = take(max_distinct * 4);
    c.off_parent = take(max_distinct * 4);
    c.off_rbits = take(c.rwords * 8);
    c.off_rpref = take(c.rwords * 4);
    c.off_rblksum = take(c.rblocks * 4);
    c.off_rblkoff = take((c.rblocks + 1) * 4);
    c.off_labelcode = c.label_by_code ? take((int64_t)c.nbits * 4) : off;
    c.total = off;
    *o = c;
    return ROGTK_OK;
}

int launch_cluster_local_bitmap(const ClusterLayout& cl, uint8_t* ws, uint64_t* out, hipStream_t s) {
    WsPtrs p = ws_ptrs(cl, ws);
    ProfScope prof(K_BITMAP, s);
    if (cl.nbits >= 1024) {
        hipLaunchKernelGGL(k_bitmap_wide, dim3(grid_for(cl.words * 4)), dim3(kBlock), 0, s,
                           p.presence, cl.words, out);
    } else if (cl.nbits >= 64) {
        // 4^3..4^4 codes: still whole 16-byte groups
        hipLaunchKernelGGL(k_bitmap_wide, dim3(1), dim3(kBlock), 0, s, p.presence, cl.words, out);
    } else {
        hipLaunchKernelGGL(k_bitmap_small, dim3(1), dim3(64), 0, s, p.presence, cl.nbits, out);
    }
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

int launch_cluster_resolve(const ClusterLayout& cl, uint8_t* ws, const uint64_t* bitmaps,
                           int n_bitmaps, int max_distance, hipStream_t s) {
    WsPtrs p = ws_ptrs(cl, ws);
    ROGTK_HIP_CHECK(hipMemsetAsync(p.stats, 0, 64, s));
    {
        ProfScope prof(K_SCAN, s);
        hipLaunchKernelGGL(k_scan_words, dim3((unsigned)cl.blocks), dim3(kBlock), 0, s, bitmaps,
                           n_bitmaps, cl.words, (const unsigned long long*)nullptr, p.G, p.wpref,
                           p.blksum);
        hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kBlock), 0, s, p.blksum, cl.blocks,
                           p.blkoff, p.stats, (int)S_NDISTINCT,
                           max_distance == 0 ? (int)S_NCLUSTERS : -1);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    {
        ProfScope prof(K_COMPACT, s);
        hipLaunchKernelGGL(k_compact, dim3(grid_for(cl.words)), dim3(kBlock), 0, s, p.G, cl.words,
                           p.wpref, p.blkoff, p.D, p.parent,
                           max_distance == 0 ? p.labelcode : (uint32_t*)nullptr, cl.max_distinct,
                           p.stats);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    if (max_distance == 0) return ROGTK_OK;
    const int pg = grid_for(cl.max_distinct, kPersistentGrid);
    {
        ProfScope prof(K_UNION, s);
        hipLaunchKernelGGL(k_union, dim3(pg), dim3(kBlock), 0, s, p.G, p.wpref, p.blkoff, p.D,
                           p.parent, cl.max_distinct, cl.L, p.stats);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    {
        ProfScope prof(K_FLATTEN, s);
        hipLaunchKernelGGL(k_flatten, dim3(pg), dim3(kBlock), 0, s, p.parent, cl.max_distinct,
                           p.rbits, p.stats);
        hipLaunchKernelGGL(k_scan_words, dim3((unsigned)cl.rblocks), dim3(kBlock), 0, s,
                           p.rbits, 1, cl.rwords, p.stats + S_NDISTINCT, (uint64_t*)nullptr,
                           p.rpref, p.rblksum);
        hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kBlock), 0, s, p.rblksum, cl.rblocks,
                           p.rblkoff, p.stats, (int)S_NCLUSTERS, -1);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    {
        ProfScope prof(K_LABEL, s);
        hipLaunchKernelGGL(k_label, dim3(pg), dim3(kBlock), 0, s, p.parent, p.D, p.rbits, p.rpref,
                           p.rblkoff, p.labelcode, cl.max_distinct, p.stats);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    return ROGTK_OK;
}

int launch_cluster_assign(const ClusterLayout& cl, const uint8_t* ws, const uint32_t* codes,
                          const uint64_t* regular_bits, int64_t n, uint32_t* cluster_id,
                          hipStream_t s) {
    if (n <= 0) return ROGTK_OK;
    WsPtrs p = ws_ptrs(cl, const_cast<uint8_t*>(ws));
    ProfScope prof(K_ASSIGN, s);
    const int g = grid_for((n + 3) / 4);
    if (cl.label_by_code)
        hipLaunchKernelGGL(k_assign<0>, dim3(g), dim3(kBlock), 0, s, codes, regular_bits, n,
                           p.labelcode, p.parent, p.G, p.wpref, p.blkoff, cluster_id);
    else
        hipLaunchKernelGGL(k_assign<1>, dim3(g), dim3(kBlock), 0, s, codes, regular_bits, n,
                           p.labelcode, p.parent, p.G, p.wpref, p.blkoff, cluster_id);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

}  // namespace rogtk
