// cluster_kernels.hip — H3 UMI cluster assignment on gfx950 (spec: DESIGN.md §H3).
//
// The reference has no clustering of its own: exact grouping is the caller's
// polars group_by('umi') (rogtk/__init__.py:206-214). This build assigns dense
// cluster ids over the packed SoA, exactly (max_distance 0) or as connected
// components of the Hamming<=1 graph (max_distance 1), deterministically and
// identically for any number of shards.
//
// Tables are indexed by the 2-bit code (4^L entries, L <= 16) or by the rank of a
// code among the distinct codes ("index space"; rank order == lexicographic order).
//   mark    presence[code] = 1 (plain byte stores; fused into k_score_packed)
//   bitmap  presence bytes -> 64-bit words (+ clears presence for the next batch)
//   scan    OR of n shard bitmaps -> global bitmap G, in-block prefix popcounts,
//           block sums; one block scans the block sums
//   rt      RT[w] = {G[w], global prefix}: rank(code) = ONE 16-B load + popcount
//   local   (max_distance 1) one workgroup per 4^7 consecutive codes: all Hamming-1
//           edges at positions 0..6 stay inside it, so their union-find runs in
//           LDS; writes D (sorted distinct codes), f (global index of the local
//           root) and UR[w] (the root shared by all codes of word w, if any)
//   rounds  positions 7..L-1: bulk-synchronous hook + jump until no edge crosses
//           two stars. Edges are enumerated as cliques: codes that differ only at
//           position p >= 3 are <= 4 mutually adjacent codes at the SAME bit of 4
//           bitmap words spaced 4^(p-3) words apart, so a coalesced word-group
//           sweep sees every edge without per-vertex probes; uniform words need
//           one root load instead of one per code.
//           hook: every clique hooks its members' star roots under the smallest
//                 one (LDS-deduplicated per workgroup, then atomicMin)
//           jump: every vertex chases its parent to the root (stars again)
//           The smallest vertex of a component is never hooked, so converged
//           stars are rooted at each component's smallest code. synth-v1 at 10M
//           reads (1.08M distinct) converges in 3 productive rounds, at 80M reads
//           (6.9M distinct, 41% of 4^12) in 2.
//   roots   ballot root flags into an index-space bitmap; scan = dense cluster ids
//   label   labelcode[code] (L <= 13) or ilab[i] := dense id (index space)
//   assign  cluster_id[row] = label(code[row])
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include <atomic>
#include <thread>
#include <chrono>
#include <cstring>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

constexpr int kBlock = 256;
constexpr int kMarkParts = 8;     // XCD partitions of the code space (mark)
constexpr int kMarkChunks = 256;  // row chunks of the XCD-partitioned kernels; grid = 8 * chunks
constexpr int kScanWords = 1024;  // words per scan block (4 per thread)
constexpr int kLocal8Words = 1024;  // words per 8-position local tile (= one scan block)
constexpr int kLocal8Cap = 8192;    // present codes an 8-position tile may hold
constexpr int kLocal8BigCap = 16384;  // the same for the denser instance (1 workgroup per CU)
constexpr int kMaxRounds = 64;
constexpr int kRoundBatch = 4;

// stats block (int64 slots): 0 n_distinct, 1 n_clusters, 2 overflow, 3 error,
// 4 rounds run; round flags (u32 per round) follow at byte 64.
// S_P0: the first code position of the global phase (7, or 8 when every 4^8-code tile
// fits the 8-position local CC), chosen on the device by the first scan
// S_LCAP: with S_P0 = 8, which 8-position instance takes the tiles (0: <= 8192 codes per
// tile, 1: <= 16384, e.g. the union bitmap of 2-4 ranks' 10M-read batches)
// S_REDO: the one local-CC instance launched (chosen from the workspace's previous resolve)
// does not take this bitmap's tiling: cluster_finish redoes the local and global phases.
enum StatSlot { S_NDISTINCT = 0, S_NCLUSTERS = 1, S_OVERFLOW = 2, S_REDO = 3, S_ROUNDS = 4, S_P0 = 6,
                S_LCAP = 7 };
// stats (8 x int64; slot 5 unused), round flags (u32 per round) at byte 64
constexpr int kFlagsOff = 64;
constexpr int kStatsBytes = kFlagsOff + 4 * kMaxRounds;

__device__ __forceinline__ uint64_t rt_word(const uint4 e) { return (uint64_t)e.x | ((uint64_t)e.y << 32); }

__device__ __forceinline__ uint32_t rt_rank(const uint4 e, uint32_t code) {
    return e.z + (uint32_t)__popcll(rt_word(e) & ((1ull << (code & 63)) - 1ull));
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

// Block-wide exclusive scan of one value per thread (NT threads, NT / 64 waves).
template <int NT = kBlock>
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
    for (int k = 0; k < NT / 64; ++k) {
        const uint32_t s = s_wave[k];
        if (k < wave) before += s;
        total += s;
    }
    __syncthreads();
    return before + incl - v;
}

// OR n_bitmaps shard bitmaps, write G (optional), per-word in-block prefix + block sums.
// count_dev != nullptr: the live word count is ceil(*count_dev / 64) (index space).
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
    uint64_t v[4] = {0, 0, 0, 0};
    for (int r = 0; r < n_bitmaps; ++r) {  // the 4 words of a bitmap loaded together
        const uint64_t* b = bitmaps + (int64_t)r * words;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (w0 + k < live) v[k] |= b[w0 + k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t w = w0 + k;
        if (G && w < words) G[w] = v[k];
        c[k] = (uint32_t)__popcll(v[k]);
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

// One workgroup: exclusive scan of block sums -> blkoff[0..nblocks], total -> stats
// (zero_stats: the stats block and round flags are cleared first).
__device__ __forceinline__ void scan_block_sums(const uint32_t* blksum, int64_t nblocks, uint32_t* blkoff,
                                                unsigned long long* stats, int slot, int copy_slot, int zero_stats,
                                                uint32_t* s_wave) {
    if (zero_stats && threadIdx.x < kStatsBytes / 8) stats[threadIdx.x] = 0;  // stats + round flags
    __syncthreads();
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

// per_live > 0: only the blocks that hold live indices (ceil(stats[S_NDISTINCT] /
// per_live)) are scanned; later offsets are never read
// p0_L > 0 (the first scan of a resolve, umi_len p0_L): also choose the local tiling.
// A scan block (kScanWords = 1024 words) is exactly one 4^8-code tile, so the largest
// block sum says whether every such tile fits the 8-position local CC (stats[S_P0]).
__global__ __launch_bounds__(kBlock) void k_scan_blocks(const uint32_t* __restrict__ blksum,
                                                        int64_t nblocks, uint32_t* __restrict__ blkoff,
                                                        unsigned long long* __restrict__ stats,
                                                        int slot, int copy_slot, int zero_stats,
                                                        int64_t per_live = 0, int p0_L = 0,
                                                        bool local8_big_on = true) {
    __shared__ uint32_t s_wave[kBlock / 64];
    __shared__ unsigned int s_max;
    if (per_live > 0) nblocks = min<int64_t>(nblocks, ((int64_t)stats[S_NDISTINCT] + per_live - 1) / per_live);
    scan_block_sums(blksum, nblocks, blkoff, stats, slot, copy_slot, zero_stats, s_wave);
    if (p0_L > 0) {
        if (threadIdx.x == 0) s_max = 0;
        __syncthreads();
        unsigned int mx = 0;
        for (int64_t b = threadIdx.x; b < nblocks; b += kBlock) mx = max(mx, blksum[b]);
        atomicMax(&s_max, mx);
        __syncthreads();
        if (threadIdx.x == 0) {
            const bool big = s_max > (unsigned int)kLocal8Cap && local8_big_on;
            stats[S_P0] = (p0_L >= 8 && s_max <= (unsigned int)(big ? kLocal8BigCap : kLocal8Cap)) ? 8 : 7;
            stats[S_LCAP] = big ? 1 : 0;
        }
    }
}

// RT[w] = {word, rank of its first code}; also zeroes the index-space live bits
// (zero_words <= words) for local_cc.
__global__ __launch_bounds__(kBlock) void k_rt(const uint64_t* __restrict__ G, int64_t words,
                                               const uint32_t* __restrict__ wpref,
                                               const uint32_t* __restrict__ blkoff, uint4* __restrict__ RT,
                                               uint64_t* __restrict__ zero, int64_t zero_words) {
    const int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (w >= words) return;
    if (w < zero_words) zero[w] = 0;
    const uint64_t m = G[w];
    RT[w] = make_uint4((uint32_t)m, (uint32_t)(m >> 32), blkoff[w / kScanWords] + wpref[w], 0u);
}

// ---- single-pass scan (decoupled look-back): k_scan_words + k_scan_blocks + k_rt in one
// launch, two kernel boundaries fewer on the resolve chain. Block b publishes its popcount
// total in lb[b] (tag << 34 | status << 32 | value; status 1 = aggregate, 2 = inclusive
// prefix), then wave 0 reads the predecessors 64 at a time, newest first, until one holds
// an inclusive prefix. Status and value share one 64-bit word, so relaxed device-scope
// atomics suffice (no release / acquire fences: on gfx950 those write back / invalidate
// the whole L2, which the kernels running beside the resolve share). Workgroups are
// dispatched in order, so every predecessor is resident or done and the waits end. The
// tag (per workspace, new for every launch) makes flags of earlier launches invalid
// without a clearing pass.
// A wait is still bounded (max_polls, ~4M polls of ~64 clocks by default): a block that
// gives up computes its prefix itself from the input bitmaps (every block total is a
// function of the bitmaps alone), so the result never depends on scheduling and no error
// state exists. rogtk_cluster_set_lookback_polls(0) forces that path for every block
// (tests/test_gpu_parity.py::test_lookback_fallback_exact).
constexpr uint64_t kLbAgg = 1, kLbIncl = 2;
constexpr int kLbMaxPolls = 1 << 22;

__device__ __forceinline__ uint64_t lb_word(uint32_t tag, uint64_t status, uint32_t v) {
    return ((uint64_t)tag << 34) | (status << 32) | v;
}

// popcount of the OR of n_bitmaps bitmaps over words [w0, w1), summed over the block
// (every thread gets the sum); the look-back's fallback
__device__ uint32_t block_popcount_or(const uint64_t* __restrict__ bitmaps, int n_bitmaps, int64_t words,
                                      int64_t w0, int64_t w1, uint32_t* s_wave) {
    uint32_t c = 0;
    for (int64_t w = w0 + threadIdx.x; w < w1; w += kBlock) {
        uint64_t v = 0;
        for (int r = 0; r < n_bitmaps; ++r) v |= bitmaps[(int64_t)r * words + w];
        c += (uint32_t)__popcll(v);
    }
    uint32_t total;
    (void)block_excl_scan(c, s_wave, total);
    return total;
}

// Exclusive prefix of `total` over blocks 0..blockIdx.x-1 (every thread of the block gets
// it). A wait that reaches max_polls hands over to the block-wide fallback.
__device__ uint32_t lookback_excl(uint64_t* lb, uint32_t tag, uint32_t total, int max_polls,
                                  const uint64_t* __restrict__ bitmaps, int n_bitmaps, int64_t words,
                                  uint32_t* s_x, uint32_t* s_gave_up, uint32_t* s_wave) {
    const int b = blockIdx.x;
    if (threadIdx.x == 0) *s_gave_up = 0;
    __syncthreads();
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        if (b == 0) {
            if (lane == 0) {
                __hip_atomic_store(&lb[0], lb_word(tag, kLbIncl, total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                *s_x = 0;
            }
        } else {
            if (lane == 0)
                __hip_atomic_store(&lb[b], lb_word(tag, kLbAgg, total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint32_t excl = 0;
            bool gave_up = false;
            int j = b - 1;
            for (int polls = 0;; ++polls) {
                const int idx = j - lane;
                const uint64_t f = idx >= 0 ? __hip_atomic_load(&lb[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                            : lb_word(tag, kLbIncl, 0);
                const uint64_t st = (f >> 32) & 3;
                const bool ready = (uint32_t)(f >> 34) == tag && st != 0;
                const uint64_t incl = __ballot(ready && st == kLbIncl);
                const int fi = incl ? __ffsll((unsigned long long)incl) - 1 : 63;  // lanes 0..fi are needed
                const uint64_t need = fi == 63 ? ~0ull : ((2ull << fi) - 1);
                if (__ballot(!ready) & need) {
                    if (polls >= max_polls) {
                        gave_up = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint32_t v = lane <= fi ? (uint32_t)f : 0u;
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
                excl += v;
                if (incl) break;
                j -= 64;
            }
            if (lane == 0) {
                if (gave_up) {
                    *s_gave_up = 1;
                } else {
                    __hip_atomic_store(&lb[b], lb_word(tag, kLbIncl, excl + total), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    *s_x = excl;
                }
            }
        }
    }
    __syncthreads();
    if (*s_gave_up) {  // block-uniform: recount every word before this block
        const uint32_t excl = block_popcount_or(bitmaps, n_bitmaps, words, 0, (int64_t)b * kScanWords, s_wave);
        if (threadIdx.x == 0) {
            __hip_atomic_store(&lb[b], lb_word(tag, kLbIncl, excl + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *s_x = excl;
        }
        __syncthreads();
    }
    return *s_x;
}

// OR of n_bitmaps shard bitmaps -> RT[w] = {word, rank of its first code} directly (no G,
// in-block prefixes or block offsets in HBM); lroot's first zero_words words zeroed. The
// last block clears the stats block and writes n_distinct (slot, copy_slot) and the local
// tiling choice (as k_scan_blocks with p0_L).
__global__ __launch_bounds__(kBlock) void k_scan_rt(const uint64_t* __restrict__ bitmaps, int n_bitmaps,
                                                    int64_t words, uint4* __restrict__ RT,
                                                    uint64_t* __restrict__ zero, int64_t zero_words,
                                                    uint64_t* agg, uint64_t* lb, uint32_t tag,
                                                    unsigned long long* __restrict__ stats, int slot, int copy_slot,
                                                    int p0_L, bool local8_big_on, int max_polls) {
    __shared__ uint32_t s_wave[kBlock / 64];
    __shared__ uint32_t s_x, s_gave_up;
    __shared__ unsigned int s_max;
    const int64_t w0 = (int64_t)blockIdx.x * kScanWords + 4 * threadIdx.x;
    uint64_t v[4] = {0, 0, 0, 0};
    if (w0 + 4 <= words) {  // a thread's 4 words: two 16-byte loads per bitmap, all in flight
        for (int r = 0; r < n_bitmaps; ++r) {
            const uint4* bm = reinterpret_cast<const uint4*>(bitmaps + (int64_t)r * words + w0);
            const uint4 x = bm[0], y = bm[1];
            v[0] |= x.x | ((uint64_t)x.y << 32);
            v[1] |= x.z | ((uint64_t)x.w << 32);
            v[2] |= y.x | ((uint64_t)y.y << 32);
            v[3] |= y.z | ((uint64_t)y.w << 32);
        }
    } else {
        for (int r = 0; r < n_bitmaps; ++r)
            for (int k = 0; k < 4; ++k)
                if (w0 + k < words) v[k] |= bitmaps[(int64_t)r * words + w0 + k];
    }
    uint32_t c[4], tsum = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        c[k] = (uint32_t)__popcll(v[k]);
        tsum += c[k];
        if (w0 + k < zero_words) zero[w0 + k] = 0;
    }
    uint32_t total;
    uint32_t ex = block_excl_scan(tsum, s_wave, total);
    if (threadIdx.x == 0)  // the block's total, tagged, for the last block's maximum
        __hip_atomic_store(&agg[blockIdx.x], ((uint64_t)tag << 32) | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ex += lookback_excl(lb, tag, total, max_polls, bitmaps, n_bitmaps, words, &s_x, &s_gave_up, s_wave);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t w = w0 + k;
        if (w < words) RT[w] = make_uint4((uint32_t)v[k], (uint32_t)(v[k] >> 32), ex, 0u);
        ex += c[k];
    }
    if (blockIdx.x != gridDim.x - 1) return;
    // the last block: the largest block total (a block whose total is not published within
    // max_polls is recounted from the bitmaps by this thread)
    const uint32_t n_distinct = s_x + total;
    if (threadIdx.x == 0) s_max = 0;
    __syncthreads();
    unsigned int mx = 0;
    for (int64_t b = threadIdx.x; b < gridDim.x; b += kBlock) {
        uint64_t a = __hip_atomic_load(&agg[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int polls = 0; (uint32_t)(a >> 32) != tag && polls < max_polls; ++polls) {
            __builtin_amdgcn_s_sleep(1);
            a = __hip_atomic_load(&agg[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        uint32_t t = (uint32_t)a;
        if ((uint32_t)(a >> 32) != tag) {
            t = 0;
            const int64_t e = min<int64_t>(words, (b + 1) * kScanWords);
            for (int64_t w = b * kScanWords; w < e; ++w) {
                uint64_t x = 0;
                for (int r = 0; r < n_bitmaps; ++r) x |= bitmaps[(int64_t)r * words + w];
                t += (uint32_t)__popcll(x);
            }
        }
        mx = max(mx, (unsigned int)t);
    }
    atomicMax(&s_max, mx);
    __syncthreads();
    if (threadIdx.x < kStatsBytes / 8) stats[threadIdx.x] = 0;  // stats + round flags
    __syncthreads();
    if (threadIdx.x == 0) {
        stats[slot] = n_distinct;
        if (copy_slot >= 0) stats[copy_slot] = n_distinct;
        if (p0_L > 0) {
            const bool big = s_max > (unsigned int)kLocal8Cap && local8_big_on;
            stats[S_P0] = (p0_L >= 8 && s_max <= (unsigned int)(big ? kLocal8BigCap : kLocal8Cap)) ? 8 : 7;
            stats[S_LCAP] = big ? 1 : 0;
        }
    }
}

// D[rank] = code (the sorted distinct UMIs) and f[rank] = rank. Lane per code: the
// 64 lanes of a wave share one RT entry (one load), present lanes store coalesced.
__global__ __launch_bounds__(kBlock) void k_build_d(const uint4* __restrict__ RT, uint64_t nbits,
                                                    uint32_t* __restrict__ D, uint32_t* __restrict__ f,
                                                    uint32_t* __restrict__ labelcode, uint32_t* __restrict__ ilab,
                                                    int64_t max_distinct,
                                                    unsigned long long* __restrict__ stats) {
    if ((int64_t)stats[S_NDISTINCT] > max_distinct && blockIdx.x == 0 && threadIdx.x == 0) stats[S_OVERFLOW] = 1;
    for (uint64_t c = (uint64_t)blockIdx.x * kBlock + threadIdx.x; c < nbits; c += (uint64_t)gridDim.x * kBlock) {
        const uint4 e = RT[c >> 6];
        if (!((rt_word(e) >> (c & 63)) & 1ull)) continue;
        const uint32_t i = rt_rank(e, (uint32_t)c);
        if ((int64_t)i >= max_distinct) continue;
        f[i] = i;
        D[i] = (uint32_t)c;
        if (labelcode) labelcode[c] = i;  // exact mode: label = rank
        else ilab[i] = i;
    }
}

__device__ __forceinline__ uint64_t multi_of4(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
    return (a & b) | (a & c) | (a & d) | (b & c) | (b & d) | (c & d);
}

// ---------------------------------------------------------------- local CC
// One workgroup owns a tile of 4^LP consecutive codes (4^LP / 64 bitmap words): every
// Hamming-1 edge at positions 0..LP-1 stays inside it, so the components over those
// positions are found in LDS (local_cc_tile below). Outputs are per word (UR[w] = the
// shared local root of word w when all its codes are in one local component, the common
// case once the code space is dense), the live vertices as bits of index space (lroot,
// zeroed before: the local roots and the codes of the other words), and f over index space
// for the live vertices.
#ifdef ROGTK_LCC_TIMING  // experiment builds (tools/lcc_timing.py): per-phase clocks of k_local_cc
__device__ unsigned long long g_lcc_clk[8];
#define LCC_T(k) do { __syncthreads(); if (threadIdx.x == 0) { const unsigned long long now_ = wall_clock64(); \
    atomicAdd(&g_lcc_clk[k], now_ - t_last_); t_last_ = now_; } } while (0)
#else
#define LCC_T(k) do { } while (0)
#endif
constexpr int kLocalWords = 256;
constexpr int kLocalCodes = kLocalWords * 64;  // 16384
constexpr int kLocalPos = 7;
constexpr uint32_t kNone = 0xFFFFFFFFu;

// relaxed workgroup-scope LDS load (the SV rounds below read parents other threads hook)
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// LDS union-find (coherent inside the workgroup; the dense 7-position tiles): path-halving
// find, CAS hook of the larger root under the smaller, so a component's root is its
// smallest local rank, as the SV rounds' rule
__device__ __forceinline__ uint32_t lfind(uint32_t* lf, uint32_t x) {
    for (;;) {
        const uint32_t p = lds_ld(lf + x);
        if (p == x) return x;
        const uint32_t gp = lds_ld(lf + p);
        if (gp == p) return p;
        __hip_atomic_store(lf + x, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        x = gp;
    }
}

__device__ __forceinline__ void lunite(uint32_t* lf, uint32_t a, uint32_t b) {
    for (;;) {
        a = lfind(lf, a);
        b = lfind(lf, b);
        if (a == b) return;
        if (a < b) {
            const uint32_t t = a;
            a = b;
            b = t;
        }
        uint32_t expected = a;
        if (__hip_atomic_compare_exchange_strong(lf + a, &expected, b, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP))
            return;
        a = expected;
    }
}

// Hamming-1 neighbours inside a 64-code word (positions 0..dims-1 of the code =
// bit strides 1, 4, 16 in groups of 4): any bit set in a group of 4 spreads to all 4.
__device__ __forceinline__ uint64_t word_spread(uint64_t x, int dims) {
    uint64_t s = x;
    const uint64_t g0 = (x | (x >> 1) | (x >> 2) | (x >> 3)) & 0x1111111111111111ull;
    s |= g0 * 0xFull;
    if (dims > 1) {
        const uint64_t g1 = (x | (x >> 4) | (x >> 8) | (x >> 12)) & 0x000F000F000F000Full;
        s |= g1 * 0x1111ull;
    }
    if (dims > 2) {
        const uint64_t g2 = (x | (x >> 16) | (x >> 32) | (x >> 48)) & 0xFFFFull;
        s |= g2 * 0x0001000100010001ull;
    }
    return s;
}

// the union of the components of word mask m that contain a bit of seed
__device__ __forceinline__ uint64_t word_component_any(uint64_t m, uint64_t seed, int dims) {
    uint64_t c = seed & m;
    for (;;) {  // <= 4 rounds: the 4x4x4 rook graph has diameter 3
        const uint64_t n = word_spread(c, dims) & m;
        if (n == c) return c;
        c = n;
    }
}

__device__ __forceinline__ uint64_t word_component(uint64_t m, uint64_t seed_bit, int dims) {
    return word_component_any(m, seed_bit, dims);
}

// The union-find runs over LOCAL RANKS (index - gbase) of the present codes, not over
// local codes: a tile of nloc present codes needs nloc LDS slots. Instances:
//  * LP = 8 (tiles of 4^8 codes = 1024 words, one thread per word, CAP 8192 ranks): when
//    every such tile holds at most 8192 codes (a sparse space, e.g. one 10M-read batch
//    at L = 12; decided on the device by the first scan, stats[S_P0] = 8). Position 7 is
//    then local too: 24% fewer local components and 41% fewer crossing pairs for the
//    global rounds, which start at position 8.
//  * LP = 7 (tiles of 4^7 codes = 256 words, CAP = kLocalCodes: 64 KB) otherwise, e.g. the
//    merged bitmap of 8 ranks, or a skewed sparse space with a crowded 4^8 tile.
// (Round 2 also had a 16 KB LP = 7 instance for the small tiles of a sparse space: 6.5%
// dense 68 -> 51 us; the LP = 8 tiling now takes those spaces, so it was dropped - its
// empty launch cost ~5 us of every resolve.)

// Pairs of present codes of word mask m that differ only at in-word position q (bit stride
// 4^q) by d in 1..3 (the lower code's digit + d <= 3): bit b set <=> codes b and b + d * 4^q.
__device__ __forceinline__ uint64_t inword_pairs(uint64_t m, int q, int d) {
    const uint64_t keep = q == 0 ? (d == 1 ? 0x7777777777777777ull : d == 2 ? 0x3333333333333333ull
                                                                            : 0x1111111111111111ull)
                        : q == 1 ? (d == 1 ? 0x0FFF0FFF0FFF0FFFull : d == 2 ? 0x00FF00FF00FF00FFull
                                                                            : 0x000F000F000F000Full)
                                 : (d == 1 ? 0x0000FFFFFFFFFFFFull : d == 2 ? 0x00000000FFFFFFFFull
                                                                            : 0x000000000000FFFFull);
    return m & (m >> (d << (2 * q))) & keep;
}

// One tile of TW words at word `base` (the body of k_local_cc), NT threads, WPT = TW / NT
// consecutive words per thread. Edge-centric (round 5): every Hamming-1 edge of the tile
// (positions 0..lpos-1) between local ranks, except that a word whose codes already form
// one component over the in-word positions (a BFS from its first code reaches all of them)
// is a single vertex: its codes point at its first code, and a pair of such words that share
// a bit is one edge. The edges go to an LDS list and are resolved by uniform hook + jump
// rounds (round 4 united in-word component lists with one union-find chain per pair: 48 us
// per workgroup at C2, most of it divergent, dependent LDS chains; the outputs are
// identical):
//   1. ranks (block scan), word masks, one-component flags, lf[r] = r (or the word's first
//      code); 2a. the edge list; 2b. hook + jump rounds until no edge crosses two roots;
//   3. outputs; 4. the live bits of index space by ballots over the codes' live marks
//      (lf bit 31).
// Roots are the smallest local rank of each component (hooks put the larger root under
// the smaller), so the labels are those of the global phase's smallest-vertex rule.
template <int CAP, int TW, int LP, int NT, int ECAP>
__device__ __forceinline__ void local_cc_tile(const int64_t base, const uint4* __restrict__ RT, int64_t words, int L,
                                              uint32_t* __restrict__ f, uint32_t* __restrict__ UR,
                                              uint64_t* __restrict__ lroot, int64_t rwords, int64_t max_distinct,
                                              unsigned long long* __restrict__ stats) {
    constexpr int WPT = TW / NT;
    static_assert(WPT * NT == TW && WPT >= 1, "words per thread");
    constexpr uint32_t kLive = 0x80000000u;
    __shared__ uint64_t wb[TW];
    __shared__ uint32_t lpre[TW];
    __shared__ uint8_t wone[TW];
    __shared__ uint32_t lf[CAP];  // by local rank: parent, then root | kLive
    __shared__ uint32_t edges[ECAP];  // a | b << 16 (local ranks < 2^16)
    __shared__ uint32_t s_wave[NT / 64];
    __shared__ uint32_t s_ch[2];
    const int t = threadIdx.x, lane = t & 63;
#ifdef ROGTK_LCC_TIMING
    const unsigned long long t_entry_ = wall_clock64();
    unsigned long long t_last_ = t_entry_;
#endif
    const int nw = (int)min<int64_t>(TW, words - base);
    const int w0 = t * WPT;
    uint64_t m[WPT];
    uint32_t tsum = 0;
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
        m[i] = w0 + i < nw ? rt_word(RT[base + w0 + i]) : 0ull;
        tsum += (uint32_t)__popcll(m[i]);
    }
    uint32_t nloc;
    uint32_t ex[WPT];
    ex[0] = block_excl_scan<NT>(tsum, s_wave, nloc);
#pragma unroll
    for (int i = 1; i < WPT; ++i) ex[i] = ex[i - 1] + (uint32_t)__popcll(m[i - 1]);
    const uint32_t gbase = RT[base].z;
    if (nloc > (uint32_t)CAP) {  // the scan's tiling choice rules this out
        if (t == 0) stats[S_OVERFLOW] = 1;
        return;
    }
    const int lpos = L < LP ? L : LP;
    const int indims = lpos < 3 ? lpos : 3;  // positions inside one 64-code word
    bool one[WPT];
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
        const int cnt = __popcll(m[i]);
        one[i] = cnt <= 1 || (indims > 0 && word_component(m[i], m[i] & (~m[i] + 1ull), indims) == m[i]);
        wb[w0 + i] = m[i];
        lpre[w0 + i] = ex[i];
        wone[w0 + i] = one[i];
        for (int j = 0; j < cnt; ++j) lf[ex[i] + j] = one[i] ? ex[i] : ex[i] + j;
    }
    if (t < 2) s_ch[t] = 0;
    __syncthreads();
    LCC_T(0);
    // 2a. the tile's edges: in-word pairs of the words that are not one component, then the
    //     cross-word pairs at positions 3..lpos-1 (word w and w + d * 4^(p-3), same bit; one
    //     edge between two one-component words), as (a | b << 16) over local ranks into the
    //     edge list (past its capacity: in batches, 2b)
    auto rank_of = [](uint32_t pre, uint64_t mask, int b) {
        return pre + (uint32_t)__popcll(mask & ((1ull << b) - 1ull));
    };
    auto for_edges = [&](auto&& emit) {
#pragma unroll
        for (int i = 0; i < WPT; ++i) {
            const uint64_t mi = m[i];
            if (!mi) continue;
            const int w = w0 + i;
            if (!one[i]) {
                for (int q = 0; q < indims; ++q)
                    for (int d = 1; d <= 3; ++d) {
                        uint64_t e = inword_pairs(mi, q, d);
                        while (e) {
                            const int b = __ffsll((long long)e) - 1;
                            e &= e - 1;
                            emit(rank_of(ex[i], mi, b), rank_of(ex[i], mi, b + (d << (2 * q))));
                        }
                    }
            }
            for (int p = 3; p < lpos; ++p) {
                const int sh = 2 * (p - 3);
                const int a = (w >> sh) & 3;
                for (int d = 1; a + d <= 3; ++d) {
                    const int w2 = w + (d << sh);
                    const uint64_t m2 = wb[w2];
                    uint64_t z = mi & m2;
                    if (!z) continue;
                    const uint32_t pre2 = lpre[w2];
                    if (one[i] && wone[w2]) {
                        emit(ex[i], pre2);
                        continue;
                    }
                    while (z) {
                        const int b = __ffsll((long long)z) - 1;
                        z &= z - 1;
                        emit(one[i] ? ex[i] : rank_of(ex[i], mi, b), rank_of(pre2, m2, b));
                    }
                }
            }
        }
    };
    // the count pass by popcounts (no per-edge loop)
    uint32_t ecount = 0;
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
        const uint64_t mi = m[i];
        if (!mi) continue;
        const int w = w0 + i;
        if (!one[i])
            for (int q = 0; q < indims; ++q)
                for (int d = 1; d <= 3; ++d) ecount += (uint32_t)__popcll(inword_pairs(mi, q, d));
        for (int p = 3; p < lpos; ++p) {
            const int sh = 2 * (p - 3);
            const int a = (w >> sh) & 3;
            for (int d = 1; a + d <= 3; ++d) {
                const int w2 = w + (d << sh);
                const uint64_t z = mi & wb[w2];
                ecount += one[i] && wone[w2] ? (z ? 1u : 0u) : (uint32_t)__popcll(z);
            }
        }
    }
    uint32_t etot;
    const uint32_t ek0 = block_excl_scan<NT>(ecount, s_wave, etot);
    // 2b. hook + jump rounds over the listed edges (Shiloach-Vishkin in LDS): jump = every
    //     vertex to its root (stars); hook = for every edge whose ends' roots differ, the
    //     larger root under the smaller (atomicMin). Parents only ever point at smaller
    //     vertices, so a component's smallest local rank is never hooked and ends as its
    //     root. Uniform passes (vertices / edges dealt over the threads) instead of one
    //     union-find chain per edge; s_ch[r & 1] = some hook in round r (reset a round ahead).
    //     More edges than the list holds (dense tiles: words that are not one component list
    //     an edge per shared bit) go through in batches of ECAP, the edges re-enumerated per
    //     batch (round 6: the overflow used to be united by one union-find chain per edge,
    //     dependent LDS CAS loops: 525 us of local CC per step at 8 emulated ranks)
    int r = 0;
    for (uint32_t e0 = 0; e0 < etot || e0 == 0; e0 += (uint32_t)ECAP) {
        if (e0) __syncthreads();  // the previous batch's rounds read the list
        uint32_t ek = ek0;
        for_edges([&](uint32_t a, uint32_t b) {
            if (ek >= e0 && ek - e0 < (uint32_t)ECAP) edges[ek - e0] = a | (b << 16);
            ++ek;
        });
        __syncthreads();
        if (e0 == 0) LCC_T(1);
        const uint32_t ne = min(etot - min(etot, e0), (uint32_t)ECAP);
        for (;; ++r) {
            for (uint32_t v = t; v < nloc; v += NT) {
                uint32_t root = lf[v];
                if (root == v) continue;
                for (uint32_t q = lds_ld(lf + root); q != root; q = lds_ld(lf + root)) root = q;
                __hip_atomic_store(lf + v, root, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            __syncthreads();
            if (t == 0) s_ch[(r + 1) & 1] = 0;  // every thread read it after the previous round's barrier
            bool ch = false;
            for (uint32_t j = t; j < ne; j += NT) {
                const uint32_t ed = edges[j];
                const uint32_t ra = lds_ld(lf + (ed & 0xFFFFu)), rb = lds_ld(lf + (ed >> 16));
                if (ra != rb) {
                    atomicMin(lf + max(ra, rb), min(ra, rb));
                    ch = true;
                }
            }
            if (ch) s_ch[r & 1] = 1;
            __syncthreads();
            if (!s_ch[r & 1]) {
                ++r;
                break;  // no hook: the jump above left stars
            }
        }
    }
    LCC_T(2);
    // 3b. outputs of this thread's words: UR = the word's shared local root (global index)
    //     or kNone; f[root] = root; the codes of a word without a shared root are all live
    //     with f[i] = their root (the global rounds read them by code); live codes marked
    if (t == 0 && (int64_t)gbase + nloc > max_distinct) stats[S_OVERFLOW] = 1;
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
        const int w = w0 + i;
        if (w >= nw) continue;
        const int cnt = __popcll(m[i]);
        uint32_t first = kNone;
        bool uniform = true;
        for (int j = 0; j < cnt; ++j) {
            const uint32_t root = lf[ex[i] + j];
            if (j == 0) first = root;
            uniform &= root == first;
        }
        for (int j = 0; j < cnt; ++j) {
            const uint32_t r = ex[i] + j, root = lf[r];
            const int64_t gi = (int64_t)gbase + r;
            if (root == r || !uniform) {
                if (gi < max_distinct) f[gi] = gbase + root;
                lf[r] = root | kLive;
            }
        }
        UR[base + w] = (cnt && uniform) ? gbase + first : kNone;
    }
    __syncthreads();
    // 4. index-space live words: the block owns the interior words of its range; the first
    //    and last are shared with the neighbouring blocks (atomic OR, zeroed before)
    {
        const uint32_t off = gbase & 63u;
        const uint32_t nlw = nloc ? (off + nloc + 63u) / 64u : 0u;
        const int64_t lw0 = (int64_t)(gbase >> 6);
        for (uint32_t k = t >> 6; k < nlw; k += NT / 64) {
            const int64_t w = lw0 + k;
            const int64_t r = (int64_t)k * 64 + lane - off;
            const bool live = r >= 0 && r < (int64_t)nloc && (lf[r] & kLive);
            const uint64_t v = __ballot(live);
            if (lane == 0 && w < rwords) {
                if (k == 0 || k == nlw - 1) {
                    if (v) atomicOr((unsigned long long*)(lroot + w), (unsigned long long)v);
                } else {
                    lroot[w] = v;
                }
            }
        }
    }
    LCC_T(3);
#ifdef ROGTK_LCC_TIMING
    if (threadIdx.x == 0) {
        atomicAdd(&g_lcc_clk[4], wall_clock64() - t_entry_);  // the workgroup's whole duration
        atomicAdd(&g_lcc_clk[5], 1ull);                        // workgroups
    }
#endif
}

// The 7-position instance (tiles of 4^7 codes, one 64-code word per thread) for DENSE spaces
// (round 6: the union bitmap of several ranks, 25-41% of the codes present). A word's
// vertices are its in-word components (up to kComp; a word with more, i.e. scattered codes,
// keeps one vertex per code as local_cc_tile does): every code points at its component's
// first code, so no in-word edge is listed, a pair of words sharing bits lists one edge per
// pair of their components that share one, and the jumps visit the representatives only.
// local_cc_tile's per-code edges for a dense tile (every word that is not ONE component, 21%
// at 41% density, listed an edge per shared bit) took 146 us per workgroup, 380-525 us of
// local CC per step at 8 emulated ranks. Outputs as local_cc_tile.
constexpr int kComp = 4;
template <int CAP, int TW, int ECAP>
__device__ __forceinline__ void local_cc_tile7(const int64_t base, const uint4* __restrict__ RT, int64_t words, int L,
                                               uint32_t* __restrict__ f, uint32_t* __restrict__ UR,
                                               uint64_t* __restrict__ lroot, int64_t rwords, int64_t max_distinct,
                                               unsigned long long* __restrict__ stats) {
    constexpr int NT = TW;
    constexpr uint32_t kLive = 0x80000000u;
    __shared__ uint64_t wb[TW];
    __shared__ uint64_t wc[kComp][TW];  // component masks of the words with 1..kComp components
    __shared__ uint32_t lpre[TW];
    __shared__ uint8_t wk[TW];  // components (1..kComp), or 0: one vertex per code
    __shared__ uint32_t lf[CAP];
    __shared__ uint32_t s_wave[NT / 64];
    const int t = threadIdx.x, lane = t & 63;
#ifdef ROGTK_LCC_TIMING
    const unsigned long long t_entry_ = wall_clock64();
    unsigned long long t_last_ = t_entry_;
#endif
    const int nw = (int)min<int64_t>(TW, words - base);
    const int w = t;
    const uint64_t m = w < nw ? rt_word(RT[base + w]) : 0ull;
    uint32_t nloc;
    const uint32_t ex = block_excl_scan<NT>((uint32_t)__popcll(m), s_wave, nloc);
    const uint32_t gbase = RT[base].z;
    if (nloc > (uint32_t)CAP) {
        if (t == 0) stats[S_OVERFLOW] = 1;
        return;
    }
    const int lpos = L < 7 ? L : 7;
    const int indims = lpos < 3 ? lpos : 3;
    auto rank_of = [](uint32_t pre, uint64_t mask, int b) {
        return pre + (uint32_t)__popcll(mask & ((1ull << b) - 1ull));
    };
    // 1. components, ranks, parents
    uint64_t comp[kComp];
    int nc = 0;
    {
        uint64_t rest = m;
        while (rest && nc <= kComp) {
            const uint64_t c = indims > 0 ? word_component(m, rest & (~rest + 1ull), indims) : (rest & (~rest + 1ull));
            if (nc < kComp) comp[nc] = c;
            ++nc;
            rest &= ~c;
        }
    }
    const int kind = nc > kComp ? 0 : nc;
    uint32_t rep[kComp];
#pragma unroll
    for (int q = 0; q < kComp; ++q) {
        rep[q] = 0;
        if (q < kind) {
            rep[q] = rank_of(ex, m, __ffsll((long long)comp[q]) - 1);
            wc[q][w] = comp[q];
        }
    }
    wb[w] = m;
    lpre[w] = ex;
    wk[w] = (uint8_t)kind;
    if (kind == 0) {
        const int cnt = __popcll(m);
        for (int j = 0; j < cnt; ++j) lf[ex + j] = ex + j;
    } else {
#pragma unroll
        for (int q = 0; q < kComp; ++q) {
            if (q >= kind) break;
            uint64_t x = comp[q];
            while (x) {
                const int b = __ffsll((long long)x) - 1;
                x &= x - 1;
                lf[rank_of(ex, m, b)] = rep[q];
            }
        }
    }
    __syncthreads();
    LCC_T(0);
    // 2. unions, straight into the LDS union-find: the in-word pairs of per-code words, then
    //    positions 3..lpos-1 as tasks of one group of 4 words {w0 + v 4^(p-3)} each (codes at
    //    one bit of a group differ only at p): components of two words that share a bit are
    //    united; a group of one-component words unites each word with the first word of its
    //    linked group (<= 3 unions instead of one per linked pair; round 4's dense rule)
    auto rep_in = [&](int w2, uint64_t m2, uint32_t pre2, int k2, int b) -> uint32_t {
        if (k2 == 0) return rank_of(pre2, m2, b);
        for (int q = 0; q < k2; ++q) {
            const uint64_t c = wc[q][w2];
            if ((c >> b) & 1ull) return rank_of(pre2, m2, __ffsll((long long)c) - 1);
        }
        return rank_of(pre2, m2, b);  // (not reached: the components cover the word)
    };
    if (kind == 0 && m)
        for (int q = 0; q < indims; ++q)
            for (int d = 1; d <= 3; ++d) {
                uint64_t e = inword_pairs(m, q, d);
                while (e) {
                    const int b = __ffsll((long long)e) - 1;
                    e &= e - 1;
                    lunite(lf, rank_of(ex, m, b), rank_of(ex, m, b + (d << (2 * q))));
                }
            }
    const int per = nw >> 2;
    for (int task = t; per > 0 && task < (lpos - 3) * per; task += NT) {
        const int p = 3 + task / per, g = task % per, s2 = 2 * p - 6, stride = 1 << s2;
        const int wg0 = ((g >> s2) << (s2 + 2)) | (g & (stride - 1));
        uint64_t mv[4];
        uint32_t pv[4];
        int kv[4];
        bool all_one = true;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int wv = wg0 + v * stride;
            mv[v] = wb[wv];
            pv[v] = lpre[wv];
            kv[v] = wk[wv];
            all_one &= kv[v] == 1 || mv[v] == 0;
        }
        if (all_one) {
            uint32_t adj[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                adj[a] = 1u << a;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (b != a && (mv[a] & mv[b])) adj[a] |= 1u << b;
            }
#pragma unroll
            for (int it = 0; it < 2; ++it)  // closure: 4 nodes, diameter <= 3
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    uint32_t rr = adj[a];
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        if ((adj[a] >> b) & 1u) rr |= adj[b];
                    adj[a] = rr;
                }
#pragma unroll
            for (int a = 1; a < 4; ++a) {
                const int lead = __ffs((int)adj[a]) - 1;
                if (lead != a) lunite(lf, pv[lead], pv[a]);  // a one-component word's vertex: its first code
            }
        } else {
#pragma unroll
            for (int x = 0; x < 3; ++x)
#pragma unroll
                for (int y = x + 1; y < 4; ++y) {
                    uint64_t z = mv[x] & mv[y];
                    if (!z) continue;
                    const int wx = wg0 + x * stride, wy = wg0 + y * stride;
                    if (kv[x] > 0 && kv[y] > 0) {
                        for (int qx = 0; qx < kv[x]; ++qx) {
                            const uint64_t cx = wc[qx][wx];
                            if (!(cx & z)) continue;
                            for (int qy = 0; qy < kv[y]; ++qy) {
                                const uint64_t cy = wc[qy][wy];
                                if (cx & cy)
                                    lunite(lf, rank_of(pv[x], mv[x], __ffsll((long long)cx) - 1),
                                           rank_of(pv[y], mv[y], __ffsll((long long)cy) - 1));
                            }
                        }
                    } else {
                        while (z) {
                            const int b = __ffsll((long long)z) - 1;
                            z &= z - 1;
                            lunite(lf, rep_in(wx, mv[x], pv[x], kv[x], b), rep_in(wy, mv[y], pv[y], kv[y], b));
                        }
                    }
                }
        }
    }
    __syncthreads();
    LCC_T(1);
    if (kind == 0) {
        const int cnt = __popcll(m);
        for (int j = 0; j < cnt; ++j) lf[ex + j] = lfind(lf, ex + j);
    } else {
#pragma unroll
        for (int q = 0; q < kComp; ++q)
            if (q < kind) lf[rep[q]] = lfind(lf, rep[q]);
    }
    __syncthreads();
    LCC_T(2);
    // 3. outputs of this thread's word: a code's root is lf[its representative] (stars: the
    //    representatives were jumped last; codes of a component still point at theirs)
    if (t == 0 && (int64_t)gbase + nloc > max_distinct) stats[S_OVERFLOW] = 1;
    if (w < nw) {
        const int cnt = __popcll(m);
        uint32_t first = kNone;
        bool uniform = true;
        for (int j = 0; j < cnt; ++j) {
            const uint32_t root = lf[lf[ex + j]] & ~kLive;  // (another thread may mark a root live)
            if (j == 0) first = root;
            uniform &= root == first;
        }
        // f first, then the live marks (a mark would hide the representative's root)
        for (int j = 0; j < cnt; ++j) {
            const uint32_t rr = ex + j, root = lf[lf[rr]] & ~kLive;
            const int64_t gi = (int64_t)gbase + rr;
            if (root == rr || !uniform) {
                if (gi < max_distinct) f[gi] = gbase + root;
            }
        }
        for (int j = 0; j < cnt; ++j) {
            const uint32_t rr = ex + j;
            const uint32_t root = lf[lf[rr] & ~kLive] & ~kLive;
            if (root == rr || !uniform) lf[rr] = root | kLive;
        }
        UR[base + w] = (cnt && uniform) ? gbase + first : kNone;
    }
    __syncthreads();
    // 4. index-space live words (as local_cc_tile)
    {
        const uint32_t off = gbase & 63u;
        const uint32_t nlw = nloc ? (off + nloc + 63u) / 64u : 0u;
        const int64_t lw0 = (int64_t)(gbase >> 6);
        for (uint32_t k = t >> 6; k < nlw; k += NT / 64) {
            const int64_t lw = lw0 + k;
            const int64_t rr = (int64_t)k * 64 + lane - off;
            const bool live = rr >= 0 && rr < (int64_t)nloc && (lf[rr] & kLive);
            const uint64_t v = __ballot(live);
            if (lane == 0 && lw < rwords) {
                if (k == 0 || k == nlw - 1) {
                    if (v) atomicOr((unsigned long long*)(lroot + lw), (unsigned long long)v);
                } else {
                    lroot[lw] = v;
                }
            }
        }
    }
    LCC_T(3);
#ifdef ROGTK_LCC_TIMING
    if (threadIdx.x == 0) {
        atomicAdd(&g_lcc_clk[4], wall_clock64() - t_entry_);
        atomicAdd(&g_lcc_clk[5], 1ull);
    }
#endif
}

#ifndef ROGTK_LCC_NT8
#define ROGTK_LCC_NT8 1024  // threads of an 8-position local-CC workgroup (experiments)
#endif
// The 8192-code 1024-thread instance's VGPRs capped for 7 waves per SIMD (<= 72; the 8192-code instance
// compiles to 63 with no spills, against 79 uncapped), so its workgroups fit beside more of the
// concurrent kernels' waves (round 5, interleaved: 0.3085-0.3106 vs 0.3116-0.3147 ms/step)
#ifndef ROGTK_LCC_WPE
#define ROGTK_LCC_WPE 7
#endif
#define ROGTK_LCC_ATTR(CAP, NT) __attribute__((amdgpu_waves_per_eu(NT == 1024 && CAP <= 8192 ? ROGTK_LCC_WPE : 1, 8)))
template <int CAP, int TW, int LP, int NT = TW>
__global__ __launch_bounds__(NT) ROGTK_LCC_ATTR(CAP, NT) void k_local_cc(const uint4* __restrict__ RT, int64_t words, int L,
                                                 uint32_t* __restrict__ f, uint32_t* __restrict__ UR,
                                                 uint64_t* __restrict__ lroot, int64_t rwords,
                                                 int64_t max_distinct, unsigned long long* __restrict__ stats,
                                                 bool any_cap = false, bool alone = false) {
    // the other tiling, or the other 8-position instance (any_cap: this one takes both caps)
    const bool mine = ((int)stats[S_P0] == 8 ? 8 : 7) == LP &&
                      (LP != 8 || any_cap || (int)stats[S_LCAP] == (CAP > kLocal8Cap ? 1 : 0));
    if (!mine) {
        // launched alone on the previous resolve's tiling, which this bitmap does not take
        if (alone && blockIdx.x == 0 && threadIdx.x == 0) stats[S_REDO] = 1;
        return;
    }
    // edge-list capacity (more edges go through in batches): C2's sparse 4^8 tiles list ~0.8
    // edges per code; the 7-position tiling takes dense spaces, whose words are few
    // components each (~1.3 edges per word pair: ~2,000 per tile at 41% density, two
    // batches); 1024 keeps that instance at 2 workgroups per CU
    constexpr int kEcap = LP == 7 ? 1024 : CAP >= 16384 ? 12288 : 8192;
    if constexpr (LP == 7 && NT == TW)
        local_cc_tile7<CAP, TW, kEcap>((int64_t)blockIdx.x * TW, RT, words, L, f, UR, lroot, rwords, max_distinct,
                                       stats);
    else
        local_cc_tile<CAP, TW, LP, NT, kEcap>((int64_t)blockIdx.x * TW, RT, words, L, f, UR, lroot, rwords,
                                              max_distinct, stats);
}

// ROGTK_LOCAL8=0: never the 8-position local tiling (A/B)
inline bool local8_enabled() {
    static const bool on = [] {
        const char* e = getenv("ROGTK_LOCAL8");
        return !(e && e[0] == '0');
    }();
    return on;
}

// ROGTK_LOCAL8_BIG=0: no 8-position instance for tiles of 8193..16384 codes (A/B)
inline bool local8_big_enabled() {
    static const bool on = [] {
        const char* e = getenv("ROGTK_LOCAL8_BIG");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Every instance of k_local_cc (each exits early for the tiles of the others).
// choice (round 4): the instance the workspace's previous resolve used (0: 8 positions,
// <= 8192 codes per tile; 1: 8 positions, <= 16384; 2: 7 positions), launched alone (one
// launch instead of three: the others exit at once, but each costs a kernel boundary on
// the resolve chain); it flags S_REDO when the bitmap needs another one. -1: all.
inline void launch_local_cc(const uint4* RT, int64_t words, int L, uint32_t* f, uint32_t* UR, uint64_t* lroot,
                            int64_t rwords, int64_t max_distinct, unsigned long long* stats, hipStream_t s,
                            int choice = -1) {
    constexpr int kNT8 = ROGTK_LCC_NT8;
    const unsigned tiles8 = (unsigned)((words + kLocal8Words - 1) / kLocal8Words);
    const unsigned tiles7 = (unsigned)((words + kLocalWords - 1) / kLocalWords);
    const bool alone = choice >= 0;
    if (alone ? choice == 0 : L >= 8 && local8_enabled())
        ROGTK_TIMED_LAUNCH(K_K_LOCAL_CC, (k_local_cc<kLocal8Cap, kLocal8Words, 8, kNT8>), dim3(tiles8), dim3(kNT8), 0, s, RT,
                           words, L, f, UR, lroot, rwords, max_distinct, stats, false, alone);
    if (alone ? choice == 1 : L >= 8 && local8_enabled() && local8_big_enabled())
        ROGTK_TIMED_LAUNCH(K_K_LOCAL_CC, (k_local_cc<kLocal8BigCap, kLocal8Words, 8, kNT8>), dim3(tiles8), dim3(kNT8), 0, s, RT,
                           words, L, f, UR, lroot, rwords, max_distinct, stats, alone, alone);
    if (alone ? choice == 2 : true)
        ROGTK_TIMED_LAUNCH(K_K_LOCAL_CC, (k_local_cc<kLocalCodes, kLocalWords, 7>), dim3(tiles7), dim3(kLocalWords), 0, s, RT, words,
                           L, f, UR, lroot, rwords, max_distinct, stats, false, alone);
}

// --------------------------------------------------------------- global CC
// Per-workgroup hook table in LDS: (root -> smallest proposed parent). Cliques that
// cross stars insert here; the block flushes one global atomicMin per distinct root.
constexpr int kHookSlots = 1024;

struct HookTable {
    uint32_t key[kHookSlots];
    uint32_t val[kHookSlots];
};

__device__ __forceinline__ void hook_insert(HookTable& T, uint32_t* f, uint32_t x, uint32_t mn) {
    uint32_t h = (x * 2654435761u) >> 22;  // 10 bits
    for (int probe = 0; probe < 16; ++probe, h = (h + 1) & (kHookSlots - 1)) {
        uint32_t k = T.key[h];
        if (k == kNone) k = atomicCAS(&T.key[h], kNone, x) == kNone ? x : T.key[h];
        if (k == x) {
            atomicMin(&T.val[h], mn);
            return;
        }
    }
    if (mn < f[x]) atomicMin(f + x, mn);  // table crowded: straight to memory
}

// Roots x[0..k): hook all above the smallest. Returns true when they differ.
__device__ __forceinline__ bool hook_roots(HookTable& T, uint32_t* f, const uint32_t* x, int k,
                                           uint32_t& last_x, uint32_t& last_mn) {
    uint32_t mn = kNone;
    for (int v = 0; v < k; ++v) mn = x[v] < mn ? x[v] : mn;
    bool crossed = false;
    for (int v = 0; v < k; ++v) {
        if (x[v] == mn) continue;
        crossed = true;
        if (x[v] == last_x && mn == last_mn) continue;  // same hook as this lane's previous one
        last_x = x[v];
        last_mn = mn;
        hook_insert(T, f, x[v], mn);
    }
    return crossed;
}

// Global hook round over positions p0..L-1 (word groups {w0 + v * 4^(p-3)}). Words
// whose codes share one root (UR) need one f load instead of one per code; when
// every word of a group is uniform, the <= 6 word pairs that share a bit are the
// only hooks.
//
// Frontier: a group whose members already share one root never crosses again (roots
// only merge), so round k > 0 visits only the groups that crossed in round k - 1.
// active holds two generations of one bit per task (written whole by ballots).

// CHECK (round 4): a read-only round: does any group of the frontier still cross? Sets
// flags[round] and hooks nothing, writes no frontier bits (a later real round `round`
// reads the same frontier). k_roots_check runs it beside the roots scan: converged, the
// forest is unchanged and the roots stand; otherwise the host runs round `round` for real
// and relabels (cluster_finish), so the last speculative round costs no launches of its own.
template <bool CHECK>
__device__ __forceinline__ void hook_block(const int64_t bid, const uint4* __restrict__ RT,
                                           const uint32_t* __restrict__ UR, int64_t words, int L, int p0,
                                           uint32_t* f, unsigned int* __restrict__ flags, int round,
                                           uint64_t* __restrict__ active, int64_t active_words,
                                           const unsigned long long* __restrict__ stats) {
    if (round > 0 && flags[round - 1] == 0) return;  // converged earlier
    // the local-CC instance launched did not take this bitmap (S_REDO): f / UR / lroot hold
    // stale or uninitialised values, so nothing may be read through them (cluster_finish
    // redoes the local and global phases)
    if (stats[S_REDO]) return;
    p0 = max(p0, (int)stats[S_P0]);  // the local phase's last position + 1 (7 or 8)
    const int64_t per = words >> 2;
    const int64_t tasks = (int64_t)(L - p0) * per;
    const int64_t u = bid * kBlock + threadIdx.x;
    const uint64_t* prev = active + (int64_t)((round - 1) & 1) * active_words;
    uint64_t* next = active + (int64_t)(round & 1) * active_words;
    const bool act = per > 0 && u < tasks && (round == 0 || ((prev[u >> 6] >> (u & 63)) & 1ull));
    if (!__syncthreads_or(act)) {
        if (!CHECK && (threadIdx.x & 63) == 0 && (u >> 6) < active_words) next[u >> 6] = 0;
        return;
    }
    __shared__ HookTable T;
    if (!CHECK) {
        for (int k = threadIdx.x; k < kHookSlots; k += kBlock) {
            T.key[k] = kNone;
            T.val[k] = kNone;
        }
        __syncthreads();
    }
    uint32_t last_x = kNone, last_mn = kNone;
    bool crossed = false;
    if (act) {
        const int p = p0 + (int)(u / per);
        const int64_t g = u % per;
        const int s2 = 2 * p - 6;
        const int64_t stride = 1ll << s2;
        const int64_t w0 = ((g >> s2) << (s2 + 2)) | (g & (stride - 1));
        uint4 e[4];
        uint64_t m[4];
        uint32_t root[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            e[v] = RT[w0 + v * stride];
            m[v] = rt_word(e[v]);
        }
        const uint64_t multi = multi_of4(m[0], m[1], m[2], m[3]);
        if (multi) {
            bool all_uniform = true;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                root[v] = kNone;
                if (m[v] & multi) {
                    const uint32_t ur = UR[w0 + v * stride];
                    if (ur != kNone) root[v] = f[ur];
                    else all_uniform = false;
                }
            }
            uint32_t x[4];
            if (all_uniform) {
                // whole words: the word pairs that share a bit link them; hook every root
                // to the smallest root of its connected group of words (<= 3 hooks instead
                // of one per linked pair: dense spaces link all 6 pairs of most groups)
                uint32_t adj[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    adj[a] = 1u << a;
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        if (b != a && (m[a] & m[b])) adj[a] |= 1u << b;
                }
#pragma unroll
                for (int it = 0; it < 2; ++it)  // closure: 4 nodes, diameter <= 3
#pragma unroll
                    for (int a = 0; a < 4; ++a) {
                        uint32_t r = adj[a];
#pragma unroll
                        for (int b = 0; b < 4; ++b)
                            if ((adj[a] >> b) & 1u) r |= adj[b];
                        adj[a] = r;
                    }
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    if (adj[a] == (1u << a)) continue;  // shares no bit with another word
                    uint32_t mn = root[a];
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        if ((adj[a] >> b) & 1u) mn = root[b] < mn ? root[b] : mn;
                    x[0] = root[a];
                    x[1] = mn;
                    crossed |= CHECK ? x[0] != x[1] : hook_roots(T, f, x, 2, last_x, last_mn);
                }
            } else {
                uint64_t mm = multi;
                while (mm) {
                    const int b = __ffsll((long long)mm) - 1;
                    mm &= mm - 1;
                    const uint64_t below = (1ull << b) - 1ull;
                    int k = 0;
#pragma unroll
                    for (int v = 0; v < 4; ++v)
                        if ((m[v] >> b) & 1ull)
                            x[k++] = root[v] != kNone ? root[v]
                                                      : f[e[v].z + (uint32_t)__popcll(m[v] & below)];
                    if (CHECK) {
                        for (int v = 1; v < k; ++v) crossed |= x[v] != x[0];
                    } else {
                        crossed |= hook_roots(T, f, x, k, last_x, last_mn);
                    }
                }
            }
        }
    }
    const uint64_t crossed_bits = __ballot(crossed);
    if ((threadIdx.x & 63) == 0) {
        if (!CHECK && (u >> 6) < active_words) next[u >> 6] = crossed_bits;
        if (crossed_bits) flags[round] = 1u;
    }
    if (CHECK) return;
    __syncthreads();
    for (int k = threadIdx.x; k < kHookSlots; k += kBlock) {
        const uint32_t x = T.key[k];
        if (x == kNone) continue;
        // atomicMin, not a plain store: with "smallest proposal wins" synth-v1 converges
        // in 3 productive rounds, with "any proposal wins" in 4 (measured)
        if (T.val[k] < f[x]) atomicMin(f + x, T.val[k]);
    }
}

__global__ __launch_bounds__(kBlock) void k_hook_g(const uint4* __restrict__ RT, const uint32_t* __restrict__ UR,
                                                   int64_t words, int L, int p0, uint32_t* f,
                                                   unsigned int* __restrict__ flags, int round,
                                                   uint64_t* __restrict__ active, int64_t active_words,
                                                   const unsigned long long* __restrict__ stats) {
    hook_block<false>(blockIdx.x, RT, UR, words, L, p0, f, flags, round, active, active_words, stats);
}

__device__ __forceinline__ int64_t live_distinct(const unsigned long long* stats, int64_t max_distinct) {
    return min<int64_t>((int64_t)stats[S_NDISTINCT], max_distinct);
}

// Stars again, over the live vertices only (bits of lroot: the local roots and the
// codes of words without a shared root); every other vertex keeps pointing at its
// local root. Only f[i] is written by lane i, and only with an ancestor, so
// concurrent chasers always see ancestors.
__global__ __launch_bounds__(kBlock) void k_jump(uint32_t* f, const uint64_t* __restrict__ lroot,
                                                 int64_t max_distinct,
                                                 const unsigned long long* __restrict__ stats,
                                                 const unsigned int* __restrict__ flags, int round) {
    if (flags[round] == 0 || stats[S_REDO]) return;  // S_REDO: f is not this bitmap's (hook_block)
    const int64_t nd = live_distinct(stats, max_distinct);
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (kBlock / 64);
    for (int64_t w = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; w * 64 < nd; w += nwaves) {
        const uint64_t lr = lroot[w];
        const int64_t i = w * 64 + lane;
        if (!((lr >> lane) & 1ull) || i >= nd) continue;
        uint32_t r = f[i];
        if (r == (uint32_t)i) continue;
        for (uint32_t p = f[r]; p != r; p = f[r]) r = p;
        f[i] = r;
    }
}

// Global roots (live vertices i with f[i] == i: only local roots can be) -> rbits over
// index space; their dense order is the label order. One pass: each workgroup owns
// kRootWords root words (16 per wave, 16 loads of f in flight per lane), stores their
// in-block prefix (rpref) and its sum; the last workgroup to finish scans the sums into
// rblksum (k_scan_blocks then makes rblkoff and the cluster count). Workgroup 0 first
// publishes the stats block (the round flags, final once the rounds' kernels are done)
// into mapped host memory and then the resolve's epoch (host != nullptr), so the host
// needs no copy or event. (Measured: letting the last workgroup to arrive scan the sums
// instead - a device-scope fence + atomic per workgroup - made this kernel 64-137 us.)
constexpr int kRootWords = 64;

// the stats block (round flags final) into mapped host memory, then the resolve's epoch
__device__ __forceinline__ void publish_stats(const unsigned long long* stats, unsigned long long* host,
                                              unsigned long long epoch) {
    for (int k = threadIdx.x; k < kStatsBytes / 8; k += blockDim.x)
        __hip_atomic_store(host + k, stats[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    if (threadIdx.x == 0) {
        // the resolve's sequence number, passed by the host at enqueue (no device-side
        // counter: nothing in the workspace has to survive between resolves)
        __hip_atomic_store(host + kStatsBytes / 8, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ __forceinline__ void roots_block(const int64_t bid, const uint32_t* __restrict__ f,
                                            const uint64_t* __restrict__ lroot, int64_t max_distinct,
                                            int64_t rwords, uint64_t* __restrict__ rbits,
                                            uint32_t* __restrict__ rpref, uint32_t* rblksum,
                                            const unsigned long long* stats) {
    __shared__ uint32_t s_cnt[kRootWords];
    const int64_t nd = live_distinct(stats, max_distinct);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int kPerWave = kRootWords / (kBlock / 64);  // 16
    const int64_t w0 = bid * kRootWords + wave * kPerWave;
    uint32_t fv[kPerWave];
    uint64_t lr[kPerWave];
#pragma unroll
    for (int k = 0; k < kPerWave; ++k) {
        const int64_t i = (w0 + k) * 64 + lane;
        lr[k] = (w0 + k) * 64 < nd ? lroot[w0 + k] : 0ull;
        fv[k] = i < nd ? f[i] : 0u;
    }
    uint64_t mine = 0;
#pragma unroll
    for (int k = 0; k < kPerWave; ++k) {
        const int64_t i = (w0 + k) * 64 + lane;
        const uint64_t m = __ballot(i < nd && ((lr[k] >> lane) & 1ull) && fv[k] == (uint32_t)i);
        if (lane == k) mine = m;
    }
    if (lane < kPerWave) {
        const int64_t w = w0 + lane;
        if (w < rwords) rbits[w] = mine;
        s_cnt[wave * kPerWave + lane] = (uint32_t)__popcll(mine);
    }
    __syncthreads();
        // in-block prefix of the kRootWords counts (one wave), block sum
    if (wave == 0) {
        const uint32_t v = lane < kRootWords ? s_cnt[lane] : 0u;
        uint32_t incl = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t t = __shfl_up(incl, off);
            if (lane >= off) incl += t;
        }
        const int64_t w = bid * kRootWords + lane;
        if (lane < kRootWords && w < rwords) rpref[w] = incl - v;
        if (lane == kRootWords - 1) rblksum[bid] = incl;
    }
}

__global__ __launch_bounds__(kBlock) void k_roots_scan(const uint32_t* __restrict__ f,
                                                       const uint64_t* __restrict__ lroot, int64_t max_distinct,
                                                       int64_t rwords, uint64_t* __restrict__ rbits,
                                                       uint32_t* __restrict__ rpref, uint32_t* rblksum,
                                                       const unsigned long long* stats, unsigned long long* host,
                                                       unsigned long long epoch) {
    if (host && blockIdx.x == 0) publish_stats(stats, host, epoch);
    roots_block(blockIdx.x, f, lroot, max_distinct, rwords, rbits, rpref, rblksum, stats);
}

// The roots scan (workgroups [0, rblocks)) and, beside it, the read-only check of hook
// round `round` (the rest; hook_block<false, true>): one launch for the last speculative
// round and the roots. The publish moves to k_word_label (the check's flag is final there).
__global__ __launch_bounds__(kBlock) void k_roots_check(const uint32_t* __restrict__ f,
                                                        const uint64_t* __restrict__ lroot, int64_t max_distinct,
                                                        int64_t rwords, uint64_t* __restrict__ rbits,
                                                        uint32_t* __restrict__ rpref, uint32_t* rblksum,
                                                        const unsigned long long* stats, int64_t rblocks,
                                                        const uint4* __restrict__ RT, const uint32_t* __restrict__ UR,
                                                        int64_t words, int L, int p0, unsigned int* flags, int round,
                                                        uint64_t* active, int64_t active_words) {
    if ((int64_t)blockIdx.x < rblocks)
        roots_block(blockIdx.x, f, lroot, max_distinct, rwords, rbits, rpref, rblksum, stats);
    else
        hook_block<true>((int64_t)blockIdx.x - rblocks, RT, UR, words, L, p0, const_cast<uint32_t*>(f), flags,
                                round, active, active_words, stats);
}

__device__ __forceinline__ uint32_t root_label(uint32_t r, const uint64_t* __restrict__ rbits,
                                               const uint32_t* __restrict__ rpref,
                                               const uint32_t* __restrict__ rblkoff) {
    const uint32_t w = r >> 6;
    return rblkoff[w / kRootWords] + rpref[w] + (uint32_t)__popcll(rbits[w] & ((1ull << (r & 63)) - 1ull));
}

// Dense label of one code: labelcode[code] (L <= 13) or ilab[index] (index space).
__device__ __forceinline__ void put_label(uint64_t c, uint32_t i, uint32_t lab, uint32_t* __restrict__ labelcode,
                                          uint32_t* __restrict__ ilab) {
    if (labelcode) labelcode[c] = lab;
    else ilab[i] = lab;
}

// Label of every word with a shared local root, and per code of the codes no word
// label covers (one pass: a word's exception codes are labelled by the lane that
// labels the word).
// A word without a shared LOCAL root still gets a word label when the global phase put
// all of its codes in one component (their f are global roots then: they are live): in
// the giant components of a 1-edit-saturated space most words end up uniform, and assign
// then needs one L2-resident load per row instead of a gather from the 4^L table.
// rblksum != nullptr (round 4): the roots scan's block sums are scanned by every workgroup
// into LDS (dynamic, nrb_max + 1 u32) instead of by a k_scan_blocks launch of their own
// (one kernel boundary fewer on the resolve chain); workgroup 0 writes the cluster count.
__global__ __launch_bounds__(kBlock) void k_word_label(const uint32_t* __restrict__ f,
                                                       const uint32_t* __restrict__ UR, int64_t words,
                                                       const uint4* __restrict__ RT, int64_t max_distinct,
                                                       const uint64_t* __restrict__ rbits,
                                                       const uint32_t* __restrict__ rpref,
                                                       const uint32_t* __restrict__ rblkoff,
                                                       uint32_t* __restrict__ wlab, uint64_t* __restrict__ wexc,
                                                       uint32_t* __restrict__ labelcode, uint32_t* __restrict__ ilab,
                                                       int exc1_on,
                                                       const uint32_t* __restrict__ rblksum = nullptr,
                                                       int64_t nrb_max = 0, unsigned long long* stats = nullptr,
                                                       const unsigned long long* pstats = nullptr,
                                                       unsigned long long* host = nullptr,
                                                       unsigned long long epoch = 0) {
    extern __shared__ uint32_t s_roff[];
    __shared__ uint32_t s_wave[kBlock / 64];
    if (host && blockIdx.x == 0) publish_stats(pstats, host, epoch);  // after k_roots_check
    if (pstats[S_REDO]) return;  // f / UR are not this bitmap's (hook_block); cluster_finish relabels
    if (rblksum) {
        const int64_t nd = live_distinct(stats, max_distinct);
        const int64_t nrb = min<int64_t>(nrb_max, (nd + (int64_t)kRootWords * 64 - 1) / ((int64_t)kRootWords * 64));
        uint32_t carry = 0;
        for (int64_t b0 = 0; b0 < nrb; b0 += kBlock) {
            const int64_t b = b0 + threadIdx.x;
            const uint32_t v = b < nrb ? rblksum[b] : 0u;
            uint32_t total;
            const uint32_t ex = block_excl_scan(v, s_wave, total);
            if (b < nrb) s_roff[b] = carry + ex;
            carry += total;
        }
        if (threadIdx.x == 0) {
            s_roff[nrb] = carry;
            if (blockIdx.x == 0) stats[S_NCLUSTERS] = carry;
        }
        __syncthreads();
        rblkoff = s_roff;
    }
    for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < words; w += (int64_t)gridDim.x * kBlock) {
        const uint32_t ur = UR[w];
        uint32_t root = kNone;
        uint64_t exc = 0;
        uint4 e = make_uint4(0, 0, 0, 0);
        uint64_t m = 0;
        if (ur != kNone) {
            root = f[ur];
        } else {
            e = RT[w];
            m = rt_word(e);
            const int cnt = __popcll(m);
            if (cnt > 0 && (int64_t)e.z + cnt <= max_distinct) {
                // the word's label is its most frequent root (Boyer-Moore vote; any choice
                // is exact): the codes of other components are the exceptions, labelled
                // per code
                uint32_t cand = f[e.z], votes = 1;
                for (int k = 1; k < cnt; ++k) {
                    const uint32_t r = f[e.z + k];
                    if (r == cand) ++votes;
                    else if (votes == 0) {
                        cand = r;
                        votes = 1;
                    } else {
                        --votes;
                    }
                }
                root = cand;
                uint64_t mm = m;
                for (int k = 0; mm; ++k) {
                    const int b = __ffsll((long long)mm) - 1;
                    mm &= mm - 1;
                    if (f[e.z + k] != cand) exc |= 1ull << b;
                }
            }
        }
        // bit 31 flags a word with exceptions (mask form: labels < 2^29, umi_len <= 14; a
        // larger label leaves the word unlabelled and all its codes are labelled per code)
        uint32_t lab = root != kNone ? root_label(root, rbits, rpref, rblkoff) : kNone;
        if (exc && lab != kNone) {  // encodings: decode_word_label (rogtk_internal.h)
            const uint64_t rest = exc & (exc - 1);  // the exceptions past the first
            if (exc1_on && !rest && lab < (1u << 24)) {
                lab |= 0xC0000000u | ((uint32_t)(__ffsll((long long)exc) - 1) << 24);
            } else if (exc1_on && !(rest & (rest - 1)) && lab < (1u << 17)) {
                lab |= 0xA0000000u | ((uint32_t)(__ffsll((long long)exc) - 1) << 17) |
                       ((uint32_t)(__ffsll((long long)rest) - 1) << 23);
            } else {
                lab = lab < 0x20000000u ? (lab | 0x80000000u) : kNone;
            }
        }
        wlab[w] = lab;
        // the codes the word label does not cover (its exceptions, or all of them when
        // the word stays unlabelled) get their own label (f[i] is their root: they are
        // live); a uniform word (ur != kNone) always has a label
        uint64_t per_code = lab == kNone ? m : exc;
        while (per_code) {
            const int b = __ffsll((long long)per_code) - 1;
            per_code &= per_code - 1;
            const uint32_t i = e.z + (uint32_t)__popcll(m & ((1ull << b) - 1ull));
            if ((int64_t)i >= max_distinct) continue;
            const uint32_t li = root_label(f[i], rbits, rpref, rblkoff);
            put_label((uint64_t)w * 64 + b, i, li, labelcode, ilab);
        }
        wexc[w] = exc;
    }
}

// The label of code c from its word (kNone: label it per code): wlab[w] = the label of
// the word's most frequent component, bit 31 set when some of its codes (wexc[w]) belong
// to other components (decode_word_label). Only words with two or more exception codes
// cost a second (2 MB-table) load; a single exception code is named in the label.
__device__ __forceinline__ uint32_t word_label_of(const uint32_t* __restrict__ wlab,
                                                  const uint64_t* __restrict__ wexc, uint64_t c) {
    return decode_word_label(wlab[c >> 6], wexc, c);
}

// MODE 0: labelcode[code]; MODE 1: flab[rank(code)] (labels by index, ilab); MODE 2 (exact
// ids, max_distance 0, round 5): the rank itself, from the 16-B-per-64-codes rank table (4 MB
// at L = 12, cache-resident) instead of a gather from the 4^L-entry label table (C3's H3:
// 100M rows 1.8 ms).
// wlab / wexc (max_distance 1 only, else NULL): per 64 codes the label of the word's most
// frequent component (1 MB at L = 12, L2-resident) and, for flagged words only, the mask
// of its other codes (2 MB): only exception codes gather from the 4^L-entry table.
// G groups of 4 rows per lane and loop trip (all loads of a trip in flight at once):
// lane l of a wave owns rows {tile + 256 g + 4 l .. + 3}, so each 16-B load / store
// instruction of a wave covers 1 KB contiguous.
template <int MODE, int G>
__global__ __launch_bounds__(kBlock) void k_assign(const uint32_t* __restrict__ codes,
                                                   const uint64_t* __restrict__ regbits, int64_t n,
                                                   const uint32_t* __restrict__ labelcode,
                                                   const uint32_t* __restrict__ flab,
                                                   const uint4* __restrict__ RT, const uint32_t* __restrict__ wlab,
                                                   const uint64_t* __restrict__ wexc, uint32_t* __restrict__ out) {
    constexpr int64_t kTile = 256 * G;  // rows per wave and trip
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (kBlock / 64);
    for (int64_t tile = (((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6) * kTile; tile < n;
         tile += nwaves * kTile) {
        uint32_t c[G][4];
        uint32_t reg[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int64_t row0 = tile + 256 * g + 4 * lane;
            c[g][0] = c[g][1] = c[g][2] = c[g][3] = 0;
            if (row0 + 4 <= n) {
                const u32x4_t v = stream_load(reinterpret_cast<const u32x4_t*>(codes + row0));
                c[g][0] = v.x; c[g][1] = v.y; c[g][2] = v.z; c[g][3] = v.w;
            } else {
                for (int k = 0; k < 4; ++k)
                    if (row0 + k < n) c[g][k] = codes[row0 + k];
            }
            reg[g] = row0 >= n ? 0u : regbits ? (uint32_t)(regbits[row0 >> 6] >> (row0 & 63)) & 0xFu : 0xFu;
        }
        uint32_t id[G][4];
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                id[g][k] = 0xFFFFFFFFu;
                if ((reg[g] >> k) & 1u) {
                    const uint32_t wl = wlab ? word_label_of(wlab, wexc, c[g][k]) : kNone;
                    id[g][k] = wl != kNone ? wl
                               : MODE == 0 ? labelcode[c[g][k]]
                               : MODE == 1 ? flab[rt_rank(RT[c[g][k] >> 6], c[g][k])]
                                           : rt_rank(RT[c[g][k] >> 6], c[g][k]);
                }
            }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int64_t row0 = tile + 256 * g + 4 * lane;
            if (row0 + 4 <= n) {
                stream_store(u32x4_t{id[g][0], id[g][1], id[g][2], id[g][3]}, reinterpret_cast<u32x4_t*>(out + row0));
            } else {
                for (int k = 0; k < 4; ++k)
                    if (row0 + k < n) out[row0 + k] = id[g][k];
            }
        }
    }
}

// Label of arbitrary packed codes (the irregular merge's neighbour probes): kNone for
// ~0 or a code that is not present, else the label k_assign would give it.
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_lookup(const uint64_t* __restrict__ q, int64_t nq, uint64_t nbits,
                                                   const uint32_t* __restrict__ labelcode,
                                                   const uint32_t* __restrict__ flab, const uint4* __restrict__ RT,
                                                   const uint32_t* __restrict__ wlab,
                                                   const uint64_t* __restrict__ wexc, uint32_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nq; i += (int64_t)gridDim.x * kBlock) {
        const uint64_t c = q[i];
        uint32_t lab = kNone;
        if (c < nbits) {
            const uint4 e = RT[c >> 6];
            if ((rt_word(e) >> (c & 63)) & 1ull) {
                const uint32_t wl = wlab ? word_label_of(wlab, wexc, c) : kNone;
                lab = wl != kNone ? wl : MODE == 0 ? labelcode[c] : flab[rt_rank(e, (uint32_t)c)];
            }
        }
        out[i] = lab;
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
    unsigned int* flags;
    uint8_t* presence;
    uint64_t* G;
    uint4* RT;
    uint32_t *wpref, *blksum, *blkoff, *D, *f, *UR;
    uint64_t *rbits, *lroot;
    uint32_t *rpref, *rblksum, *rblkoff, *labelcode, *ilab;
    uint64_t* active;
    uint64_t* lb;               // look-back flags of k_scan_rt (+ its error word)
};

inline WsPtrs ws_ptrs(const ClusterLayout& cl, uint8_t* ws) {
    WsPtrs p;
    p.stats = (unsigned long long*)(ws + cl.off_stats);
    p.flags = (unsigned int*)(ws + cl.off_stats + kFlagsOff);
    p.presence = ws + cl.off_presence;
    p.G = (uint64_t*)(ws + cl.off_bitmap);
    p.RT = (uint4*)(ws + cl.off_rt);
    p.wpref = (uint32_t*)(ws + cl.off_wpref);
    p.blksum = (uint32_t*)(ws + cl.off_blksum);
    p.blkoff = (uint32_t*)(ws + cl.off_blkoff);
    p.D = (uint32_t*)(ws + cl.off_D);
    p.f = (uint32_t*)(ws + cl.off_f);
    p.UR = (uint32_t*)(ws + cl.off_ur);
    p.rbits = (uint64_t*)(ws + cl.off_rbits);
    p.lroot = (uint64_t*)(ws + cl.off_lroot);
    p.rpref = (uint32_t*)(ws + cl.off_rpref);
    p.rblksum = (uint32_t*)(ws + cl.off_rblksum);
    p.rblkoff = (uint32_t*)(ws + cl.off_rblkoff);
    p.labelcode = cl.label_by_code ? (uint32_t*)(ws + cl.off_labelcode) : nullptr;
    p.ilab = cl.label_by_code ? nullptr : (uint32_t*)(ws + cl.off_ilab);
    p.active = (uint64_t*)(ws + cl.off_active);
    p.lb = (uint64_t*)(ws + cl.off_lb);
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
    c.rblocks = (c.rwords + kRootWords - 1) / kRootWords;
    // labels by code (a 4^L-entry table) up to L = 13 (64 MB at L = 12), else by rank (index
    // space); by rank at L = 12 measured slower (two dependent gathers per exception row)
    c.label_by_code = L <= 13;
    int64_t off = 0;
    auto take = [&](int64_t bytes) {
        const int64_t at = off;
        off += (bytes + 255) / 256 * 256;
        return at;
    };
    c.off_stats = take(kStatsBytes);
    c.off_presence = take((int64_t)(c.nbits < 64 ? 64 : c.nbits));
    c.off_bitmap = take(c.words * 8);
    c.off_rt = take(c.words * 16);
    c.off_wpref = take(c.words * 4);
    c.off_blksum = take(c.blocks * 4);
    c.off_blkoff = take((c.blocks + 1) * 4);
    c.off_D = take(max_distinct * 4);
    c.off_f = take(max_distinct * 4);
    c.off_ur = take(c.words * 4);
    c.off_rbits = take(c.rwords * 8);
    c.off_lroot = take(c.rwords * 8);
    c.off_rpref = take(c.rwords * 4);
    c.off_rblksum = take(c.rblocks * 4);
    c.off_rblkoff = take((c.rblocks + 1) * 4);
    c.off_labelcode = c.label_by_code ? take((int64_t)c.nbits * 4) : off;
    c.off_ilab = c.label_by_code ? off : take(max_distinct * 4);
    // hook-round frontier: one bit per (position, word group) task, two generations
    const int64_t tasks = L > kLocalPos ? (int64_t)(L - kLocalPos) * (c.words >> 2) : 0;
    c.active_words = (tasks + 63) / 64;
    c.off_active = take(2 * std::max<int64_t>(c.active_words, 1) * 8);
    // look-back flags + error word + tagged block totals (k_scan_rt)
    c.off_lb = take((2 * std::max(c.blocks, c.rblocks) + 1) * 8);
    c.total = off;
    *o = c;
    return ROGTK_OK;
}

// ------------------------------------------------------------------ mark
// presence[code] = 1 for every regular row, partitioned by XCD: block b marks only
// the codes of partition b % 8 (code range [p, p+1) * 4^L / 8) from its chunk of
// rows. Under the observed round-robin placement blocks b and b + 8 share an XCD,
// so each XCD's scattered byte stores land in its own 1/8 of the table (2 MB at
// L = 12), which stays resident in that XCD's 4 MB L2 until the kernel ends; the
// 8x re-read of the codes is served by the Infinity Cache. Placement only affects
// speed: every (partition, chunk) pair is handled by exactly one block.

__global__ __launch_bounds__(kBlock) void k_mark_xcd(const uint32_t* __restrict__ codes,
                                                      const uint64_t* __restrict__ regbits, int64_t n,
                                                      int two_l, int64_t chunk, uint8_t* __restrict__ pres) {
    const uint32_t part = blockIdx.x % kMarkParts;
    const int64_t c0 = (int64_t)(blockIdx.x / kMarkParts) * chunk;
    const int64_t c1 = c0 + chunk < n ? c0 + chunk : n;
    for (int64_t r = c0 + 4 * (int64_t)threadIdx.x; r < c1; r += 4 * kBlock) {
        uint32_t c[4];
        uint32_t reg = regbits ? (uint32_t)(regbits[r >> 6] >> (r & 63)) & 0xFu : 0xFu;
        if (r + 4 <= n) {
            const u32x4_t v = stream_load(reinterpret_cast<const u32x4_t*>(codes + r));
            c[0] = v.x; c[1] = v.y; c[2] = v.z; c[3] = v.w;
        } else {
            reg &= (1u << (uint32_t)(n - r)) - 1u;
            for (int k = 0; k < 4; ++k) c[k] = r + k < n ? codes[r + k] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (((reg >> k) & 1u) && (uint32_t)(((uint64_t)c[k] * kMarkParts) >> two_l) == part)
                pres[c[k]] = 1;  // benign same-value race
    }
}

int launch_cluster_mark(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int L,
                        uint8_t* presence, hipStream_t s) {
    if (n <= 0) return ROGTK_OK;
    ProfScope prof(K_MARK, s);
    // chunk: a multiple of 4 * kBlock rows (keeps r 4-aligned for the uint4 loads)
    int64_t chunk = (n + kMarkChunks - 1) / kMarkChunks;
    chunk = (chunk + 4 * kBlock - 1) / (4 * kBlock) * (4 * kBlock);
    const int64_t chunks = (n + chunk - 1) / chunk;
    hipLaunchKernelGGL(k_mark_xcd, dim3((unsigned)(chunks * kMarkParts)), dim3(kBlock), 0, s, codes, regular_bits,
                       n, 2 * L, chunk, presence);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

int launch_cluster_local_bitmap(const ClusterLayout& cl, uint8_t* ws, uint64_t* out, hipStream_t s) {
    WsPtrs p = ws_ptrs(cl, ws);
    ProfScope prof(K_BITMAP, s);
    if (cl.nbits >= 64) {
        hipLaunchKernelGGL(k_bitmap_wide, dim3(grid_for(cl.words * 4)), dim3(kBlock), 0, s, p.presence,
                           cl.words, out);
    } else {
        hipLaunchKernelGGL(k_bitmap_small, dim3(1), dim3(64), 0, s, p.presence, cl.nbits, out);
    }
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

namespace {

constexpr int kSpecRounds = 4;  // speculative global rounds (synth-v1 needs 3-4)
std::atomic<int> g_spec_rounds{kSpecRounds};
// rogtk_cluster_set_spec_rounds(0) (the default): a workspace whose previous resolve needed
// more rounds than the default launches one more than that, so denser batches (e.g. the union bitmap of many
// ranks) do not fall back to the host-synchronous completion every time
std::atomic<bool> g_spec_adaptive{true};
std::atomic<int> g_lb_polls{kLbMaxPolls};  // look-back polls before the recount (tests)

// Host-side state of an in-flight resolve, keyed by workspace: the round flags are
// copied asynchronously to pinned host memory so resolve never blocks the host;
// assign (or rogtk_cluster_stats) checks them and only then, if the speculative
// rounds were not enough, runs more rounds and relabels.
struct ResolveState {
    // the stats block (round flags, local-CC redo) published by k_roots_scan into
    // mapped, coherent host memory, followed by a sequence word = the resolve's epoch
    uint8_t* hstats = nullptr;
    uint8_t* hstats_dev = nullptr;  // its device address
    uint64_t epoch = 0;             // resolves with rounds enqueued so far (the published sequence number)
    int launched = 0;
    bool pending = false;
    int rounds = 0;  // hook rounds the last resolve needed (the converged round included)
    int needed = 0;  // the same, kept across launches (adaptive speculative rounds)
    bool word_labels = false;  // wpref holds word labels (max_distance 1)
    bool exact = false;        // max_distance 0: the ids are the codes' ranks
    uint32_t scan_tag = 0;     // the last k_scan_rt launch's look-back tag (1..2^30-1)
    int lcc_choice = -1;       // the local-CC instance of the last resolve (launch_local_cc)
    bool checked = false;      // flags[launched] holds a read-only check round (k_roots_check)
    ClusterLayout cl{};
    // an assign enqueued before the flags were checked (rogtk_cluster_assign_deferred)
    struct {
        bool on = false;
        const uint32_t* codes;
        const uint64_t* regbits;
        int64_t n;
        uint32_t* cid;
    } deferred;
};
std::mutex g_rs_mu;
std::map<const void*, ResolveState> g_rs;

// Host side: spin until this resolve's stats are published (normally long done).
int wait_published(const ResolveState& st) {
    const volatile unsigned long long* seq = (const volatile unsigned long long*)(st.hstats + kStatsBytes);
    const auto t0 = std::chrono::steady_clock::now();
    while (*seq != st.epoch) {
        std::this_thread::yield();
        ROGTK_REQUIRE(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(120), ROGTK_E_HIP,
                      "cluster: resolve flags not published within 120 s (stream stalled?)");
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return ROGTK_OK;
}

// Global hook + jump rounds [from, to) (each exits at once once a round found nothing).
int enqueue_rounds(const ClusterLayout& cl, const WsPtrs& p, int from, int to, hipStream_t s) {
    const int pg = grid_for(cl.max_distinct, kPersistentGrid);
    const int64_t tasks = (int64_t)(cl.L - kLocalPos) * (cl.words >> 2);
    for (int k = from; k < to; ++k) {
        ROGTK_TIMED_LAUNCH(K_K_HOOK, k_hook_g, dim3(grid_for(tasks)), dim3(kBlock), 0, s, p.RT, p.UR, cl.words, cl.L, kLocalPos,
                           p.f, p.flags, k, p.active, cl.active_words, (const unsigned long long*)p.stats);
        ROGTK_TIMED_LAUNCH(K_K_JUMP, k_jump, dim3(pg), dim3(kBlock), 0, s, p.f, p.lroot, cl.max_distinct, p.stats, p.flags, k);
    }
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

// rogtk_cluster_resolve's completion event, armed by its caller (rogtk_event_attach_next):
// recorded on k_word_label's dispatch packet, or by a marker after the resolve's launches
thread_local hipEvent_t t_resolve_fin = nullptr;

// host_stats != nullptr: k_roots_scan also publishes the stats block (the resolve's
// first labels pass; never the re-run after extra rounds, which the host waits for)
// check_round >= 0: the read-only check of that hook round runs inside the roots scan's
// launch (k_roots_check), and the stats publish moves to k_word_label.
int enqueue_labels(const ClusterLayout& cl, const WsPtrs& p, hipStream_t s,
                   unsigned long long* host_stats = nullptr, int check_round = -1, uint64_t epoch = 0) {
    // the block offsets of the roots scan in every k_word_label workgroup's LDS when they
    // fit (<= 16K root blocks: 67M distinct codes), else a k_scan_blocks launch
    const bool lds_off = (cl.rblocks + 1) * 4 <= 65536;
    {
        ProfScope prof(K_FLATTEN, s);
        if (check_round >= 0) {
            const int64_t tasks = (int64_t)(cl.L - kLocalPos) * (cl.words >> 2);
            ROGTK_TIMED_LAUNCH(K_K_ROOTS, k_roots_check, dim3((unsigned)(cl.rblocks + grid_for(tasks))), dim3(kBlock), 0, s, p.f,
                               p.lroot, cl.max_distinct, cl.rwords, p.rbits, p.rpref, p.rblksum,
                               (const unsigned long long*)p.stats, cl.rblocks, p.RT, p.UR, cl.words, cl.L, kLocalPos,
                               p.flags, check_round, p.active, cl.active_words);
        } else {
            ROGTK_TIMED_LAUNCH(K_K_ROOTS, k_roots_scan, dim3((unsigned)cl.rblocks), dim3(kBlock), 0, s, p.f, p.lroot,
                               cl.max_distinct, cl.rwords, p.rbits, p.rpref, p.rblksum,
                               (const unsigned long long*)p.stats, host_stats, (unsigned long long)epoch);
        }
        if (!lds_off)
            hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kBlock), 0, s, p.rblksum, cl.rblocks, p.rblkoff, p.stats,
                               (int)S_NCLUSTERS, -1, 0, (int64_t)kRootWords * 64);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    {
        ProfScope prof(K_LABEL, s);
        // wpref and G (consumed into RT by k_rt) hold the word labels and exception masks
        // ROGTK_WORD_EXC1=0: words with one or two exception codes also take the mask load (A/B)
        static const int exc1_on = [] {
            const char* e = getenv("ROGTK_WORD_EXC1");
            return e && e[0] == '0' ? 0 : 1;
        }();
        // the resolve's completion event (armed by the caller, taken at rogtk_cluster_resolve's
        // entry) rides on this last launch's dispatch packet
        if (t_resolve_fin) arm_attached_event(t_resolve_fin);
        ROGTK_TIMED_LAUNCH(K_K_WORD_LABEL, k_word_label, dim3(grid_for(cl.words, kPersistentGrid)), dim3(kBlock),
                           lds_off ? (size_t)(cl.rblocks + 1) * 4 : 0, s, p.f, p.UR, cl.words, p.RT, cl.max_distinct,
                           p.rbits, p.rpref, p.rblkoff, p.wpref, p.G, p.labelcode, p.ilab, exc1_on,
                           lds_off ? p.rblksum : nullptr, (int64_t)cl.rblocks, lds_off ? p.stats : nullptr,
                           (const unsigned long long*)p.stats, check_round >= 0 ? host_stats : nullptr,
                           (unsigned long long)epoch);
        if (t_resolve_fin && attached_event_taken()) t_resolve_fin = nullptr;
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    return ROGTK_OK;
}

// index of the first round that found nothing to hook, or -1
int first_zero(const unsigned int* f, int from, int to) {
    for (int k = from; k < to; ++k)
        if (f[k] == 0) return k;
    return -1;
}

}  // namespace

#ifndef ROGTK_ASSIGN_WGS
#define ROGTK_ASSIGN_WGS 2  // workgroups per CU of k_assign (experiment builds)
#endif
#ifndef ROGTK_ASSIGN_G
#define ROGTK_ASSIGN_G 2  // 4-row groups per lane and trip (experiment builds)
#endif
namespace {
int enqueue_assign(const ClusterLayout& cl, const WsPtrs& p, int labels, const uint32_t* codes,
                   const uint64_t* regular_bits, int64_t n, uint32_t* cluster_id, hipStream_t s);
int finish_locked(const void* ws, ResolveState& st, hipStream_t s, int* redone = nullptr);
}  // namespace

namespace {
// ROGTK_FUSED_SCAN=0: the rank tables by three kernels (scan words, scan blocks, RT)
// instead of the single-pass k_scan_rt (A/B; also what the look-back's fallback tests
// compare against)
bool fused_scan_enabled() {
    static const bool on = [] {
        const char* e = getenv("ROGTK_FUSED_SCAN");
        return !(e && e[0] == '0');
    }();
    return on;
}

// ROGTK_LCC_PREDICT=0: launch every local-CC instance (each exits at once for the tilings
// of the others) instead of the previous resolve's alone (A/B)
bool lcc_predict_enabled() {
    static const bool on = [] {
        const char* e = getenv("ROGTK_LCC_PREDICT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// The kernels of one resolve, enqueued on s. Returns the number of speculative hook
// rounds launched for real (0: no global rounds), -1 on error. scan_tag: the look-back tag
// of k_scan_rt (0 = the three-kernel scan). lcc_choice >= 0: the local-CC instance to
// launch alone (launch_local_cc). *checked: the last speculative round ran as a read-only
// check inside the roots scan's launch.
int enqueue_resolve(const ClusterLayout& cl, const WsPtrs& p, const uint64_t* bitmaps, int n_bitmaps,
                    int max_distance, int spec, unsigned long long* host_stats, uint64_t epoch, hipStream_t s,
                    uint32_t scan_tag, int lcc_choice, bool* checked) {
    *checked = false;
    {
        ProfScope prof(K_SCAN, s);
        if (scan_tag) {  // single pass: RT, n_distinct and the tiling in one launch
            ROGTK_TIMED_LAUNCH(K_K_SCAN_RT, k_scan_rt, dim3((unsigned)cl.blocks), dim3(kBlock), 0, s, bitmaps, n_bitmaps, cl.words,
                               p.RT, p.lroot, max_distance == 0 ? (int64_t)0 : cl.rwords,
                               p.lb + std::max(cl.blocks, cl.rblocks) + 1, p.lb, scan_tag, p.stats, (int)S_NDISTINCT,
                               max_distance == 0 ? (int)S_NCLUSTERS : -1, local8_enabled() ? cl.L : 0,
                               local8_big_enabled(), g_lb_polls.load());
        } else {
            hipLaunchKernelGGL(k_scan_words, dim3((unsigned)cl.blocks), dim3(kBlock), 0, s, bitmaps, n_bitmaps,
                               cl.words, (const unsigned long long*)nullptr, p.G, p.wpref, p.blksum);
            hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kBlock), 0, s, p.blksum, cl.blocks, p.blkoff, p.stats,
                               (int)S_NDISTINCT, max_distance == 0 ? (int)S_NCLUSTERS : -1, 1, (int64_t)0,
                               local8_enabled() ? cl.L : 0, local8_big_enabled());
            hipLaunchKernelGGL(k_rt, dim3(grid_for(cl.words)), dim3(kBlock), 0, s, p.G, cl.words, p.wpref, p.blkoff,
                               p.RT, p.lroot, max_distance == 0 ? 0 : cl.rwords);
        }
    }
    if (max_distance == 0) {  // labels = ranks (labelcode / ilab)
        const int cgrid = grid_for((int64_t)std::min<uint64_t>(cl.nbits, 1ull << 30), 16384);
        hipLaunchKernelGGL(k_build_d, dim3(cgrid), dim3(kBlock), 0, s, p.RT, cl.nbits, p.D, p.f, p.labelcode, p.ilab,
                           cl.max_distinct, p.stats);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    ProfScope prof(K_UNION, s);
    launch_local_cc(p.RT, cl.words, cl.L, p.f, p.UR, p.lroot, cl.rwords, cl.max_distinct, p.stats, s, lcc_choice);
    if (cl.L <= kLocalPos) {
        if (enqueue_labels(cl, p, s, nullptr)) return -1;
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    // the last speculative round as a read-only check inside the roots scan's launch
    // (round 4: two kernel boundaries fewer on the resolve chain; a round that still finds
    // crossings runs for real in cluster_finish)
    const bool fuse = host_stats && spec >= 2;
    const int real = fuse ? spec - 1 : spec;
    if (enqueue_rounds(cl, p, 0, real, s)) return -1;
    *checked = fuse;
    // k_roots_scan (or k_word_label after a check) stores the flags into mapped host memory
    // and then the resolve's sequence number: no copy-engine transfer, no
    // event, no kernel of its own (a D2H copy + event record cost ~15 us of the resolve chain)
    if (enqueue_labels(cl, p, s, host_stats, fuse ? real : -1, epoch)) return -1;
    return hipGetLastError() == hipSuccess ? real : -1;
}
}  // namespace

int launch_cluster_resolve(const ClusterLayout& cl, uint8_t* ws, const uint64_t* bitmaps, int n_bitmaps,
                           int max_distance, hipStream_t s) {
    WsPtrs p = ws_ptrs(cl, ws);
    hipEvent_t fin = take_attached_event();  // armed by the caller: recorded at the end
    std::lock_guard<std::mutex> lk(g_rs_mu);
    ResolveState& st = g_rs[ws];
    if (st.pending && st.deferred.on) {  // a deferred assign must see its resolve complete first
        if (int rc = finish_locked(ws, st, s)) {
            if (fin) (void)hipEventRecord(fin, s);
            return rc;
        }
    }
    ProfScope prof_chain(K_RESOLVE, s);
    st.pending = false;
    st.deferred.on = false;
    st.rounds = 0;
    st.cl = cl;
    st.word_labels = max_distance == 1;
    st.exact = max_distance == 0;
    int spec = g_spec_rounds.load();
    if (g_spec_adaptive.load() && st.needed > spec) spec = std::min(st.needed + 1, kMaxRounds);
    const bool rounds = max_distance == 1 && cl.L > kLocalPos;
    if (rounds && !st.hstats) {
        ROGTK_HIP_CHECK(hipHostMalloc((void**)&st.hstats, kStatsBytes + 64, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(st.hstats, 0, kStatsBytes + 64);
        ROGTK_HIP_CHECK(hipHostGetDevicePointer((void**)&st.hstats_dev, st.hstats, 0));
    }
    // a new look-back tag per single-pass scan (0 = the three-kernel scan)
    uint32_t tag = 0;
    if (fused_scan_enabled()) {
        st.scan_tag = st.scan_tag >= (1u << 30) - 1 ? 1u : st.scan_tag + 1;
        tag = st.scan_tag;
    }
    // one local-CC instance, the previous resolve's (checked on the device: S_REDO)
    const int choice = rounds && lcc_predict_enabled() ? st.lcc_choice : -1;
    bool checked = false;
    t_resolve_fin = fin;
    const int launched = enqueue_resolve(cl, p, bitmaps, n_bitmaps, max_distance, spec,
                                         rounds ? (unsigned long long*)st.hstats_dev : nullptr, st.epoch + 1, s, tag,
                                         choice, &checked);
    if (t_resolve_fin) {  // no k_word_label took it (or the launch failed): a marker
        (void)hipEventRecord(t_resolve_fin, s);
        t_resolve_fin = nullptr;
    }
    if (fin) set_attached_taken();  // recorded either way (rogtk_event_attach_done says so)
    ROGTK_REQUIRE(launched >= 0, ROGTK_E_HIP, "cluster: resolve launch failed (%s)", hipGetErrorString(hipGetLastError()));
    if (rounds) {
        ++st.epoch;  // the sequence number k_roots_scan / k_word_label publish (passed at enqueue)
        st.launched = launched;
        st.checked = checked;
        st.pending = true;
    }
    return ROGTK_OK;
}

int cluster_finish(const void* ws, hipStream_t s, int* redone) {
    if (redone) *redone = 0;
    std::lock_guard<std::mutex> lk(g_rs_mu);
    auto it = g_rs.find(ws);
    if (it == g_rs.end() || !it->second.pending) return ROGTK_OK;
    return finish_locked(ws, it->second, s, redone);
}

namespace {
int finish_locked(const void* ws, ResolveState& st, hipStream_t s, int* redone) {
    if (int rc = wait_published(st)) return rc;
    unsigned int* hflags = (unsigned int*)(st.hstats + kFlagsOff);
    const unsigned long long* hs = (const unsigned long long*)st.hstats;
    // the local-CC instance this bitmap's tiling takes: the next resolve launches it alone
    st.lcc_choice = hs[S_P0] == 8 ? (int)hs[S_LCAP] : 2;
    const bool redo = hs[S_REDO] != 0;
    const int scanned = st.launched + (st.checked ? 1 : 0);  // a check round's flag too
    st.checked = false;
    if (!redo) {
        if (int z = first_zero(hflags, 0, scanned); z >= 0) {
            st.pending = false;
            st.deferred.on = false;
            st.rounds = z + 1;
            st.needed = st.rounds;
            return ROGTK_OK;
        }
    }
    // the speculative rounds were not enough: continue synchronously, then relabel
    if (redone) *redone = 1;
    WsPtrs p = ws_ptrs(st.cl, const_cast<uint8_t*>((const uint8_t*)ws));
    if (redo) {
        // the launched local-CC instance did not take this tiling (nothing of the local or
        // global phase stands): the local CC again (every instance; it reads only RT),
        // then the global rounds from round 0
        ProfScope prof(K_UNION, s);
        ROGTK_HIP_CHECK(hipMemsetAsync(p.stats + S_REDO, 0, 8, s));
        launch_local_cc(p.RT, st.cl.words, st.cl.L, p.f, p.UR, p.lroot, st.cl.rwords, st.cl.max_distinct, p.stats, s,
                        -1);
        ROGTK_HIP_CHECK(hipGetLastError());
        ROGTK_HIP_CHECK(hipMemsetAsync(p.flags, 0, kMaxRounds * sizeof(unsigned int), s));
        std::memset(hflags, 0, kMaxRounds * sizeof(unsigned int));
        st.launched = 0;
    }
    bool converged = false;
    while (!converged && st.launched < kMaxRounds) {
        const int to = std::min(st.launched + kRoundBatch, kMaxRounds);
        {
            ProfScope prof(K_UNION, s);
            if (int rc = enqueue_rounds(st.cl, p, st.launched, to, s)) return rc;
        }
        ROGTK_HIP_CHECK(hipMemcpyAsync(hflags + st.launched, p.flags + st.launched,
                                       (to - st.launched) * sizeof(unsigned int), hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipStreamSynchronize(s));
        const int z = first_zero(hflags, st.launched, to);
        converged = z >= 0;
        if (converged) st.rounds = st.needed = z + 1;
        st.launched = to;
    }
    st.pending = false;
    ROGTK_REQUIRE(converged, ROGTK_E_HIP, "cluster: union rounds did not converge in %d rounds", kMaxRounds);
    if (int rc = enqueue_labels(st.cl, p, s, nullptr)) return rc;
    if (st.deferred.on) {  // the assign that ran on the speculative labels, again
        st.deferred.on = false;
        return enqueue_assign(st.cl, p, st.word_labels ? 1 : st.exact ? 2 : 0, st.deferred.codes, st.deferred.regbits, st.deferred.n,
                              st.deferred.cid, s);
    }
    return ROGTK_OK;
}
}  // namespace

int cluster_set_spec_rounds(int n) {
    ROGTK_REQUIRE(n >= 0 && n <= kMaxRounds, ROGTK_E_INVALID, "spec rounds %d outside 0..%d", n, kMaxRounds);
    g_spec_rounds.store(n == 0 ? kSpecRounds : n);
    g_spec_adaptive.store(n == 0);
    return ROGTK_OK;
}

int cluster_set_lookback_polls(int n) {
    ROGTK_REQUIRE(n >= -1, ROGTK_E_INVALID, "look-back polls %d < -1", n);
    g_lb_polls.store(n < 0 ? kLbMaxPolls : n);
    return ROGTK_OK;
}

int cluster_rounds(const void* ws, hipStream_t s, int* rounds) {
    if (int rc = cluster_finish(ws, s)) return rc;
    std::lock_guard<std::mutex> lk(g_rs_mu);
    auto it = g_rs.find(ws);
    *rounds = it == g_rs.end() ? 0 : it->second.rounds;
    return ROGTK_OK;
}

void cluster_release(const void* ws) {
    std::lock_guard<std::mutex> lk(g_rs_mu);
    auto it = g_rs.find(ws);
    if (it == g_rs.end()) return;
    if (it->second.hstats) {
        if (it->second.pending) (void)wait_published(it->second);  // the kernel writes into it
        hipHostFree(it->second.hstats);
    }
    g_rs.erase(it);
}

int launch_cluster_assign(const ClusterLayout& cl, const uint8_t* ws, const uint32_t* codes,
                          const uint64_t* regular_bits, int64_t n, uint32_t* cluster_id,
                          hipStream_t s, bool deferred) {
    if (!deferred)
        if (int rc = cluster_finish(ws, s)) return rc;
    WsPtrs p = ws_ptrs(cl, const_cast<uint8_t*>(ws));
    int wl = 0;
    {
        std::lock_guard<std::mutex> lk(g_rs_mu);
        auto it = g_rs.find(ws);
        if (it != g_rs.end()) {
            wl = it->second.word_labels ? 1 : it->second.exact ? 2 : 0;
            if (deferred && it->second.pending) {
                auto& d = it->second.deferred;
                d.on = true;
                d.codes = codes;
                d.regbits = regular_bits;
                d.n = n;
                d.cid = cluster_id;
            }
        }
    }
    return enqueue_assign(cl, p, wl, codes, regular_bits, n, cluster_id, s);
}

int cluster_assign_prepare(const ClusterLayout& cl, const uint8_t* ws, const uint32_t* codes,
                           const uint64_t* regular_bits, int64_t n, uint32_t* cluster_id, hipStream_t s,
                           bool deferred, AssignIn* a) {
    a->wlab = nullptr;
    a->wexc = nullptr;
    a->labelcode = nullptr;
    a->out = nullptr;
    if (!deferred)
        if (int rc = cluster_finish(ws, s)) return rc;
    bool wl = false;
    {
        std::lock_guard<std::mutex> lk(g_rs_mu);
        auto it = g_rs.find(ws);
        if (it != g_rs.end()) {
            wl = it->second.word_labels;
            if (deferred && it->second.pending) {  // re-run as a plain assign if not converged
                auto& d = it->second.deferred;
                d.on = true;
                d.codes = codes;
                d.regbits = regular_bits;
                d.n = n;
                d.cid = cluster_id;
            }
        }
    }
    if (!wl || !cl.label_by_code) return ROGTK_OK;
    WsPtrs p = ws_ptrs(cl, const_cast<uint8_t*>(ws));
    a->wlab = p.wpref;
    a->wexc = p.G;
    a->labelcode = p.labelcode;
    a->out = cluster_id;
    return ROGTK_OK;
}

int launch_cluster_lookup(const ClusterLayout& cl, const uint8_t* ws, const uint64_t* q, int64_t nq, uint32_t* lab,
                          hipStream_t s) {
    if (nq <= 0) return ROGTK_OK;
    if (int rc = cluster_finish(ws, s)) return rc;
    WsPtrs p = ws_ptrs(cl, const_cast<uint8_t*>(ws));
    bool wl = false;
    {
        std::lock_guard<std::mutex> lk(g_rs_mu);
        auto it = g_rs.find(ws);
        if (it != g_rs.end()) wl = it->second.word_labels;
    }
    const uint32_t* wlab = wl ? p.wpref : nullptr;
    const uint64_t* wexc = wl ? p.G : nullptr;
    const int g = grid_for(nq, 4096);
    if (cl.label_by_code)
        hipLaunchKernelGGL(k_lookup<0>, dim3(g), dim3(kBlock), 0, s, q, nq, cl.nbits, p.labelcode, p.D, p.RT, wlab,
                           wexc, lab);
    else
        hipLaunchKernelGGL(k_lookup<1>, dim3(g), dim3(kBlock), 0, s, q, nq, cl.nbits, p.labelcode, p.ilab, p.RT, wlab,
                           wexc, lab);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

#ifndef ROGTK_ASSIGN_WGS
#define ROGTK_ASSIGN_WGS 2  // workgroups per CU of k_assign (experiment builds)
#endif
#ifndef ROGTK_ASSIGN_G
#define ROGTK_ASSIGN_G 2  // 4-row groups per lane and trip (experiment builds)
#endif
namespace {
int enqueue_assign(const ClusterLayout& cl, const WsPtrs& p, int labels, const uint32_t* codes,
                   const uint64_t* regular_bits, int64_t n, uint32_t* cluster_id, hipStream_t s) {
    if (n <= 0) return ROGTK_OK;
    const uint32_t* wlab = labels == 1 ? p.wpref : nullptr;
    const uint64_t* wexc = labels == 1 ? p.G : nullptr;
    ProfScope prof(K_ASSIGN, s, true);  // events on the dispatch packet (kernel time only)
    // Two workgroups per CU, grid-stride: assign runs beside the next batch's resolve,
    // whose hook rounds are latency-bound; a full grid of gathers (40k waves at 10M rows)
    // slowed the concurrent hook round 0 from 31 to 94 us. Measured at 10M rows, 2-deep
    // pipeline: 0.425 ms/step full grid, 0.382-0.385 at 512 workgroups (256 CUs); 4-row
    // groups per lane and trip 1 / 4 instead of 2, or a full grid, measured slower (round 3)
    static const int64_t cap = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return (int64_t)ROGTK_ASSIGN_WGS * cus;
    }();
    constexpr int kGroups = ROGTK_ASSIGN_G;
    const int g = grid_for((n + 4 * kGroups - 1) / (4 * kGroups), cap);
    if (labels == 2)  // exact ids: the ranks
        hipExtLaunchKernelGGL((k_assign<2, kGroups>), dim3(g), dim3(kBlock), 0, s, prof.start(), prof.stop(), 0, codes,
                              regular_bits, n, p.labelcode, p.ilab, p.RT, wlab, wexc, cluster_id);
    else if (cl.label_by_code)
        hipExtLaunchKernelGGL((k_assign<0, kGroups>), dim3(g), dim3(kBlock), 0, s, prof.start(), prof.stop(), 0, codes,
                              regular_bits, n, p.labelcode, p.D, p.RT, wlab, wexc, cluster_id);
    else
        hipExtLaunchKernelGGL((k_assign<1, kGroups>), dim3(g), dim3(kBlock), 0, s, prof.start(), prof.stop(), 0, codes,
                              regular_bits, n, p.labelcode, p.ilab, p.RT, wlab, wexc, cluster_id);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}
}  // namespace



// ------------------------------------------------- mark by partition sort
// The presence bitmap straight from the codes, without the 4^L presence bytes: one
// 8-bit radix pass (hipcub onesweep) groups the codes by their top 8 bits (256 code
// partitions of 4^L / 256 codes), then one workgroup per partition sets its bits in an
// LDS bitmap (4^(L-4) bits: 8 KB at L = 12, 32 KB at L = 13) and writes that slice of the
// bitmap with plain coalesced stores. HBM traffic: codes read 3x + written once (~160 MB
// at 10M rows) against 8x re-reads + scattered byte stores + the presence sweep.
namespace {

constexpr int kPartBits = 8;
constexpr int kPartBlock = 512;

__global__ __launch_bounds__(kBlock) void k_mark_keys(const uint32_t* __restrict__ codes,
                                                      const uint64_t* __restrict__ regbits, int64_t n,
                                                      uint32_t* __restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const bool reg = (regbits[i >> 6] >> (i & 63)) & 1ull;
    keys[i] = reg ? codes[i] : 0xFFFFFFFFu;  // sentinel >= 4^L: skipped by k_part_bitmap
}

// First index i with a[i] >= v (n if none), found by the whole workgroup: each round
// probes kPartBlock evenly spaced positions of [lo, hi] at once, so 10M keys take ~4
// dependent loads instead of ~24. a[0, n) must be ordered by the predicate a[i] < v.
__device__ int64_t wg_lower_bound(const uint32_t* __restrict__ a, int64_t n, uint64_t v) {
    int64_t lo = 0, hi = n;  // the answer lies in [lo, hi]
    while (lo < hi) {
        const int64_t step = (hi - lo + kPartBlock - 1) / kPartBlock;
        const int64_t pos = lo + (int64_t)threadIdx.x * step;
        const bool less = pos < hi && (uint64_t)a[pos] < v;
        const int64_t cnt = __syncthreads_count(less);
        const int64_t nlo = cnt ? lo + (cnt - 1) * step + 1 : lo;
        const int64_t nhi = min(hi, lo + cnt * step);
        lo = nlo;
        hi = nhi;
    }
    return lo;
}

__global__ __launch_bounds__(kPartBlock) void k_part_bitmap(const uint32_t* __restrict__ sorted, int64_t n,
                                                            int two_l, uint64_t* __restrict__ bitmap) {
    extern __shared__ uint32_t lbits[];  // 2^(two_l - 8) bits
    const int p = blockIdx.x;
    const int shift = two_l - kPartBits;
    const uint32_t pwords32 = (1u << shift) >> 5;  // >= 1 for two_l >= 13
    for (uint32_t k = threadIdx.x; k < pwords32; k += kPartBlock) lbits[k] = 0;
    __shared__ int64_t range[2];
    const int64_t r0 = wg_lower_bound(sorted, n, (uint64_t)p << shift);
    // the sort orders the partition bits only: sentinels share the last bucket with real
    // codes, so that bucket runs to the end and skips them one by one
    const int64_t r1 = p + 1 == (1 << kPartBits) ? n : wg_lower_bound(sorted, n, (uint64_t)(p + 1) << shift);
    if (threadIdx.x == 0) {
        range[0] = r0;
        range[1] = r1;
    }
    __syncthreads();
    const uint32_t mask = (1u << shift) - 1u;
    // 8 independent loads in flight per lane before the LDS atomics that consume them
    constexpr int kUnroll = 8;
    const int64_t rend = range[1];
    for (int64_t i0 = range[0] + threadIdx.x; i0 < rend; i0 += (int64_t)kPartBlock * kUnroll) {
        uint32_t key[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t i = i0 + (int64_t)u * kPartBlock;
            key[u] = i < rend ? __builtin_nontemporal_load(sorted + i) : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            if ((uint64_t)key[u] >> two_l) continue;  // irregular-row sentinel / past the range
            const uint32_t c = key[u] & mask;
            atomicOr(&lbits[c >> 5], 1u << (c & 31));
        }
    }
    __syncthreads();
    uint64_t* out = bitmap + ((uint64_t)p << shift >> 6);
    for (uint32_t k = threadIdx.x; k < pwords32 / 2; k += kPartBlock)
        out[k] = (uint64_t)lbits[2 * k] | ((uint64_t)lbits[2 * k + 1] << 32);
}

// ---- mark by code slices in LDS (umi_len 7..12, default)
// The code space is cut into slices of 2^20 codes (128 KB of LDS as a bitmap) and the
// rows into kSliceChunks chunks; workgroup (slice s, chunk c) reads chunk c's codes and
// sets the bits of the codes that fall in slice s, then stores its slice of chunk c's
// partial bitmap; one pass ORs the chunks' partials. Every code is read once from HBM:
// the slices of one chunk are the workgroups b = s * chunks + c, which share the XCD
// c % 8 under the round-robin placement (measured exact; speed only), so their repeated
// reads of the chunk hit that XCD's L2. No sort, no scattered global stores.
#ifndef ROGTK_SLICE_BLOCK
#define ROGTK_SLICE_BLOCK 1024
#endif
constexpr int kSliceBlock = ROGTK_SLICE_BLOCK;
constexpr int kSliceChunks = 8;    // a multiple of the 8 XCDs (round 3: 8 vs 16 chunks 0.318-0.327 vs 0.322-0.345 ms/step)
#ifndef ROGTK_SLICE_LOG2
#define ROGTK_SLICE_LOG2 20
#endif
constexpr int kSliceLog2 = ROGTK_SLICE_LOG2;  // codes per slice (LDS bits)
constexpr int kSliceBits = 24 - kSliceLog2;   // log2 of the slices of 4^12
constexpr int kMaxSlices = 1 << kSliceBits;
constexpr int kBucketRows = 8192;  // rows per segment workgroup (8 per lane; default)
constexpr int kSegCap = kBucketRows * 4 / kMaxSlices;  // codes per (slice, workgroup) segment: 4x the mean share

// Segment mode (segs != nullptr, written by k_slice_bucket): workgroup (s, c) reads only
// slice s's segments of the bucket workgroups of chunk c (every code is read once in
// all); if one of them overflowed, it reads those workgroups' rows instead.
__global__ __launch_bounds__(kSliceBlock) void k_slice_mark(const uint32_t* __restrict__ codes,
                                                            const uint64_t* __restrict__ regbits, int64_t n,
                                                            int slice_log2, int chunks, int64_t chunk_rows,
                                                            uint64_t* __restrict__ out, int64_t words,
                                                            const uint32_t* __restrict__ segs = nullptr,
                                                            const uint32_t* __restrict__ seglen = nullptr,
                                                            int nbuckets = 0, int bucket_rows = kBucketRows,
                                                            int seg_cap = kSegCap) {
    __shared__ uint32_t sbits[(1u << kSliceLog2) / 32];  // 128 KB at 2^20: the slice's bits (2^slice_log2 used)
    const int c = blockIdx.x % chunks, sl = blockIdx.x / chunks;
    const uint32_t sw32 = (1u << slice_log2) >> 5;
    for (uint32_t k = threadIdx.x; k < sw32; k += kSliceBlock) sbits[k] = 0;
    __syncthreads();
    const uint32_t smask = (1u << slice_log2) - 1u;
    int64_t r0 = (int64_t)c * chunk_rows, r1 = min(n, r0 + chunk_rows);
    if (segs) {
        // the bucket workgroups of this chunk; a segment longer than kSegCap was not stored
        // (its workgroup overflowed): then this chunk's rows are read instead
        const int b0 = (int)((int64_t)c * nbuckets / chunks), b1 = (int)((int64_t)(c + 1) * nbuckets / chunks);
        bool over = false;
        for (int b = b0 + (int)threadIdx.x; b < b1; b += kSliceBlock)
            over |= seglen[(int64_t)sl * nbuckets + b] > (uint32_t)seg_cap;
        r0 = (int64_t)b0 * bucket_rows;
        r1 = min(n, (int64_t)b1 * bucket_rows);
        if (!__syncthreads_or(over)) {
            // a wave takes kSegInFlight segments at a time (256 codes of each per pass of 16-B
            // loads), all their loads in flight before the LDS atomics: one segment at a time
            // left a wave ~2 dependent HBM round trips per segment (~10 segments per wave at
            // 10M rows, ~60 at 62.5M: the C4 rank's 736 us, round 6)
            constexpr int kSegInFlight = 8;
            constexpr int kWaves = kSliceBlock / 64;
            const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
            for (int bb = b0 + wave; bb < b1; bb += kWaves * kSegInFlight) {
                uint32_t len[kSegInFlight];
                uint32_t mx = 0;
#pragma unroll
                for (int u = 0; u < kSegInFlight; ++u) {
                    const int b = bb + u * kWaves;
                    len[u] = b < b1 ? seglen[(int64_t)sl * nbuckets + b] : 0u;
                    mx = max(mx, len[u]);
                }
                for (uint32_t i = 4 * lane; i < mx; i += 256) {
                    uint4 v[kSegInFlight];
#pragma unroll
                    for (int u = 0; u < kSegInFlight; ++u) {
                        const uint32_t* seg = segs + ((int64_t)sl * nbuckets + bb + u * kWaves) * seg_cap;
                        v[u] = i < len[u] ? *reinterpret_cast<const uint4*>(seg + i) : make_uint4(0, 0, 0, 0);
                    }
#pragma unroll
                    for (int u = 0; u < kSegInFlight; ++u) {
                        const uint32_t cc[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            if (i + k < len[u]) {
                                const uint32_t b2 = cc[k] & smask;
                                atomicOr(&sbits[b2 >> 5], 1u << (b2 & 31));
                            }
                    }
                }
            }
            r1 = r0;  // no row pass
        }
    }
    // kSliceUnroll independent 16-B loads in flight per lane before the LDS atomics that
    // consume them (one load per iteration left the kernel latency-bound: 125 us)
    constexpr int kSliceUnroll = 8;
    constexpr int64_t kStep = 4 * (int64_t)kSliceBlock;
    for (int64_t rb = r0 + 4 * (int64_t)threadIdx.x; rb < r1; rb += kStep * kSliceUnroll) {
        uint4 v[kSliceUnroll];
        uint32_t reg[kSliceUnroll];
#pragma unroll
        for (int u = 0; u < kSliceUnroll; ++u) {
            const int64_t r = rb + u * kStep;
            reg[u] = 0;
            v[u] = make_uint4(0, 0, 0, 0);
            if (r + 4 <= r1) {
                v[u] = *reinterpret_cast<const uint4*>(codes + r);
                reg[u] = regbits ? (uint32_t)(regbits[r >> 6] >> (r & 63)) & 0xFu : 0xFu;  // r % 4 == 0
            } else if (r < r1) {
                v[u].x = codes[r];
                if (r + 1 < r1) v[u].y = codes[r + 1];
                if (r + 2 < r1) v[u].z = codes[r + 2];
                reg[u] = (regbits ? (uint32_t)(regbits[r >> 6] >> (r & 63)) & 0xFu : 0xFu) &
                         ((1u << (uint32_t)(r1 - r)) - 1u);
            }
        }
#pragma unroll
        for (int u = 0; u < kSliceUnroll; ++u) {
            const uint32_t cc[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (((reg[u] >> k) & 1u) && (cc[k] >> slice_log2) == (uint32_t)sl) {  // codes >= 4^L never match
                    const uint32_t b = cc[k] & smask;
                    atomicOr(&sbits[b >> 5], 1u << (b & 31));
                }
        }
    }
    __syncthreads();
    uint64_t* o = out + (int64_t)c * words + (((int64_t)sl << slice_log2) >> 6);
    for (uint32_t k = threadIdx.x; k < sw32 / 2; k += kSliceBlock)
        o[k] = (uint64_t)sbits[2 * k] | ((uint64_t)sbits[2 * k + 1] << 32);
}

// Pass 1 of the segment mode: one workgroup per kBucketRows rows ranks its valid codes
// by slice (lanes of a wave with one slice found by 4 ballots, one LDS atomic per slice
// and wave) and stores them into its own segment of each slice (kSegCap codes, 4x the
// mean share at 16 slices), with the segment lengths: no global atomics (a global
// cursor per slice, hit by every workgroup, serialised the pass to 236 us). A segment
// that would overflow is not stored (its length says so), and the slice pass reads the
// rows of that chunk instead.
constexpr int kBucketThreads = 1024;  // 8 rows per lane: short rank chains per wave
template <int kBucketRows, int kBucketThreads>
__global__ __launch_bounds__(kBucketThreads) void k_slice_bucket(const uint32_t* __restrict__ codes,
                                                         const uint64_t* __restrict__ regbits, int64_t n,
                                                         int slice_log2, int nslices, uint32_t* __restrict__ segs,
                                                         uint32_t* __restrict__ seglen, int nbuckets) {
    __shared__ unsigned int cnt[kMaxSlices], lbase[kMaxSlices + 1];
    constexpr int kSegCap = kBucketRows * 4 / kMaxSlices;  // 4x the mean share
    __shared__ uint32_t stage[kBucketRows];
    const int t = threadIdx.x, lane = t & 63;
    if (t < kMaxSlices) cnt[t] = 0;
    __syncthreads();
    const int64_t row0 = (int64_t)blockIdx.x * kBucketRows;
    constexpr int kPer = kBucketRows / kBucketThreads / 4;  // uint4 loads per lane
    uint32_t key[kPer * 4];  // slice << 16 | index within the slice's segment, or kNone
    uint32_t val[kPer * 4];
    uint32_t regs[kPer];
    // all kPer 16-B loads in flight before the ranking that consumes them
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const int64_t r = row0 + 4 * ((int64_t)u * kBucketThreads + t);
        uint4 v = make_uint4(0, 0, 0, 0);
        uint32_t reg = 0;
        if (r + 4 <= n) {
            v = *reinterpret_cast<const uint4*>(codes + r);
            reg = regbits ? (uint32_t)(regbits[r >> 6] >> (r & 63)) & 0xFu : 0xFu;
        } else if (r < n) {
            v.x = codes[r];
            if (r + 1 < n) v.y = codes[r + 1];
            if (r + 2 < n) v.z = codes[r + 2];
            reg = (regbits ? (uint32_t)(regbits[r >> 6] >> (r & 63)) & 0xFu : 0xFu) & ((1u << (uint32_t)(n - r)) - 1u);
        }
        val[4 * u] = v.x;
        val[4 * u + 1] = v.y;
        val[4 * u + 2] = v.z;
        val[4 * u + 3] = v.w;
        regs[u] = reg;
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t sl = val[4 * u + k] >> slice_log2;
            const bool ok = ((regs[u] >> k) & 1u) && sl < (uint32_t)nslices;
            uint64_t peers = __ballot(ok);
#pragma unroll
            for (int bit = 0; bit < kSliceBits; ++bit) {
                const uint64_t b = __ballot((sl >> bit) & 1u);
                peers &= ((sl >> bit) & 1u) ? b : ~b;
            }
            const int leader = peers ? __ffsll((long long)peers) - 1 : 0;
            unsigned int base = 0;
            if (ok && lane == leader) base = atomicAdd(&cnt[sl], (unsigned int)__popcll(peers));
            base = __shfl(base, leader);
            key[4 * u + k] = ok ? (sl << 16) | (base + (uint32_t)__popcll(peers & ((1ull << lane) - 1ull))) : kNone;
        }
    }
    __syncthreads();
    if (t < nslices) seglen[(int64_t)t * nbuckets + blockIdx.x] = cnt[t];  // > kSegCap: not stored
    if (t == 0) {
        unsigned int acc = 0;
        for (int k = 0; k < nslices; ++k) {
            lbase[k] = acc;
            acc += cnt[k];
        }
        lbase[nslices] = acc;
    }
    __syncthreads();
    // stage sorted by slice in LDS, then store each slice's run contiguously
#pragma unroll
    for (int u = 0; u < kPer * 4; ++u) {
        const uint32_t kk = key[u];
        if (kk != kNone) stage[lbase[kk >> 16] + (kk & 0xFFFFu)] = val[u];
    }
    __syncthreads();
    const unsigned int total = lbase[nslices];
    for (unsigned int i = t; i < total; i += kBucketThreads) {
        const uint32_t c = stage[i];
        const uint32_t sl = c >> slice_log2;
        if (cnt[sl] <= (unsigned int)kSegCap) segs[((int64_t)sl * nbuckets + blockIdx.x) * kSegCap + (i - lbase[sl])] = c;
    }
}

__global__ __launch_bounds__(kBlock) void k_or_partials(const uint64_t* __restrict__ partials, int chunks,
                                                        int64_t words, uint64_t* __restrict__ out) {
    for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < words; w += (int64_t)gridDim.x * kBlock) {
        uint64_t v = 0;
        for (int c = 0; c < chunks; ++c) v |= __builtin_nontemporal_load(partials + (int64_t)c * words + w);
        out[w] = v;
    }
}

// chunks of the slice mark for n rows (1 = the slices write the bitmap directly; with one
// chunk at 10M rows only 16 workgroups run: measured 2x slower; 16 chunks measured slower
// than 8, round 3)
inline int slice_chunks(int64_t n) { return n >= (1 << 20) ? kSliceChunks : 1; }
inline bool slice_segments(int64_t n) { return n >= (1 << 20); }  // the bucket pass runs
inline int slices_of(int L) { return 1 << (2 * L - std::min(2 * L, kSliceLog2)); }
inline int64_t seg_buckets(int64_t n) { return (n + kBucketRows - 1) / kBucketRows; }
// segments + their lengths of the segment mode (bucket workgroups of 2048 / 4096 rows
// measured neutral against 8192, round 3)
inline int64_t seg_bytes(int64_t n) {
    return ((int64_t)kMaxSlices * seg_buckets(n) * kSegCap * 4) + ((int64_t)kMaxSlices * seg_buckets(n) * 4 + 255) / 256 * 256;
}
// ROGTK_SLICE_BUCKETS=0: slices read all rows (A/B)
inline bool slice_buckets_on() {
    static const bool on = [] {
        const char* e = getenv("ROGTK_SLICE_BUCKETS");
        return !(e && e[0] == '0');
    }();
    return on;
}

size_t part_sort_temp(int64_t n) {
    size_t tb = 0;
    hipcub::DeviceRadixSort::SortKeys(nullptr, tb, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 8);
    return tb;
}

}  // namespace

namespace {
// mark_bitmap method: 0 auto (slices for umi_len <= 12, partition sort for 13), 1 sort, 2 slices
std::atomic<int> g_mark_method{0};
bool use_slices(int L) {
    const int m = g_mark_method.load();
    return L <= 12 && m != 1;
}
}  // namespace

int cluster_set_mark_method(int m) {
    ROGTK_REQUIRE(m >= 0 && m <= 2, ROGTK_E_INVALID, "mark method %d outside 0..2", m);
    g_mark_method.store(m);
    return ROGTK_OK;
}

int cluster_mark_bitmap_temp(int64_t n, int L, int64_t* bytes) {
    ROGTK_REQUIRE(L >= 7 && L <= 13, ROGTK_E_UNSUPPORTED, "mark_bitmap needs umi_len 7..13, got %d", L);
    ROGTK_REQUIRE(n >= 0 && n < ((int64_t)1 << 31), ROGTK_E_INVALID, "n outside 0..2^31-1");
    const int64_t nn = std::max<int64_t>(n, 1);
    // both methods' scratch, so that the method can be switched on a live buffer
    const int64_t sort_bytes = 2 * ((nn * 4 + 255) / 256 * 256) + (int64_t)part_sort_temp(nn) + 256;
    const int64_t words = ((int64_t)1 << (2 * L)) / 64;
    int64_t slice_bytes = 0;
    if (L <= 12 && slice_segments(nn)) {
        slice_bytes = slice_chunks(nn) > 1 ? (int64_t)slice_chunks(nn) * words * 8 : 0;
        if (slices_of(L) > 1) slice_bytes += seg_bytes(nn);
    }
    *bytes = std::max(sort_bytes, slice_bytes);
    return ROGTK_OK;
}

int launch_cluster_mark_bitmap(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int L,
                               uint64_t* bitmap, void* temp, int64_t temp_bytes, hipStream_t s) {
    return launch_cluster_mark_phase(codes, regular_bits, n, L, bitmap, temp, temp_bytes, 0, s);
}

// phase 0: the whole mark; 1: the slice-bucket pass alone (nothing when the code-slice
// segments do not apply to (n, L)); 2: the rest (slice mark + OR of the chunk partials, or
// the partition sort), to be enqueued after phase 1 (round 5: the pipeline runs phase 1 on
// the main stream and phase 2 at the head of the resolve stream, beside the score kernel)
int launch_cluster_mark_phase(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int L,
                              uint64_t* bitmap, void* temp, int64_t temp_bytes, int phase, hipStream_t s) {
    ROGTK_REQUIRE(phase >= 0 && phase <= 2, ROGTK_E_INVALID, "mark_bitmap: phase %d", phase);
    int64_t need = 0;
    if (int rc = cluster_mark_bitmap_temp(n, L, &need)) return rc;
    ROGTK_REQUIRE((temp || n == 0) && temp_bytes >= need, ROGTK_E_INVALID, "temp_bytes %lld < %lld", (long long)temp_bytes,
                  (long long)need);
    ProfScope prof(K_MARK, s);
    const int two_l = 2 * L;
    if (n == 0) {
        if (phase != 1) ROGTK_HIP_CHECK(hipMemsetAsync(bitmap, 0, ((size_t)1 << two_l) / 8, s));
        return ROGTK_OK;
    }
    ROGTK_REQUIRE(((uintptr_t)codes & 15u) == 0, ROGTK_E_INVALID, "mark_bitmap: codes must be 16-byte aligned");
    if (use_slices(L)) {
        const int slog = std::min(two_l, kSliceLog2);
        const int slices = 1 << (two_l - slog);
        const int chunks = slice_chunks(n);
        int64_t chunk_rows = (n + chunks - 1) / chunks;
        chunk_rows = (chunk_rows + 3) / 4 * 4;  // rows of a chunk start 4-aligned (uint4 loads)
        const int64_t words = ((int64_t)1 << two_l) / 64;
        uint64_t* dst = chunks > 1 ? (uint64_t*)temp : bitmap;
        const uint32_t* segs = nullptr;
        uint32_t* seglen = nullptr;
        const int nb = (int)seg_buckets(n);
        if (slice_segments(n) && slices > 1 && slices <= kMaxSlices && slice_buckets_on()) {
            // segment pass: every slice workgroup then reads only its slice's codes (the
            // chunks of all rows were read once per slice: 16x at L = 12, from L2)
            segs = (const uint32_t*)((uint8_t*)temp + (chunks > 1 ? (int64_t)chunks * words * 8 : 0));
            seglen = (uint32_t*)((uint8_t*)segs + (int64_t)kMaxSlices * nb * kSegCap * 4);
            if (phase != 2)
                ROGTK_TIMED_LAUNCH(K_K_SLICE_BUCKET, (k_slice_bucket<kBucketRows, kBucketThreads>), dim3((unsigned)nb),
                                   dim3(kBucketThreads), 0, s, codes, regular_bits, n, slog, slices, (uint32_t*)segs,
                                   seglen, nb);
        }
        if (phase == 1) {
            ROGTK_HIP_CHECK(hipGetLastError());
            return ROGTK_OK;
        }
        ROGTK_TIMED_LAUNCH(K_K_SLICE_MARK, k_slice_mark, dim3((unsigned)(slices * chunks)), dim3(kSliceBlock), 0, s, codes, regular_bits,
                           n, slog, chunks, chunk_rows, dst, words, segs, (const uint32_t*)seglen, nb, kBucketRows, kSegCap);
        if (chunks > 1)
            ROGTK_TIMED_LAUNCH(K_K_OR_PARTIALS, k_or_partials, dim3(grid_for(words, 4096)), dim3(kBlock), 0, s, dst, chunks, words,
                               bitmap);
        ROGTK_HIP_CHECK(hipGetLastError());
        return ROGTK_OK;
    }
    if (phase == 1) return ROGTK_OK;  // the partition sort is one phase
    const int64_t slab = (n * 4 + 255) / 256 * 256;
    uint32_t* keys_in = (uint32_t*)temp;
    uint32_t* keys_out = (uint32_t*)((uint8_t*)temp + slab);
    void* cub = (uint8_t*)temp + 2 * slab;
    const uint32_t* src = codes;
    if (regular_bits) {
        hipLaunchKernelGGL(k_mark_keys, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, codes,
                           regular_bits, n, keys_in);
        src = keys_in;
    }
    size_t tb = part_sort_temp(n);
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(cub, tb, src, keys_out, (int)n, two_l - kPartBits, two_l, s));
    const size_t lds = ((size_t)1 << (two_l - kPartBits)) / 8;
    hipLaunchKernelGGL(k_part_bitmap, dim3(1u << kPartBits), dim3(kPartBlock), lds, s, keys_out, n, two_l, bitmap);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

}  // namespace rogtk

#ifdef ROGTK_LCC_TIMING
// experiment builds only: the accumulated k_local_cc clocks (wall_clock64 ticks, summed
// over workgroups: phases 0..3, whole workgroup, workgroup count), then zeroed
extern "C" int rogtk_debug_lcc_clock(unsigned long long* out8) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(rogtk::g_lcc_clk), 64) != hipSuccess) return 1;
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(rogtk::g_lcc_clk), z, 64) == hipSuccess ? 0 : 1;
}
#endif
