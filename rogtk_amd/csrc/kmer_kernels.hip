// kmer_kernels.hip — H4: k-mer spectra of read groups on gfx950.
//
// Replaces, per polars group, the k-mer front end of rogtk's fracture assembly:
//   expressions.rs:739-744  sequences = column.into_iter().flatten()
//   fracture.rs:200-229     auto_k (estimate_k :24-54), k > 64 -> nothing, uppercase,
//                           drop sequences with any non-ACGT byte
//   fracture.rs:246-256     effective k = 4 / 8 / 16 / 32 / 64
//   fracture.rs:105-116     debruijn 0.3.4 filter_kmers(CountFilter(min_cov), stranded,
//                           report_all) + remove_censored_exts
//   fracture.rs:118-146     node / terminal / isolated counts
// Output per group: its valid k-mers in ascending order (the crate's pre-MPHF order)
// with the censored Exts byte (low nibble = left bases, high = right) and the
// saturating u16 count. Spec and the oracle: oracle/kmer_oracle.cpp.
//
// Device pipeline for one effective k (groups of other k are skipped):
//   rows    one wave per row: group lookup, ACGT check (ballot), observation count
//   emit    one wave per row: every k-mer observation -> (key lo[, hi], ext, group)
//   sort    LSD radix passes (hipcub, stable): key lo, [key hi], group -> permutation
//   runs    run heads -> run count (saturating) + OR of exts -> CountFilter
//   censor  binary search of each extension's neighbour inside the group's valid run
//   out     entries at the group's capacity offset; host packs them densely
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstdlib>
#include <memory>
#include <vector>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / 64;
constexpr int64_t kMaxObsPerLaunch = int64_t(1) << 30;  // u32 permutation indices

__device__ __forceinline__ uint32_t base2(uint8_t c) { return (uint32_t)((c >> 1) ^ (c >> 2)) & 3u; }
__device__ __forceinline__ bool acgt(uint8_t c) {
    const uint8_t u = c & 0xDF;  // ASCII upper case for letters; other bytes stay non-ACGT
    return u == 'A' || u == 'C' || u == 'G' || u == 'T';
}

template <int OW>
__device__ __forceinline__ void span(const void* offsets, int64_t r, int64_t& st, int64_t& len) {
    if (OW == 4) {
        const int32_t* o = (const int32_t*)offsets;
        st = o[r];
        len = (int64_t)o[r + 1] - o[r];
    } else {
        const int64_t* o = (const int64_t*)offsets;
        st = o[r];
        len = o[r + 1] - o[r];
    }
}

// Grouped row r -> its span in the column (one thread per row: the rows[] ->
// offsets[] chain runs 64x wider than per wave). raw_len = -1 for rows that take no
// part (null, or a group of another effective k); words = 2-bit words to stage.
template <int OW>
__global__ __launch_bounds__(kBlock) void k_row_meta(const void* offsets, const uint8_t* __restrict__ validity,
                                                     int64_t voff, const int64_t* __restrict__ rows, int64_t n_rows,
                                                     const uint8_t* __restrict__ gk, int K,
                                                     const uint32_t* __restrict__ row_group,
                                                     int64_t* __restrict__ row_st, int32_t* __restrict__ raw_len,
                                                     int64_t* __restrict__ row_words) {
    for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < n_rows; r += (int64_t)gridDim.x * kBlock) {
        const int64_t pr = rows ? rows[r] : r;
        bool valid = gk[row_group[r]] == K;
        if (valid && validity) {
            const int64_t b = voff + pr;
            valid = (validity[b >> 3] >> (b & 7)) & 1;
        }
        int64_t st = 0, len = 0;
        if (valid) span<OW>(offsets, pr, st, len);
        row_st[r] = st;
        raw_len[r] = valid ? (int32_t)len : -1;
        row_words[r] = valid ? (len + 31) >> 5 : 0;
    }
}

// 32 bits -> 64: bit i of x moves to bit 2i
__device__ __forceinline__ uint64_t spread2(uint32_t x) {
    uint64_t v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
}

// 64 bases of one row, one byte per lane (base j0 + lane): the ACGT check and the 2-bit
// pack by two ballots (base j at bits 62 - 2 (j % 32) of word j / 32, first base most
// significant; bytes past the row end pack as 0). Returns this lane's "bad byte".
__device__ __forceinline__ bool stage_chunk(uint8_t c, int64_t j0, int64_t len, int lane, uint64_t* out) {
    const bool in = j0 + lane < len;
    const uint32_t b = in ? base2(c) : 0u;
    const uint64_t lo = __ballot(b & 1u), hi = __ballot(b & 2u);
    if (lane < 2) {
        const int64_t w = (j0 >> 5) + lane;
        const uint32_t l32 = (uint32_t)(lo >> (32 * lane)), h32 = (uint32_t)(hi >> (32 * lane));
        if (w * 32 < len)
            out[w] = (spread2(__builtin_bitreverse32(h32)) << 1) | spread2(__builtin_bitreverse32(l32));
    }
    return in && !acgt(c);
}

// One wave per 64 grouped rows: every row's metadata in one coalesced load (a lane per
// row), then the rows' bytes kRowBatch rows at a time (their first 256 bytes in flight
// together), loaded once: the ACGT check of fracture.rs:217-229 (ballot), the 2-bit
// staging (packed[woff[r] ..], base j in word j / 32 at bits 62 - 2 (j % 32)), and, a
// lane per row again, the observation counts and n_sequences (one atomic per run of
// same-group rows).
__global__ __launch_bounds__(kBlock) void k_row_stage(const uint8_t* __restrict__ values, int64_t n_rows, int K,
                                                      const uint32_t* __restrict__ row_group,
                                                      const int64_t* __restrict__ row_st,
                                                      const int32_t* __restrict__ raw_len,
                                                      const int64_t* __restrict__ woff,
                                                      uint64_t* __restrict__ packed,
                                                      int64_t* __restrict__ row_obs, int32_t* __restrict__ row_len,
                                                      unsigned long long* __restrict__ gstat) {
    constexpr int kRowBatch = 4;
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t rb = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 64; rb < n_rows;
         rb += waves * 64) {
        const int64_t r = rb + lane;
        const bool live = r < n_rows;
        const int32_t my_len = live ? raw_len[r] : -1;
        const int64_t my_st = live ? row_st[r] : 0, my_wo = live ? woff[r] : 0;
        const uint32_t my_g = live ? row_group[r] : 0u;
        const int nq = (int)min<int64_t>(64, n_rows - rb);
        uint64_t okbits = 0;  // rows of this trip that pass the ACGT check
        for (int q0 = 0; q0 < nq; q0 += kRowBatch) {
            int64_t L[kRowBatch], S[kRowBatch];
            uint8_t cb[kRowBatch][4];
#pragma unroll
            for (int k = 0; k < kRowBatch; ++k) {
                const int q = min(q0 + k, nq - 1);
                L[k] = q0 + k < nq ? __shfl(my_len, q) : -1;
                S[k] = __shfl(my_st, q);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int64_t j = (int64_t)u * 64 + lane;
                    cb[k][u] = j < L[k] ? values[S[k] + j] : (uint8_t)'A';
                }
            }
#pragma unroll
            for (int k = 0; k < kRowBatch; ++k) {
                if (L[k] < 0) continue;  // past the trip, or no part in this call
                uint64_t* out = packed + __shfl(my_wo, q0 + k);
                bool bad = false;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if ((int64_t)u * 64 < L[k]) bad |= stage_chunk(cb[k][u], (int64_t)u * 64, L[k], lane, out);
                for (int64_t j0 = 256; j0 < L[k]; j0 += 64) {  // rows longer than 256 bases
                    const uint8_t c = j0 + lane < L[k] ? values[S[k] + j0 + lane] : (uint8_t)'A';
                    bad |= stage_chunk(c, j0, L[k], lane, out);
                }
                if (__ballot(bad) == 0) okbits |= 1ull << (q0 + k);
            }
        }
        if (live) {
            const bool ok = my_len >= 0 && ((okbits >> lane) & 1ull);
            const bool use = ok && my_len >= K;
            row_obs[r] = use ? my_len - K + 1 : 0;
            row_len[r] = use ? my_len : 0;
            // n_sequences: the first lane of each run of same-group rows adds the run's ok rows
            const uint32_t g_prev = __shfl_up(my_g, 1);
            const uint64_t heads = __ballot(lane == 0 || my_g != g_prev);
            const uint64_t oks = __ballot(ok);
            if ((heads >> lane) & 1ull) {
                const uint64_t above = lane == 63 ? 0ull : heads & (~0ull << (lane + 1));
                const uint64_t run = (above ? (above & (0ull - above)) - 1ull : ~0ull) & (~0ull << lane);
                const int cnt = __popcll(oks & run);
                if (cnt) atomicAdd(gstat + 5 * (int64_t)my_g + 1, (unsigned long long)cnt);
            }
        }
    }
}

// ------------------------------------------------- reads as fixed-stride 2-bit blocks
// A read column packed once, in column order (coalesced), into B-word blocks (B = 8, 16
// or 32: one, two or four 64-B lines per row): word 0 = len (bits 0..31; 0xFFFFFFFF for
// a null row) | ACGT-clean << 32 (fracture.rs:217-229, after upper-casing); words
// 1..B-1 = the bases, 32 per word, first base most significant. The spectrum call then
// gathers each grouped row as whole lines (k_row_gather) instead of re-reading its ASCII
// bytes from a random place (k_row_meta + k_row_stage).
constexpr int kPackInBytes = 40 * 1024;  // a workgroup's rows' bytes, staged in LDS

// per byte of v: 0x80 where the byte is zero (exact, no borrow between bytes)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
    const uint32_t t = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    return ~(t | v | 0x7F7F7F7Fu);
}
// 4 bytes (first base in the low byte) -> 8 bits of 2-bit codes (first base most
// significant), and the 0x80 marks of bytes that are not A/C/G/T in either case
__device__ __forceinline__ uint32_t pack4(uint32_t x, uint32_t& notacgt) {
    const uint32_t c = ((x >> 1) ^ (x >> 2)) & 0x03030303u;  // base2 of every byte
    const uint32_t u = x | 0x20202020u;                       // A/C/G/T -> a/c/g/t (only those map there)
    // a byte is A/C/G/T iff it equals the letter its own 2-bit code names: one byte
    // permute of "acgt" by the codes (v_perm_b32; the table in both sources, so either
    // selector half reads it) and one zero-byte test, instead of four
    constexpr uint32_t kAcgt = 0x74676361u;  // 'a' 'c' 'g' 't', byte 0 first
    const uint32_t expect = __builtin_amdgcn_perm(kAcgt, kAcgt, c);
    notacgt = ~zero_bytes(u ^ expect) & 0x80808080u;
    return ((c & 0xFFu) << 6) | (((c >> 8) & 0xFFu) << 4) | (((c >> 16) & 0xFFu) << 2) | (c >> 24);
}

// Round 4: the repeat certificate of a row (block meta bit 33, set = certified). If no
// 16-mer at an aligned position 16 j (16 j + 16 <= len) occurs again at any other position
// of the row, no K-mer with K >= 31 occurs twice in it: an occurrence [p, p + K) holds the
// whole aligned 16-mer [a, a + 16) for the multiple a of 16 in [p, p + K - 16] (K - 15 >= 16
// consecutive integers), and a second occurrence at p + d holds it again at a + d > a:
// only positions after the aligned one are compared (about half the pairs).
// A group whose rows are all certified and that has fewer than min_cov rows with
// observations then has no k-mer counted min_cov times: nothing passes CountFilter, and
// k_group_classify takes it off the LDS kernels (class kClsEmpty). Necessary-condition
// check only: a pair found (even across the row's end padding) just withholds the bit.
// One lane per row over its NW packed words; compares 16-mers as u32 (alignbit).
// lmax: a wave-uniform bound >= the length of every lane that calls (the loops' exits are
// scalar branches, not a VALU compare + ballot per chunk and aligned position)
template <int NW>
__device__ __forceinline__ bool may_repeat16(const uint64_t (&wd)[NW], int len, int lmax) {
    constexpr int NA = (32 * NW - 16) / 16 + 1;  // aligned 16-mers the words can hold
    // all in VALU, no lane masks: a pair matches when (v ^ a) + inv == 0, where inv = 1 for
    // an aligned position past this row's end (a carry out of 0xFFFFFFFF + 1 also reads as
    // a match: conservative), and the running minimum keeps any zero (v_xad + v_min3; the
    // lane-mask form cost two scalar instructions per pair and doubled the pack kernel)
    uint32_t a[NA], inv[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        a[j] = (j & 1) ? (uint32_t)wd[j >> 1] : (uint32_t)(wd[j >> 1] >> 32);
        inv[j] = 16 * j + 16 <= len ? 0u : 1u;
    }
    // four running minima (by aligned position j & 3): four independent v_min3 chains
    uint32_t acc4[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
#pragma unroll
    for (int wi = 0; wi < NW; ++wi) {
        const uint32_t h0 = (uint32_t)(wd[wi] >> 32), h1 = (uint32_t)wd[wi];
        const uint32_t h2 = wi + 1 < NW ? (uint32_t)(wd[wi + 1] >> 32) : 0u;
#pragma unroll
        for (int t0 = 0; t0 < 32; t0 += 8) {  // 8 positions at a time (few live registers)
            if (32 * wi + t0 + 16 > lmax) break;  // no lane has a 16-mer from here on
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int t = t0 + u;
                v[u] = t == 0 ? h0 : t == 16 ? h1 : t < 16 ? __builtin_amdgcn_alignbit(h0, h1, 32 - 2 * t)
                                                          : __builtin_amdgcn_alignbit(h1, h2, 64 - 2 * t);
            }
#pragma unroll
            for (int j = 0; j < NA; ++j) {
                if (16 * j + 16 > lmax) break;  // aligned positions are valid in order
                // only positions past the aligned one: the first occurrence holds an
                // aligned 16-mer that the second holds again further on. The compared
                // positions of this (chunk, j) are known at compile time: pairs of them
                // fold into acc with one v_min3 each (a chain per (chunk, j); one chain
                // over the chunk is rebalanced by the compiler into min + min3 pairs)
                uint32_t pend = 0;
                bool has = false;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    if (!(32 * wi + t0 + u > 16 * j)) continue;
                    const uint32_t x = (v[u] ^ a[j]) + inv[j];
                    if (has) {
                        acc4[j & 3] = min(min(acc4[j & 3], pend), x);
                        has = false;
                    } else {
                        pend = x;
                        has = true;
                    }
                }
                if (has) acc4[j & 3] = min(acc4[j & 3], pend);
            }
        }
    }
    return min(min(acc4[0], acc4[1]), min(acc4[2], acc4[3])) == 0;
}

// R rows per workgroup (one wave), a lane per row. Each lane stores its row's block itself
// (16-B stores; the lanes' blocks are consecutive, so a wave covers 64 * 8 * B contiguous
// bytes and L2 merges the lines) instead of staging the blocks in LDS for one coalesced
// store: less LDS per workgroup, more workgroups per CU (round 3, 100M 150-bp reads: 12.6
// vs 18.8 ms for 256 rows with LDS-staged stores; 256- and 128-row workgroups with lane
// stores were slower too; a word-parallel variant, B lanes per row, measured neutral).
// Software-pipelined (round 4): the next trip's bytes are loaded into registers (kVin
// dwords per lane) before this trip's rows are packed, and written to LDS after them, so
// each wave's HBM round trip hides behind its own VALU work (the repeat certificate made
// the pack phase ~3.5 us per 64-row trip) instead of being added to it; the row offsets
// are loaded two trips ahead. R = 64: at least 3 waves per SIMD (<= 168 VGPRs: the 40 prefetch
// registers sit beside the certificate's).
template <int B, int R = 64>
__global__ __launch_bounds__(R, 3) void k_pack_reads(const int64_t* __restrict__ offsets,
                                                  const uint8_t* __restrict__ values,
                                                  const uint8_t* __restrict__ validity, int64_t voff,
                                                  int64_t n, uint64_t* __restrict__ blocks,
                                                  unsigned long long* __restrict__ max_len) {
    constexpr int kIn = kPackInBytes * R / kBlock;  // staged bytes: 160 per row
    constexpr int kVin = kIn / 4 / R;               // staged dwords per lane (40)
    // + the funnel shift's 2 zero dwords, a dummy slot, and slack for a word's 9-dword read
    // past the last row's end (< 8 dwords past nw)
    __shared__ uint32_t in32[kIn / 4 + 12];
    __shared__ int64_t s_off[R + 1];
    const int tid = threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * R;
    // a trip's row offsets: lane t holds offsets[a + t] (t <= nr) and offsets[a + t + R]
    // (t + R <= nr, i.e. lane 0 when the trip is full); b0 / b1 = offsets[a], offsets[a + nr]
    // by uniform (scalar) loads
    struct Offs {
        int64_t o0, o1, b0, b1;
    };
    auto load_offs = [&](int64_t aa) {
        Offs f{0, 0, 0, 0};
        if (aa < n) {
            const int nrr = (int)min<int64_t>(R, n - aa);
            f.o0 = offsets[aa + min(tid, nrr)];
            f.o1 = offsets[aa + min(tid + R, nrr)];
            f.b0 = offsets[aa];
            f.b1 = offsets[aa + nrr];
        }
        return f;
    };
    // the bytes [a4, b1) of a trip, in kVin dword registers per lane (+ the last partial
    // dword's bytes); only when they fit the staging area
    uint32_t vin[kVin];
    uint32_t tail = 0;
    auto load_bytes = [&](int64_t b0, int64_t b1) {
        const int64_t a4 = b0 & ~3ll;
        if (b1 - a4 > kIn) return;  // not staged: read byte by byte below
        const int full = (int)((b1 - a4) >> 2);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(values + a4);
        if (full > 0) {
            // all kVin loads, clamped: no branch around a load (which would make the
            // compiler keep vin in scratch), and every load is inside [a4, b1)
#pragma unroll
            for (int u = 0; u < kVin; ++u) vin[u] = src[min(u * R + tid, full - 1)];
        }
        if (4 * full < (int)(b1 - a4)) {  // the last partial dword, byte by byte (never past b1)
            const uint8_t* tb = values + a4 + 4 * full;
            const int left = (int)(b1 - a4) - 4 * full;
            tail = tb[0];
            if (left > 1) tail |= (uint32_t)tb[1] << 8;
            if (left > 2) tail |= (uint32_t)tb[2] << 16;
        }
    };
    int64_t a = (int64_t)blockIdx.x * R;
    Offs cur = load_offs(a), nxt = load_offs(a + stride);
    if (a < n) load_bytes(cur.b0, cur.b1);
    int run_max = 0;  // the longest row of this wave's trips (max_len: one atomic per wave)
    for (; a < n; a += stride) {
        const int nr = (int)min<int64_t>(R, n - a);
        if (tid <= nr) s_off[tid] = cur.o0;
        if (tid + R <= nr) s_off[tid + R] = cur.o1;
        const int64_t b0 = cur.b0, b1 = cur.b1;
        const int64_t a4 = b0 & ~3ll;  // dword-aligned start
        const bool staged = b1 - a4 <= kIn;
        if (staged) {
            const int nw = (int)((b1 - a4 + 3) >> 2);
            const int full = (int)((b1 - a4) >> 2);
            // every lane writes all kVin registers: past `full` into a dummy slot (no branch)
#pragma unroll
            for (int u = 0; u < kVin; ++u) in32[u * R + tid < full ? u * R + tid : kIn / 4 + 2] = vin[u];
            if (full < nw && tid == 0) in32[full] = tail;
            if (tid < 2) in32[nw + tid] = 0;  // the funnel shift below may read one dword past
        }
        __syncthreads();
        // the next trip's bytes and the offsets of the one after, in flight while this trip
        // is packed
        const int64_t an = a + stride;
        if (an < n) load_bytes(nxt.b0, nxt.b1);
        const Offs nn = load_offs(an + stride);
        // a wave-uniform bound on the rows' lengths (the certificate's loop exits)
        int my_len = tid < nr ? (int)(s_off[tid + 1] - s_off[tid]) : 0;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) my_len = max(my_len, __shfl_xor(my_len, m, 64));
        const int lmax = __builtin_amdgcn_readfirstlane(my_len);
        run_max = max(run_max, lmax);
        if (tid < nr) {  // this lane's row, entirely in registers: no cross-lane steps
            const int64_t r = a + tid;
            bool valid = true;
            if (validity) {
                const int64_t bit = voff + r;
                valid = (validity[bit >> 3] >> (bit & 7)) & 1;
            }
            const int64_t st = s_off[tid];
            const int len = (int)(s_off[tid + 1] - st);
            uint32_t bad = 0;
            const int used = valid ? (len + 31) >> 5 : 0;
            const int rel = (int)(st - a4);
            const uint32_t sh = (uint32_t)(rel & 3) * 8;
            // 16-B stores of word pairs (2k, 2k+1); word 1 waits for the meta word
            uint64_t w1 = 0, pend = 0;
            uint64_t* const ob = blocks + r * B;
            uint64_t wd[B == 8 ? B - 1 : 1];  // B = 8: the row's words, for the repeat certificate
#pragma unroll 1
            for (int w = 0; w < B - 1; ++w) {
                uint64_t acc = 0;
                if (w < used) {
                    uint32_t by[8];
                    // the word's 32 bytes: 9 staged dwords from (rel >> 2) + 8 w (read past the
                    // row's end into the slack of in32: masked below)
                    uint32_t t9[9];
                    if (staged) {
                        const int qb = (rel >> 2) + 8 * w;
#pragma unroll
                        for (int i = 0; i < 9; ++i) t9[i] = in32[qb + i];
                    }
#pragma unroll
                    for (int d = 0; d < 8; ++d) {
                        const int j = w * 32 + d * 4;  // first byte of these 4
                        const int left = len - j;      // bytes of the row from j on
                        uint32_t x = 0;
                        if (staged) {
                            x = __builtin_amdgcn_alignbit(t9[d + 1], t9[d], sh);
                        } else if (left > 0) {
                            for (int t = 0; t < 4; ++t)
                                if (j + t < len) x |= (uint32_t)values[st + j + t] << (8 * t);
                        }
                        const uint32_t inmask = left >= 4 ? 0xFFFFFFFFu : left <= 0 ? 0u : (1u << (8 * left)) - 1u;
                        x = (x & inmask) | (0x41414141u & ~inmask);  // past the end: 'A' (code 0, valid)
                        uint32_t nb;
                        by[d] = pack4(x, nb);
                        bad |= nb;
                    }
                    // the 8 bytes into the word as a tree (not a chain of 64-bit shifts)
                    const uint32_t hi = (((by[0] << 8) | by[1]) << 16) | ((by[2] << 8) | by[3]);
                    const uint32_t lo = (((by[4] << 8) | by[5]) << 16) | ((by[6] << 8) | by[7]);
                    acc = ((uint64_t)hi << 32) | lo;
                }
                if constexpr (B == 8) {
                    switch (w) {  // static register indices in a rolled loop (w is uniform)
                        case 0: wd[0] = acc; break;
                        case 1: wd[1] = acc; break;
                        case 2: wd[2] = acc; break;
                        case 3: wd[3] = acc; break;
                        case 4: wd[4] = acc; break;
                        case 5: wd[5] = acc; break;
                        default: wd[6] = acc; break;
                    }
                }
                if (w == 0) {
                    w1 = acc;
                } else if (w & 1) {  // block word w + 1 is even: it starts a pair
                    pend = acc;
                } else {
                    *reinterpret_cast<ulonglong2*>(ob + w) = make_ulonglong2(pend, acc);
                }
            }
            // bit 33: the repeat certificate (B = 8 only: rows of at most 224 bases)
            bool norep = false;
            if constexpr (B == 8) norep = valid && bad == 0 && !may_repeat16(wd, len, lmax);
            const uint64_t meta = valid ? ((uint64_t)(uint32_t)len | ((uint64_t)(bad == 0) << 32) |
                                           ((uint64_t)norep << 33))
                                        : 0xFFFFFFFFull;
            *reinterpret_cast<ulonglong2*>(ob) = make_ulonglong2(meta, w1);
        }
        __syncthreads();
        cur = nxt;
        nxt = nn;
    }
    if (max_len && tid == 0 && run_max > 0) atomicMax(max_len, (unsigned long long)run_max);
}

// One wave per 64 grouped rows: each row's block (B words: B lanes, 64 / B rows per
// wave-instruction, all of the trip's loads in flight before any is used), then its
// bases to the grouped staging buffer at a fixed stride S = words per row (row r at
// packed[r * S]), row lengths / observation counts for this call's effective k, and
// n_sequences as one atomic per run of same-group rows (as k_row_stage).
template <int B>
__global__ __launch_bounds__(kBlock) void k_row_gather(const uint64_t* __restrict__ blocks,
                                                       const int64_t* __restrict__ rows, int64_t n_rows, int K,
                                                       int S, const uint8_t* __restrict__ gk,
                                                       const uint32_t* __restrict__ row_group,
                                                       uint64_t* __restrict__ packed, int64_t* __restrict__ row_obs,
                                                       int32_t* __restrict__ row_len,
                                                       unsigned long long* __restrict__ gstat,
                                                       unsigned long long* __restrict__ long_rows) {
    constexpr int RPI = 64 / B;  // rows per wave-instruction
    const int lane = threadIdx.x & 63, w = lane & (B - 1), sub = lane / B;
    const int64_t waves = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t rb = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 64; rb < n_rows;
         rb += waves * 64) {
        const int64_t r = rb + lane;
        const bool live = r < n_rows;
        const int64_t my_pr = live ? (rows ? rows[r] : r) : 0;
        const uint32_t my_g = live ? row_group[r] : 0u;
        const bool my_k = live && gk[my_g] == K;
        uint64_t v[B];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const int q = j * RPI + sub;
            const int64_t pr = __shfl(my_pr, q);
            v[j] = rb + q < n_rows ? blocks[pr * B + w] : 0xFFFFFFFFull;
        }
        uint64_t okbits = 0, unc = 0;
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const int q = j * RPI + sub;
            const int64_t rr = rb + q;
            const uint64_t meta = __shfl(v[j], lane & ~(B - 1));
            const uint32_t len = (uint32_t)meta;
            const bool inK = __shfl(my_k, q) && rr < n_rows && len != 0xFFFFFFFFu;
            const bool ok = inK && ((meta >> 32) & 1ull);
            const bool use = ok && (int64_t)len >= K;
            if (rr < n_rows && w >= 1 && w <= S) packed[rr * S + (w - 1)] = v[j];
            if (rr < n_rows && w == 0) {
                // a row longer than S words (a max_len below the real lengths, or past the
                // block) would read the next row's bases: counted, and the call fails
                if (inK && (int64_t)len > 32 * (int64_t)S) atomicAdd(long_rows, 1ull);
                row_obs[rr] = use ? (int64_t)len - K + 1 : 0;
                row_len[rr] = use ? (int32_t)len : 0;
            }
            const uint64_t m = __ballot(w == 0 && ok);
            // rows with observations but without the repeat certificate (meta bit 33)
            const uint64_t m2 = __ballot(w == 0 && use && !((meta >> 33) & 1ull));
#pragma unroll
            for (int t = 0; t < RPI; ++t) {
                okbits |= ((m >> (t * B)) & 1ull) << (j * RPI + t);
                unc |= ((m2 >> (t * B)) & 1ull) << (j * RPI + t);
            }
        }
        if (live) {  // n_sequences: the first lane of each run of same-group rows adds the run's ok rows
            const uint32_t g_prev = __shfl_up(my_g, 1);
            const uint64_t heads = __ballot(lane == 0 || my_g != g_prev);
            if ((heads >> lane) & 1ull) {
                const uint64_t above = lane == 63 ? 0ull : heads & (~0ull << (lane + 1));
                const uint64_t run = (above ? (above & (0ull - above)) - 1ull : ~0ull) & (~0ull << lane);
                const int cnt = __popcll(okbits & run);
                if (cnt) atomicAdd(gstat + 5 * (int64_t)my_g + 1, (unsigned long long)cnt);
                const int ucnt = __popcll(unc & run);  // gstat[5 g + 2]: read by k_group_classify only
                if (ucnt) atomicAdd(gstat + 5 * (int64_t)my_g + 2, (unsigned long long)ucnt);
            }
        }
    }
}

// Round 5: grouped rows packed straight from their ASCII bytes (no block column): the
// per-row packing and repeat certificate of k_pack_reads fused with k_row_gather's staging,
// for calls whose rows fit NW words (NW = 5: <= 160 bases, 7: <= 224; the caller knows a
// bound). A wave per 64 consecutive grouped rows, one workgroup per wave: each row's bytes
// come by ONE coalesced load instruction of the wave (lane l takes the row's dword l; 16
// rows' loads in flight before their LDS stores), staged in LDS at a fixed slot per row;
// then each lane packs and certifies its own row from its slot, as k_pack_reads does from
// its trip's bytes (a lane loading its own row's bytes took 19 ms for 100M rows, every
// load instruction touching 64 rows' lines). Outputs as k_row_gather: the row's S words at
// packed[r * S], its length / observation count, and per group the ok rows and the
// uncertified rows with observations (gstat[5 g + 1], [5 g + 2]). Saves the block column's
// 64-B write and re-read per row and one kernel per call (k_pack_reads + k_row_gather).
template <int NW>
__global__ __launch_bounds__(64, 3) void k_pack_gather(const int64_t* __restrict__ offsets,
                                                      const uint8_t* __restrict__ values,
                                                      const uint8_t* __restrict__ validity, int64_t voff,
                                                      int64_t vlen,
                                                      const int64_t* __restrict__ rows, int64_t n_rows, int K, int S,
                                                      const uint8_t* __restrict__ gk,
                                                      const uint32_t* __restrict__ row_group,
                                                      uint64_t* __restrict__ packed, int64_t* __restrict__ row_obs,
                                                      int32_t* __restrict__ row_len,
                                                      unsigned long long* __restrict__ gstat,
                                                      unsigned long long* __restrict__ long_rows) {
    // dwords per row slot: the row's 16-B chunks from the aligned address below its first
    // byte (<= 32 NW + 15 bytes), which also covers the 9-dword reads below
    constexpr int kChunks = (32 * NW + 15 + 15) / 16;
    constexpr int kSlot = 4 * kChunks;
    static_assert(kSlot >= 8 * NW + 4, "slot covers the word reads");
    __shared__ uint4 stg4[64 * kChunks];
    const uint32_t* const stg = reinterpret_cast<const uint32_t*>(stg4);
    const int lane = threadIdx.x;
    const bool cert = K >= 31 && K <= 32;  // k_group_classify reads the certificate only there
    // Software pipeline over the wave's trips: during trip t the loads of trip t + 1's
    // offsets, validity byte and group k (their row index and group came a trip earlier)
    // and of trip t + 2's row index and group are in flight, so a trip waits for its row
    // bytes only (round 5: three dependent round trips per trip before)
    const int64_t rstride = (int64_t)gridDim.x * 64;
    auto l1 = [&](int64_t r, int64_t& pr, uint32_t& g) {
        pr = 0;
        g = 0;
        if (r < n_rows) {
            pr = rows ? rows[r] : r;
            g = row_group[r];
        }
    };
    auto l2 = [&](int64_t r, int64_t pr, uint32_t g, int64_t& o0, int64_t& o1, uint32_t& vb, uint32_t& gv) {
        o0 = o1 = 0;
        vb = 1;
        gv = 0xFFFFFFFFu;
        if (r < n_rows) {
            o0 = offsets[pr];
            o1 = offsets[pr + 1];
            if (validity) {
                const int64_t bit = voff + pr;
                vb = (uint32_t)(validity[bit >> 3] >> (bit & 7));
            }
            gv = gk[g];
        }
    };
    int64_t c_pr, n_pr, c_o0, c_o1;
    uint32_t c_g, n_g, c_vb, c_gv;
    {
        const int64_t r = (int64_t)blockIdx.x * 64 + lane;
        l1(r, c_pr, c_g);
        l1(r + rstride, n_pr, n_g);
        l2(r, c_pr, c_g, c_o0, c_o1, c_vb, c_gv);
    }
    for (int64_t rb = (int64_t)blockIdx.x * 64; rb < n_rows; rb += rstride) {
        const int64_t r = rb + lane;
        const bool live = r < n_rows;
        const uint32_t my_g = c_g;
        const bool valid = live && (c_vb & 1u);
        const bool inK = valid && c_gv == (uint32_t)K;
        const int64_t st = live ? c_o0 : 0;
        const int len = live ? (int)min<int64_t>(c_o1 - c_o0, 1 << 30) : 0;
        // trip t + 1's second level, trip t + 2's first (consumed a trip later)
        c_pr = n_pr;
        c_g = n_g;
        l2(r + rstride, c_pr, c_g, c_o0, c_o1, c_vb, c_gv);
        l1(r + 2 * rstride, n_pr, n_g);
        const int clen = min(len, 32 * NW);
        const int64_t a16 = st & ~15ll;
        const int rel = (int)(st & 15);
        const int nch = inK ? (rel + clen + 15) >> 4 : 0;  // 16-B chunks of the row's slot to load
        // the rows' chunks into their slots: 16 lanes per row, 4 rows per load instruction,
        // all 64 rows' loads in flight before their LDS stores (a row whose chunks end within
        // 16 B of the buffer's end takes the byte-wise path after them)
        const int sub = lane >> 4, c = lane & 15;
        uint4 v[16];
        bool tail[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int row = 4 * u + sub;
            const int64_t ar = __shfl(a16, row);
            const int nr = __shfl(nch, row);
            const int64_t at = ar + 16 * c;
            v[u] = make_uint4(0, 0, 0, 0);
            tail[u] = c < nr && at + 16 > vlen;
            if (c < nr && !tail[u]) v[u] = *reinterpret_cast<const uint4*>(values + at);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            if (__builtin_amdgcn_ballot_w64(tail[u])) {  // wave-uniform: the shuffle needs every lane
                const int64_t at = __shfl(a16, 4 * u + sub) + 16 * c;
                if (tail[u]) {  // the buffer's last bytes: none read past values_len
                    uint32_t t4[4] = {0, 0, 0, 0};
                    for (int b = 0; b < 16; ++b)
                        if (at + b < vlen) t4[b >> 2] |= (uint32_t)values[at + b] << (8 * (b & 3));
                    v[u] = make_uint4(t4[0], t4[1], t4[2], t4[3]);
                }
            }
            if (c < kChunks) stg4[(4 * u + sub) * kChunks + c] = v[u];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        int my_len = inK ? clen : 0;  // the certificate's loop bound (wave-uniform)
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) my_len = max(my_len, __shfl_xor(my_len, m, 64));
        const int lmax = __builtin_amdgcn_readfirstlane(my_len);
        const int used = inK ? (clen + 31) >> 5 : 0;
        const uint32_t sh = (uint32_t)(rel & 3) * 8;
        const uint32_t* const slot = stg + lane * kSlot + (rel >> 2);
        uint64_t wd[NW];
        uint32_t bad = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            uint64_t acc = 0;
            if (w < used) {
                uint32_t t9[9];
#pragma unroll
                for (int i = 0; i < 9; ++i) t9[i] = slot[8 * w + i];  // past the row: masked below
                uint32_t by[8];
#pragma unroll
                for (int d = 0; d < 8; ++d) {
                    const int j = w * 32 + d * 4;  // first byte of these 4
                    const int left = len - j;
                    uint32_t x = __builtin_amdgcn_alignbit(t9[d + 1], t9[d], sh);
                    const uint32_t inmask = left >= 4 ? 0xFFFFFFFFu : left <= 0 ? 0u : (1u << (8 * left)) - 1u;
                    x = (x & inmask) | (0x41414141u & ~inmask);  // past the end: 'A' (code 0, valid)
                    uint32_t nb;
                    by[d] = pack4(x, nb);
                    bad |= nb;
                }
                const uint32_t hi = (((by[0] << 8) | by[1]) << 16) | ((by[2] << 8) | by[3]);
                const uint32_t lo = (((by[4] << 8) | by[5]) << 16) | ((by[6] << 8) | by[7]);
                acc = ((uint64_t)hi << 32) | lo;
            }
            wd[w] = acc;
        }
        const bool ok = inK && bad == 0 && len <= 32 * NW;
        const bool use = ok && len >= K;
        const bool norep = cert && use && !may_repeat16(wd, len, lmax);
        if (live) {
#pragma unroll
            for (int w = 0; w < NW; ++w)
                if (w < S) packed[r * S + w] = wd[w];
            // a row longer than S words would read the next row's bases: counted, the call fails
            if (inK && len > 32 * S) atomicAdd(long_rows, 1ull);
            row_obs[r] = use ? (int64_t)len - K + 1 : 0;
            row_len[r] = use ? (int32_t)len : 0;
        }
        const uint64_t okbits = __ballot(ok), unc = __ballot(use && !norep);
        if (live) {  // n_sequences: the first lane of each run of same-group rows adds the run's ok rows
            const uint32_t g_prev = __shfl_up(my_g, 1);
            const uint64_t heads = __ballot(lane == 0 || my_g != g_prev);
            if ((heads >> lane) & 1ull) {
                const uint64_t above = lane == 63 ? 0ull : heads & (~0ull << (lane + 1));
                const uint64_t run = (above ? (above & (0ull - above)) - 1ull : ~0ull) & (~0ull << lane);
                const int cnt = __popcll(okbits & run);
                if (cnt) atomicAdd(gstat + 5 * (int64_t)my_g + 1, (unsigned long long)cnt);
                const int ucnt = __popcll(unc & run);
                if (ucnt) atomicAdd(gstat + 5 * (int64_t)my_g + 2, (unsigned long long)ucnt);
            }
        }
        __builtin_amdgcn_s_barrier();  // the slots are rewritten by the next trip
    }
}

// the longest row of a column (rogtk_kmer_spectrum_fused without a bound): one atomic per wave
__global__ __launch_bounds__(kBlock) void k_max_row_len(const int64_t* __restrict__ offsets, int64_t n,
                                                        unsigned long long* __restrict__ out) {
    int64_t m = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        m = max(m, offsets[i + 1] - offsets[i]);
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) m = max(m, (int64_t)__shfl_xor(m, s, 64));
    if ((threadIdx.x & 63) == 0 && m > 0) atomicMax(out, (unsigned long long)m);
}

// row -> group map: one wave per group writes its rows' group id (coalesced)
// 16 lanes per group (no shuffles: segments run independently)
__global__ __launch_bounds__(kBlock) void k_row_groups(const int64_t* __restrict__ go, int64_t G,
                                                       uint32_t* __restrict__ row_group) {
    const int sub = threadIdx.x & 15;
    const int64_t step = (int64_t)gridDim.x * (kBlock / 16);
    for (int64_t g = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / 16; g < G; g += step)
        for (int64_t r = go[g] + sub; r < go[g + 1]; r += 16) row_group[r] = (uint32_t)g;
}

template <int OW, bool WIDE>
__global__ __launch_bounds__(kBlock) void k_kmer_emit(const void* offsets, const uint8_t* __restrict__ values,
                                                      const int64_t* __restrict__ rows, int64_t n_rows, int K, const uint32_t* __restrict__ row_group,
                                                      const int64_t* __restrict__ row_obs,
                                                      const int64_t* __restrict__ obs_off,
                                                      uint64_t* __restrict__ key_lo, uint64_t* __restrict__ key_hi,
                                                      uint8_t* __restrict__ ext, uint32_t* __restrict__ grp,
                                                      uint32_t* __restrict__ idx) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); r < n_rows; r += waves) {
        const int64_t nobs = row_obs[r];
        if (nobs == 0) continue;
        int64_t st, len;
        span<OW>(offsets, rows ? rows[r] : r, st, len);
        const uint8_t* s = values + st;
        const int64_t o0 = obs_off[r];
        const uint32_t g = row_group[r];
        for (int64_t p = lane; p < nobs; p += 64) {
            uint64_t lo = 0, hi = 0;
            if (WIDE) {
                for (int j = 0; j < 32; ++j) hi = (hi << 2) | base2(s[p + j]);
                for (int j = 32; j < 64; ++j) lo = (lo << 2) | base2(s[p + j]);
            } else {
                for (int j = 0; j < K; ++j) lo = (lo << 2) | base2(s[p + j]);
            }
            uint8_t e = 0;
            if (p > 0) e |= (uint8_t)(1u << base2(s[p - 1]));
            if (p + K < len) e |= (uint8_t)(1u << (4 + base2(s[p + K])));
            const int64_t o = o0 + p;
            key_lo[o] = lo;
            if (WIDE) key_hi[o] = hi;
            ext[o] = e;
            grp[o] = g;
            idx[o] = (uint32_t)o;
        }
    }
}

template <class T>
__global__ __launch_bounds__(kBlock) void k_gather(const T* __restrict__ src, const uint32_t* __restrict__ perm,
                                                   int64_t n, T* __restrict__ dst) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        dst[i] = src[perm[i]];
}

template <bool WIDE>
__device__ __forceinline__ bool same_key(const uint64_t* lo, const uint64_t* hi, const uint32_t* grp, int64_t a,
                                         int64_t b) {
    return grp[a] == grp[b] && lo[a] == lo[b] && (!WIDE || hi[a] == hi[b]);
}

template <bool WIDE>
__global__ __launch_bounds__(kBlock) void k_heads(const uint64_t* __restrict__ lo, const uint64_t* __restrict__ hi,
                                                  const uint32_t* __restrict__ grp, int64_t n,
                                                  uint32_t* __restrict__ head) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        head[i] = (i == 0 || !same_key<WIDE>(lo, hi, grp, i, i - 1)) ? 1u : 0u;
}

// One lane per run head: count (u16 saturating), OR of exts, CountFilter.
template <bool WIDE>
__global__ __launch_bounds__(kBlock) void k_runs(const uint64_t* __restrict__ lo, const uint64_t* __restrict__ hi,
                                                 const uint32_t* __restrict__ grp, const uint8_t* __restrict__ ext,
                                                 const uint32_t* __restrict__ head, const uint32_t* __restrict__ rid,
                                                 int64_t n, int64_t min_cov, uint32_t* __restrict__ r_valid,
                                                 uint32_t* __restrict__ r_first, uint8_t* __restrict__ r_ext,
                                                 uint16_t* __restrict__ r_cnt) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        if (!head[i]) continue;
        uint32_t count = 0;
        uint8_t e = 0;
        int64_t j = i;
        do {
            if (count < 0xFFFFu) ++count;
            e |= ext[j];
            ++j;
        } while (j < n && !head[j]);
        const uint32_t r = rid[i];
        r_valid[r] = (int64_t)count >= min_cov ? 1u : 0u;
        r_first[r] = (uint32_t)i;
        r_ext[r] = e;
        r_cnt[r] = (uint16_t)count;
    }
}

template <bool WIDE>
__global__ __launch_bounds__(kBlock) void k_compact_valid(const uint32_t* __restrict__ r_valid,
                                                          const uint32_t* __restrict__ vpos,
                                                          const uint32_t* __restrict__ r_first,
                                                          const uint8_t* __restrict__ r_ext,
                                                          const uint16_t* __restrict__ r_cnt, int64_t n_runs,
                                                          const uint64_t* __restrict__ lo,
                                                          const uint64_t* __restrict__ hi,
                                                          const uint32_t* __restrict__ grp,
                                                          uint64_t* __restrict__ v_lo, uint64_t* __restrict__ v_hi,
                                                          uint32_t* __restrict__ v_grp, uint8_t* __restrict__ v_ext,
                                                          uint16_t* __restrict__ v_cnt) {
    for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < n_runs; r += (int64_t)gridDim.x * kBlock) {
        if (!r_valid[r]) continue;
        const uint32_t j = vpos[r], f = r_first[r];
        v_lo[j] = lo[f];
        if (WIDE) v_hi[j] = hi[f];
        v_grp[j] = grp[f];
        v_ext[j] = r_ext[r];
        v_cnt[j] = r_cnt[r];
    }
}

__global__ __launch_bounds__(kBlock) void k_group_ranges(const uint32_t* __restrict__ v_grp, int64_t nv,
                                                         int64_t* __restrict__ gstart, int64_t* __restrict__ gcount) {
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < nv; j += (int64_t)gridDim.x * kBlock) {
        const uint32_t g = v_grp[j];
        if (j == 0 || v_grp[j - 1] != g) gstart[g] = j;
        if (j == nv - 1 || v_grp[j + 1] != g) gcount[g] = j + 1;  // end; made a count below
    }
}

__global__ __launch_bounds__(kBlock) void k_group_counts(const uint8_t* __restrict__ gk, int K, int64_t G,
                                                         const uint8_t* __restrict__ gsmall,
                                                         const int64_t* __restrict__ gstart,
                                                         int64_t* __restrict__ gcount) {
    for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < G; g += (int64_t)gridDim.x * kBlock)
        if (gk[g] == K && !(gsmall && gsmall[g]) && gcount[g] > 0) gcount[g] -= gstart[g];
}

// remove_censored_exts + terminal / isolated counts + output at the group's capacity offset
template <bool WIDE>
__global__ __launch_bounds__(kBlock) void k_censor(const uint64_t* __restrict__ v_lo, const uint64_t* __restrict__ v_hi,
                                                   const uint32_t* __restrict__ v_grp,
                                                   const uint8_t* __restrict__ v_ext,
                                                   const uint16_t* __restrict__ v_cnt, int64_t nv, int K,
                                                   const int64_t* __restrict__ gstart,
                                                   const int64_t* __restrict__ gcount,
                                                   const int64_t* __restrict__ cap_off,
                                                   uint64_t* __restrict__ o_kmer, uint8_t* __restrict__ o_ext,
                                                   uint16_t* __restrict__ o_cnt,
                                                   unsigned long long* __restrict__ gstat, int lo_only) {
    const uint64_t mask = (WIDE || K == 32) ? ~0ull : ((1ull << (2 * K)) - 1ull);
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < nv; j += (int64_t)gridDim.x * kBlock) {
        const uint32_t g = v_grp[j];
        const int64_t a0 = gstart[g], b0 = a0 + gcount[g];
        const uint64_t lo = v_lo[j], hi = WIDE ? v_hi[j] : 0ull;
        const uint8_t e = v_ext[j];
        uint8_t ne = 0;
        for (int bit = 0; bit < 8; ++bit) {
            if (!((e >> bit) & 1u)) continue;
            const uint64_t b = (uint64_t)(bit & 3);
            uint64_t nlo, nhi = 0;
            if (bit < 4) {  // extend_left: b + kmer[0..K-1]
                if (WIDE) {
                    nlo = (lo >> 2) | ((hi & 3ull) << 62);
                    nhi = (hi >> 2) | (b << 62);
                } else {
                    nlo = (lo >> 2) | (b << (2 * K - 2));
                }
            } else {  // extend_right: kmer[1..K] + b
                if (WIDE) {
                    nhi = (hi << 2) | (lo >> 62);
                    nlo = (lo << 2) | b;
                } else {
                    nlo = ((lo << 2) | b) & mask;
                }
            }
            int64_t a = a0, c = b0;
            while (a < c) {
                const int64_t m = (a + c) >> 1;
                const bool less = WIDE ? (v_hi[m] < nhi || (v_hi[m] == nhi && v_lo[m] < nlo)) : v_lo[m] < nlo;
                if (less) a = m + 1;
                else c = m;
            }
            const bool found = a < b0 && v_lo[a] == nlo && (!WIDE || v_hi[a] == nhi);
            if (found) ne |= (uint8_t)(1u << bit);
        }
        const int64_t o = cap_off[g] + (j - a0);
        if (lo_only) {
            o_kmer[o] = lo;
        } else {
            o_kmer[2 * o] = hi;
            o_kmer[2 * o + 1] = lo;
        }
        o_ext[o] = ne;
        o_cnt[o] = v_cnt[j];
        const bool l0 = (ne & 0xF) == 0, r0 = (ne >> 4) == 0;
        if (l0 || r0) atomicAdd(gstat + 5 * g + 3, 1ull);
        if (l0 && r0) atomicAdd(gstat + 5 * g + 4, 1ull);
    }
}

// dense packing: one wave per group copies its entries to the final offsets, up to 256
// entries per trip with all their loads issued before the first store (a C3 group at k_eff
// 16 has ~157 valid k-mers: one trip instead of three dependent ones); V16: the k-mer pairs
// as one 16-B access (both arrays 16-B aligned); LO: the staged k-mers are one word each
// (k_eff <= 32), the high word written as 0 here
template <bool V16, bool LO>
__global__ __launch_bounds__(kBlock) void k_pack(const uint64_t* __restrict__ t_kmer, const uint8_t* __restrict__ t_ext,
                                                 const uint16_t* __restrict__ t_cnt, int64_t G,
                                                 const int64_t* __restrict__ cap_off,
                                                 const int64_t* __restrict__ gcount,
                                                 const int64_t* __restrict__ out_off, uint64_t* __restrict__ kmer,
                                                 uint8_t* __restrict__ ext, uint16_t* __restrict__ cnt) {
    constexpr int kU = 4;
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t g = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); g < G; g += waves) {
        const int64_t n = gcount[g], s = cap_off[g], d = out_off[g];
        for (int64_t t0 = 0; t0 < n; t0 += 64 * kU) {
            uint64_t k0[kU], k1[kU];
            uint8_t e[kU];
            uint16_t c[kU];
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const int64_t t = t0 + lane + 64 * j;
                if (t < n) {
                    if constexpr (LO) {
                        k0[j] = 0ull;
                        k1[j] = t_kmer[s + t];
                    } else if constexpr (V16) {
                        const ulonglong2 v = reinterpret_cast<const ulonglong2*>(t_kmer)[s + t];
                        k0[j] = v.x;
                        k1[j] = v.y;
                    } else {
                        k0[j] = t_kmer[2 * (s + t)];
                        k1[j] = t_kmer[2 * (s + t) + 1];
                    }
                    e[j] = t_ext[s + t];
                    c[j] = t_cnt[s + t];
                }
            }
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const int64_t t = t0 + lane + 64 * j;
                if (t < n) {
                    if constexpr (V16) {
                        reinterpret_cast<ulonglong2*>(kmer)[d + t] = make_ulonglong2(k0[j], k1[j]);
                    } else {
                        kmer[2 * (d + t)] = k0[j];
                        kmer[2 * (d + t) + 1] = k1[j];
                    }
                    ext[d + t] = e[j];
                    cnt[d + t] = c[j];
                }
            }
        }
    }
}

// ----------------------------------------------------------- LDS fast path
// One workgroup per small group (size class CLS: rows and packed words, and for class
// 3 observations, within LdsCfg<CLS>; k_eff <= 32): the group's rows, already packed
// to 2-bit words in HBM by k_row_stage, are loaded into LDS in one pass; every observation is
// inserted into an LDS hash table (64-bit CAS on the key; the count and the OR of
// exts share one u32: count in bits 0..23, exts in 24..31), the valid entries are
// compacted, bitonic-sorted and censored by binary search, all in LDS. The all-ones
// key (TTT..T at k = 32) equals the empty marker and gets a dedicated slot.
constexpr int kLdsBlock = 512;  // 8 waves per group workgroup (16 per CU for class 1; 1024 measured slower)
constexpr bool kRankSort = true;  // 65..512 valid entries by a rank sort (round 5; bitonic above)

// Size classes, tried in the order 3, 1, 4; larger groups take the global radix-sort
// path. Class 3 (<= 192 rows, <= 576 words, a 2048-slot table for up to 1472 distinct
// and 1024 valid k-mers, ~37 KB and at most 64 VGPRs: 4 workgroups per CU) takes the
// typical C3 group (~10 reads of 119 k-mers); past either bound a group moves on to
// class 1. Class 1 (<= 256 rows, <= 768 packed words, any number of observations): a 4096-slot
// table takes up to 2048 distinct k-mers (~78 KB, 2 workgroups per CU). Class 4 (round
// 2; <= 512 rows, <= 4096 words): an 8192-slot table for up to 6144 distinct and 2048
// valid k-mers (~150 KB, 1 workgroup per CU). A class-1 group past its claim cap goes
// on to class 4 (whose instance runs last), a class-4 group past either bound to the
// global path: its class is rewritten before k_drop_small_rows, which then keeps its
// rows, so the outputs never depend on where a group ends up.
template <int CLS>
struct LdsCfg {
    static_assert(CLS == 1 || CLS == 3 || CLS == 4, "LDS size classes 3, 1, 4");
    // valid k-mers (the sort buffer; a power of two: the bitonic sort pads to one)
    static constexpr int kObs = CLS == 3 ? 1024 : 2048;
    static_assert((kObs & (kObs - 1)) == 0, "sort buffer: a power of two");
    static constexpr int kSlots = CLS == 3 ? 2048 : CLS == 4 ? 8192 : 2 * kObs;  // power of two
    // distinct k-mers (claimed slots): at most TB more can be claimed by the inserts in
    // flight when the cap is passed, and the table keeps an empty slot after those
    static constexpr int kClaim = CLS == 4 ? 6144 : CLS == 3 ? 1472 : kObs;
    static constexpr int kRows = CLS == 3 ? 192 : CLS == 1 ? 256 : 512;    // rows of one group
    static constexpr int kWords = CLS == 3 ? 576 : CLS == 1 ? 768 : 4096;  // packed words
    // insert phase (packed words + row metadata) and sort phase (valid entries) share LDS
    static constexpr int kInsertWords = kWords + 1 + (kRows * 12 + 7) / 8;
    static constexpr int kUnionWords = (kObs * 12 + 7) / 8 > kInsertWords ? (kObs * 12 + 7) / 8 : kInsertWords;
    static_assert(kSlots - kClaim > 512, "one in-flight insert per thread past the claim cap");
};
constexpr unsigned long long kEmpty = ~0ull;

// ROGTK_KMER_CERT=0: no group skips the LDS kernels by the repeat certificate (A/B; read once)
inline bool kmer_cert_on() {
    static const bool on = [] {
        const char* e = getenv("ROGTK_KMER_CERT");
        return !(e && e[0] == '0');
    }();
    return on;
}

#ifdef ROGTK_KMER_TIMING  // experiment builds only: per-phase clocks of k_kmer_lds (thread 0)
__device__ unsigned long long g_kmer_clk[8];
#define KT(k) do { if (tid == 0) { const unsigned long long now_ = wall_clock64(); kt_acc[k] += now_ - kt_last; kt_last = now_; } } while (0)
#else
#define KT(k) do { } while (0)
#endif

__device__ __forceinline__ bool kless(uint64_t ka, uint32_t ia, uint64_t kb, uint32_t ib) {
    return ka < kb || (ka == kb && (ia >> 31) < (ib >> 31));  // real entries before pads
}

// What an LDS-path group needs to start: its first grouped row, first packed word,
// row count and packed word count (written by k_group_classify).
struct GroupDesc {
    int64_t r0, w0;
    int32_t nrows, nwords;
};

// (Round 4 measured two other insert loops for class 3 - all LDS word reads of a trip behind
// one wait with a 32-bit hash: +0.3%; wave-private claimed lists: 31% slower - removed in
// round 5.)
template <int CLS, int TB>
__global__ __launch_bounds__(TB, CLS == 3 ? 8 : 1) void k_kmer_lds(const GroupDesc* __restrict__ gdesc, int64_t G,
                                                     uint8_t* __restrict__ gsmall, int K, int64_t min_cov,
                                                     const int32_t* __restrict__ row_len,
                                                     const int64_t* __restrict__ woff, int stride,
                                                     const uint64_t* __restrict__ packed,
                                                     const int64_t* __restrict__ cap_off,
                                                     uint64_t* __restrict__ t_kmer, uint8_t* __restrict__ t_ext,
                                                     uint16_t* __restrict__ t_cnt, int64_t* __restrict__ gcount,
                                                     unsigned long long* __restrict__ gstat, int lo_only) {
    using C = LdsCfg<CLS>;
    constexpr int kWaves = TB / 64;
    // every class takes groups of any observation count: their distinct k-mers are
    // bounded by the claim cap (and class 4's valid ones by its sort buffer) instead
    constexpr bool kBounded = true;
    constexpr int kLdsObs = C::kObs, kLdsSlots = C::kSlots, kLdsRows = C::kRows, kLdsWords = C::kWords;
    __shared__ unsigned long long tkey[kLdsSlots + 1];
    __shared__ uint32_t tinfo[kLdsSlots + 1];  // count (bits 0..23) | exts << 24
    __shared__ uint16_t claimed[C::kClaim + 1];  // slots first touched by this group
    __shared__ __attribute__((aligned(16))) uint64_t ubuf[C::kUnionWords];
    uint64_t* const words = ubuf;                                      // the group's packed rows
    int32_t* const m_len = reinterpret_cast<int32_t*>(ubuf + kLdsWords + 1);
    int32_t* const m_nobs = m_len + kLdsRows;
    int32_t* const m_w = m_nobs + kLdsRows;
    uint64_t* const vkey = ubuf;                                       // after the inserts
    uint32_t* const vinfo = reinterpret_cast<uint32_t*>(ubuf + kLdsObs);  // count | exts << 16 | pad << 31
    __shared__ uint32_t s_claimed, s_term, s_iso, s_over, s_hit, s_nv;
    // s_hit: some k-mer's count reached min_cov during the inserts (counts grow by one per
    // insert, so one insert sees exactly min_cov). Without it nothing is valid and the
    // CountFilter pass, its scan and a barrier are skipped (most groups at the usual floor)
    const uint32_t hit_at = min_cov <= 1 ? 1u : min_cov <= 0xFFFF ? (uint32_t)min_cov : 0u;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hbits = 31 - __clz(kLdsSlots);
    const uint64_t kmask = K == 32 ? ~0ull : ((1ull << (2 * K)) - 1ull);
    for (int i = tid; i <= kLdsSlots; i += TB) {  // once; groups reset only what they touch
        tkey[i] = kEmpty;
        tinfo[i] = 0;
    }
    if (tid == 0) {
        s_claimed = 0;
        s_over = 0;
    }
#ifdef ROGTK_KMER_TIMING
    unsigned long long kt_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, kt_last = wall_clock64();
#endif
    // Groups are taken in chunks of 64 consecutive ids: one coalesced load of their
    // classes and a ballot give this class's groups of the chunk, so the instances of
    // the rarer classes skip 64 groups per load. Within a chunk, the next group's rows (lengths, word offsets, packed words) are
    // loaded into registers while the current group is processed, and the descriptor
    // of the group after it as well, so a group's HBM round trips overlap the previous
    // group's work; only a chunk's first group waits for its rows.
    constexpr int kWPT = (kLdsWords + TB - 1) / TB;  // packed words per thread
    static_assert(kLdsRows <= TB, "one row per thread");
    int32_t p_len = 0, p_w = 0;
    uint64_t p_words[kWPT];
    auto load_rows = [&](const GroupDesc& dd) {
        if (tid < dd.nrows) {
            p_len = row_len[dd.r0 + tid];
            p_w = stride ? tid * stride : (int32_t)(woff[dd.r0 + tid] - dd.w0);
        }
#pragma unroll
        for (int j = 0; j < kWPT; ++j) {
            const int i = tid + j * TB;
            p_words[j] = i < dd.nwords ? packed[dd.w0 + i] : 0;
        }
    };
    const int64_t n_chunks = (G + 63) >> 6;
    for (int64_t ch = blockIdx.x; ch < n_chunks; ch += gridDim.x) {
    const int64_t g0 = ch << 6;
    uint64_t own = __ballot(g0 + lane < G && gsmall[g0 + lane] == CLS);
    if (!own) continue;
    int i0 = __ffsll((unsigned long long)own) - 1;
    own &= own - 1;
    GroupDesc d = gdesc[g0 + i0];
    GroupDesc d1 = own ? gdesc[g0 + __ffsll((unsigned long long)own) - 1] : GroupDesc{0, 0, 0, 0};
    GroupDesc d2{0, 0, 0, 0};
    load_rows(d);
    bool more = true;
    int i1 = -1;
    uint64_t own2 = 0;
    auto advance = [&]() {
        if (i1 < 0) return false;
        i0 = i1;
        own = own2;
        d = d1;
        d1 = d2;
        return true;
    };
    for (; more; more = advance()) {
        const int64_t g = g0 + i0;
        KT(0);
        const int nrows = d.nrows, nwords = d.nwords;  // within LdsCfg<CLS> (classification)
        if (tid < nrows) {
            m_len[tid] = p_len;
            m_nobs[tid] = p_len ? p_len - K + 1 : 0;
            m_w[tid] = p_w;
        }
#pragma unroll
        for (int j = 0; j < kWPT; ++j) {
            const int i = tid + j * TB;
            if (i < nwords) words[i] = p_words[j];
        }
        if (tid == 0) {
            words[nwords] = 0;
            s_term = 0;
            s_hit = 0;
            s_iso = 0;
        }
        __syncthreads();
        i1 = own ? __ffsll((unsigned long long)own) - 1 : -1;
        own2 = own & (own - 1);
        if (i1 >= 0) load_rows(d1);  // in flight while this group is processed
        if (own2) d2 = gdesc[g0 + __ffsll((unsigned long long)own2) - 1];
        KT(1);
        // every k-mer observation of the group, straight from the packed words in LDS.
        // Work unit = (row, half): half h takes the row's positions 64 h + lane + 128 i, so
        // a C3 group (~10 rows of 119 observations) deals 2 units per row over the 8 waves
        // instead of whole rows (waves with two rows set the pace otherwise)
        {
            for (int u = wave; u < 2 * nrows; u += kWaves) {
                const int ri = u >> 1;
                const int nobs = m_nobs[ri];
                if (nobs <= ((u & 1) << 6)) continue;
                const int len = m_len[ri];
                const uint64_t* rw = words + m_w[ri];
                for (int p = lane + ((u & 1) << 6); p < nobs; p += 128) {
                    const int b = 2 * (p & 31);
                    const uint64_t x0 = rw[p >> 5], x1 = rw[(p >> 5) + 1];
                    const uint64_t top = b ? (x0 << b) | (x1 >> (64 - b)) : x0;
                    const uint64_t key = (top >> (64 - 2 * K)) & kmask;
                    // extension bases from the two words already loaded (k_eff <= 32: base p + K
                    // lies in x0 or x1); only a k-mer starting a word loads its left base
                    uint32_t e = 0;
                    if (p > 0) e |= 1u << (b ? (uint32_t)(x0 >> (64 - b)) & 3u : (uint32_t)rw[(p >> 5) - 1] & 3u);
                    if (p + K < len) {
                        const int t = (p & 31) + K;
                        e |= 1u << (4 + ((uint32_t)((t < 32 ? x0 : x1) >> (62 - 2 * (t & 31))) & 3u));
                    }
                    if (kBounded && __hip_atomic_load(&s_over, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                    uint32_t slot;
                    if (key == kEmpty) {
                        slot = kLdsSlots;
                    } else {
                        slot = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - hbits));
                        while (true) {
                            const unsigned long long prev = atomicCAS(&tkey[slot], kEmpty, (unsigned long long)key);
                            if (prev == kEmpty || prev == key) break;
                            slot = (slot + 1) & (kLdsSlots - 1);
                        }
                    }
                    const uint32_t old = atomicAdd(&tinfo[slot], 1u);
                    const uint32_t cnt0 = old & 0xFFFFFFu;
                    if (cnt0 == 0) {
                        const uint32_t ci = atomicAdd(&s_claimed, 1u);
                        if (!kBounded || ci < (uint32_t)C::kClaim) claimed[ci] = (uint16_t)slot;
                        else s_over = 1;  // more distinct k-mers than the table takes
                    }
                    if (cnt0 + 1 == hit_at) s_hit = 1;
                    // the extension bits only when one is new (the count's old value carries them)
                    if (e & ~(old >> 24)) atomicOr(&tinfo[slot], e << 24);
                }
            }
        }
        __syncthreads();
        KT(2);
        const uint32_t ncl = s_claimed;
        auto cl_at = [&](uint32_t i) -> uint32_t { return claimed[i]; };
        // reset the touched slots
        auto reset_claimed = [&]() {
            for (uint32_t i = tid; i < ncl; i += TB) {
                const uint32_t sl = claimed[i];
                tkey[sl] = kEmpty;
                tinfo[sl] = 0;
            }
        };
        const bool hit = s_hit;
        if (kBounded) {
            const bool over = s_over;
            if (tid == 0) s_nv = 0;  // every thread read the previous group's count before its first barrier
            __syncthreads();  // every thread has read the flags before they are cleared
            if (over) {
                // the claimed list is incomplete: clear the whole table; the group goes
                // to class 4 (from class 1) or the global path (the next group's first
                // barrier orders the resets)
                for (int i = tid; i <= kLdsSlots; i += TB) {
                    tkey[i] = kEmpty;
                    tinfo[i] = 0;
                }
                if (tid == 0) {
                    gsmall[g] = CLS == 3 ? 1 : CLS == 1 ? 4 : 0;
                    s_claimed = 0;
                    s_over = 0;
                }
                continue;
            }
        }
        if (!hit) {
            // no count reached min_cov: nothing passes CountFilter (as nv == 0 below,
            // without the count pass): reset the touched slots, record the empty group
            reset_claimed();
            if (tid == 0) {
                gcount[g] = 0;
                gstat[5 * g + 3] = 0;
                gstat[5 * g + 4] = 0;
                s_claimed = 0;
            }
            continue;
        }
        // CountFilter + compaction in one pass over the claimed slots (round 5: the sorts
        // below order the valid entries, so their order here is free): each wave reserves
        // its valid entries' places with one LDS atomic (round 4 counted them in a pass of
        // its own, then scanned)
        for (uint32_t i0 = 0; i0 < ncl; i0 += TB) {  // a uniform trip count (ballots)
            const uint32_t i = i0 + tid;
            uint32_t sl = 0, info = 0;
            bool v = false;
            if (i < ncl) {
                sl = cl_at(i);
                info = tinfo[sl];
                v = (int64_t)min(info & 0xFFFFFFu, 0xFFFFu) >= min_cov;
            }
            const uint64_t m = __ballot(v);
            if (!m) continue;
            const int leader = __ffsll((unsigned long long)m) - 1;
            uint32_t wb = 0;
            if (lane == leader) wb = atomicAdd(&s_nv, (uint32_t)__popcll(m));
            wb = __shfl(wb, leader);
            if (v) {
                const uint32_t w = wb + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (w < (uint32_t)kLdsObs) {
                    vkey[w] = sl == kLdsSlots ? kEmpty : tkey[sl];
                    vinfo[w] = min(info & 0xFFFFFFu, 0xFFFFu) | ((info >> 24) << 16);
                }
            }
        }
        __syncthreads();
        KT(3);
        const uint32_t nv = s_nv;
        if (nv == 0) {
            // nothing passed CountFilter: reset the touched slots and record the empty
            // group, no compaction, sort or further barrier (the next group's first
            // barrier orders these resets before its inserts)
            reset_claimed();
            if (tid == 0) {
                gcount[g] = 0;
                gstat[5 * g + 3] = 0;
                gstat[5 * g + 4] = 0;
                s_claimed = 0;
            }
            KT(5);
            continue;
        }
        if (nv > (uint32_t)kLdsObs) {
            // more valid k-mers than the sort buffer takes: the next class or the global path
            reset_claimed();
            if (tid == 0) {
                gsmall[g] = CLS == 3 ? 1 : CLS == 1 ? 4 : 0;
                s_claimed = 0;
            }
            continue;
        }
        KT(4);
        // the censoring below finds a k-mer's neighbours in the hash table itself (a probe
        // or two, round 5) instead of by binary search over the sorted valid entries (eight
        // dependent LDS reads per extension); the touched slots are reset after it
        auto valid_at = [&](uint64_t nb) -> bool {
            uint32_t sl = kLdsSlots;
            if (nb != kEmpty) {
                sl = (uint32_t)((nb * 0x9E3779B97F4A7C15ull) >> (64 - hbits));
                while (true) {
                    const unsigned long long k = tkey[sl];
                    if (k == nb) break;
                    if (k == kEmpty) return false;
                    sl = (sl + 1) & (kLdsSlots - 1);
                }
            }
            return (int64_t)min(tinfo[sl] & 0xFFFFFFu, 0xFFFFu) >= min_cov;
        };
        const int64_t base = cap_off[g];
        if (nv <= 64) {
            // small valid set: wave 0 sorts it in registers (bitonic over shuffles),
            // censors and writes it
            if (wave == 0) {
                uint64_t key = lane < (int)nv ? vkey[lane] : kEmpty;
                uint32_t info = lane < (int)nv ? vinfo[lane] : (1u << 31);
                // bitonic over the first P lanes only (P = nv rounded up to a power of
                // two): the last merge leaves lanes 0..P-1 ascending, pads last
#pragma unroll
                for (int k2 = 2; k2 <= 64; k2 <<= 1) {
                    if (k2 >= 2 * (int)nv && k2 > 2) break;
#pragma unroll
                    for (int j = k2 >> 1; j > 0; j >>= 1) {
                        const uint64_t ok = __shfl_xor(key, j);
                        const uint32_t oi = __shfl_xor(info, j);
                        const bool lower = (lane & j) == 0, up = (lane & k2) == 0;
                        const bool other_less = kless(ok, oi, key, info);
                        const bool take = (lower == up) ? other_less : !other_less && !(ok == key && oi == info);
                        if (take) {
                            key = ok;
                            info = oi;
                        }
                    }
                }
                vkey[lane] = key;  // sorted (pads last) for the neighbour searches
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                uint32_t term = 0, iso = 0;
                if (lane < (int)nv) {
                    const uint32_t e = (info >> 16) & 0xFFu;
                    uint32_t ne = 0;
                    for (int bit = 0; bit < 8; ++bit) {
                        if (!((e >> bit) & 1u)) continue;
                        const uint64_t bb = (uint64_t)(bit & 3);
                        const uint64_t nb = bit < 4 ? (key >> 2) | (bb << (2 * K - 2)) : ((key << 2) | bb) & kmask;
                        if (valid_at(nb)) ne |= 1u << bit;
                    }
                    const int64_t o = base + lane;
                    if (lo_only) {
                        t_kmer[o] = key;
                    } else {
                        t_kmer[2 * o] = 0;
                        t_kmer[2 * o + 1] = key;
                    }
                    t_ext[o] = (uint8_t)ne;
                    t_cnt[o] = (uint16_t)(info & 0xFFFFu);
                    const bool l0 = (ne & 0xFu) == 0, r0b = (ne >> 4) == 0;
                    term = (l0 || r0b) ? 1u : 0u;
                    iso = (l0 && r0b) ? 1u : 0u;
                }
                const uint64_t tb = __ballot(term), ib = __ballot(iso);
                if (lane == 0) {
                    gcount[g] = nv;
                    gstat[5 * g + 3] = (unsigned long long)__popcll(tb);
                    gstat[5 * g + 4] = (unsigned long long)__popcll(ib);
                    s_claimed = 0;
                }
            }
            __syncthreads();
            reset_claimed();  // the next group's first barrier orders these before its inserts
            KT(5);
            continue;
        }
        uint32_t P = 2;
        while (P < nv) P <<= 1;
        // rank sort: every thread keeps its own entry and writes it at its rank (the
        // censoring reads the hash table, not the sorted order), so the entries never move
        bool direct = false;
        uint64_t myk = 0;
        uint32_t myi = 0, rank = 0;
        if (nv <= (uint32_t)TB && kRankSort) {
            // 65..TB valid entries (round 5; C3 at k_eff 16, min_coverage 5: ~157 per group):
            // a rank sort instead of a bitonic network - thread i counts the keys below its
            // own (distinct: one table slot each), every wave reading the same vkey[j] at once
            // (an LDS broadcast), then writes its entry out at that rank: two barriers instead
            // of one per bitonic stage (36 at 256 entries)
            direct = true;
            if ((uint32_t)tid < nv) {
                myk = vkey[tid];
                myi = vinfo[tid];
            }
            if (K <= 16) {
                // 32-bit keys: packed densely over the front of vkey first (every u64 key read
                // above), so one 16-B broadcast read gives 4 of them; pads compare as the
                // largest key and count for nobody
                uint32_t* const vk = reinterpret_cast<uint32_t*>(vkey);
                const uint32_t n4 = (nv + 3) & ~3u;
                __syncthreads();
                if ((uint32_t)tid < n4) vk[tid] = (uint32_t)tid < nv ? (uint32_t)myk : 0xFFFFFFFFu;
                __syncthreads();
                if ((uint32_t)tid < nv) {
                    const uint32_t mk = (uint32_t)myk;
                    const uint4* const v4 = reinterpret_cast<const uint4*>(vk);
                    for (uint32_t j = 0; j < n4 / 4; ++j) {
                        const uint4 q = v4[j];
                        rank += (q.x < mk) + (q.y < mk) + (q.z < mk) + (q.w < mk);
                    }
                }
            } else if ((uint32_t)tid < nv) {
                uint32_t j = 0;
                for (; j + 4 <= nv; j += 4)
                    rank += (vkey[j] < myk) + (vkey[j + 1] < myk) + (vkey[j + 2] < myk) + (vkey[j + 3] < myk);
                for (; j < nv; ++j) rank += vkey[j] < myk;
            }
        } else if (P == 128) {
            // 65..128 valid entries (a family of min_cov or more reads, e.g. C3's uncertified
            // groups: a 150-bp template has 119 k-mers): wave 0 sorts them in registers, two
            // per lane (element lane and 64 + lane: partners j < 64 by shuffles, j = 64 inside
            // the lane), one barrier instead of one per bitonic stage (28) with 7 waves idle
            if (wave == 0) {
                uint64_t ka = vkey[lane];
                uint32_t ia = vinfo[lane];
                uint64_t kb = (uint32_t)(64 + lane) < nv ? vkey[64 + lane] : kEmpty;
                uint32_t ib = (uint32_t)(64 + lane) < nv ? vinfo[64 + lane] : (1u << 31);
                for (uint32_t k2 = 2; k2 <= 128; k2 <<= 1) {
                    for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
                        if (j == 64) {  // elements lane and 64 + lane: k2 = 128, ascending
                            if (kless(kb, ib, ka, ia)) {
                                const uint64_t tk = ka;
                                const uint32_t ti = ia;
                                ka = kb;
                                ia = ib;
                                kb = tk;
                                ib = ti;
                            }
                            continue;
                        }
                        const bool lower = (lane & (int)j) == 0;
                        {
                            const uint64_t ok = __shfl_xor(ka, (int)j);
                            const uint32_t oi = __shfl_xor(ia, (int)j);
                            const bool up = ((uint32_t)lane & k2) == 0;
                            const bool other_less = kless(ok, oi, ka, ia);
                            if ((lower == up) ? other_less : !other_less && !(ok == ka && oi == ia)) {
                                ka = ok;
                                ia = oi;
                            }
                        }
                        {
                            const uint64_t ok = __shfl_xor(kb, (int)j);
                            const uint32_t oi = __shfl_xor(ib, (int)j);
                            const bool up = ((uint32_t)(64 + lane) & k2) == 0;
                            const bool other_less = kless(ok, oi, kb, ib);
                            if ((lower == up) ? other_less : !other_less && !(ok == kb && oi == ib)) {
                                kb = ok;
                                ib = oi;
                            }
                        }
                    }
                }
                vkey[lane] = ka;
                vinfo[lane] = ia;
                vkey[64 + lane] = kb;
                vinfo[64 + lane] = ib;
            }
            __syncthreads();
        } else {
        for (uint32_t i = nv + tid; i < P; i += TB) {
            vkey[i] = kEmpty;
            vinfo[i] = 1u << 31;
        }
        __syncthreads();
        for (uint32_t k2 = 2; k2 <= P; k2 <<= 1) {  // bitonic sort, ascending
            for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
                for (uint32_t i = tid; i < P; i += TB) {
                    const uint32_t ij = i ^ j;
                    if (ij > i) {
                        const uint64_t ka = vkey[i], kb = vkey[ij];
                        const uint32_t ia = vinfo[i], ib = vinfo[ij];
                        const bool up = (i & k2) == 0;
                        if (kless(kb, ib, ka, ia) == up) {
                            vkey[i] = kb;
                            vkey[ij] = ka;
                            vinfo[i] = ib;
                            vinfo[ij] = ia;
                        }
                    }
                }
                __syncthreads();
            }
        }
        }
        // remove_censored_exts + output at the group's capacity offset (terminal / isolated
        // counts by ballots: one LDS atomic per wave, not per entry)
        for (uint32_t i0 = 0; i0 < nv; i0 += TB) {
            const uint32_t i = i0 + tid;
            bool term = false, iso = false;
            if (i < nv) {
            const uint64_t key = direct ? myk : vkey[i];
            const uint32_t info = direct ? myi : vinfo[i];
            const uint32_t e = (info >> 16) & 0xFFu;
            uint32_t ne = 0;
            for (int bit = 0; bit < 8; ++bit) {
                if (!((e >> bit) & 1u)) continue;
                const uint64_t bb = (uint64_t)(bit & 3);
                const uint64_t nb = bit < 4 ? (key >> 2) | (bb << (2 * K - 2)) : ((key << 2) | bb) & kmask;
                if (valid_at(nb)) ne |= 1u << bit;
            }
            const int64_t o = base + (direct ? rank : i);
            if (lo_only) {
                t_kmer[o] = key;
            } else {
                t_kmer[2 * o] = 0;
                t_kmer[2 * o + 1] = key;
            }
            t_ext[o] = (uint8_t)ne;
            t_cnt[o] = (uint16_t)(info & 0xFFFFu);
            const bool l0 = (ne & 0xFu) == 0, r0b = (ne >> 4) == 0;
            term = l0 || r0b;
            iso = l0 && r0b;
            }
            const uint64_t tb = __ballot(term), ib = __ballot(iso);
            if (lane == 0) {
                if (tb) atomicAdd(&s_term, (uint32_t)__popcll(tb));
                if (ib) atomicAdd(&s_iso, (uint32_t)__popcll(ib));
            }
        }
        __syncthreads();
        reset_claimed();  // the barrier below orders these before the next group's inserts
        if (tid == 0) {
            gcount[g] = nv;
            gstat[5 * g + 3] = s_term;
            gstat[5 * g + 4] = s_iso;
            s_claimed = 0;
        }
        __syncthreads();
        KT(6);
    }
    }
#ifdef ROGTK_KMER_TIMING
    KT(7);
    if (tid == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&g_kmer_clk[k], kt_acc[k]);
#endif
}

// ------------------------------------------------------ wave-per-group path (round 6)
// Class 2 (k_eff <= 16, <= 64 rows, <= kWaveWords packed words): ONE wave per group, with
// a wave-private LDS hash table and no workgroup barrier. The workgroup kernel above holds
// 8 waves per group through barrier-separated phases in which most waves idle (a C3 group
// at k_eff 16: ~1,650 observations, ~157 valid k-mers, ~30k clocks per group); here each
// wave runs its own group start to end, so the CU interleaves up to 16 groups' inserts.
//   * table: 32-bit keys TK (k_eff <= 16) beside 32-bit count << 8 | exts TV; empty = all-ones
//     key, so the all-T 16-mer counts in a slot of its own (TV[kWaveSlots]);
//   * insert: a 32-bit CAS claims an empty key slot or finds the key, a returning add counts
//     it, and an OR follows only when the add's old value lacks one of its extension bits
//     (half the LDS dwords of a 64-bit slot's CAS + add);
//   * lane task = (row, segment of the row), each segment started at a rotation of its row so
//     the rows' lanes - copies of one template - hit different k-mers in a trip; a lane rolls
//     a 32-base window along its segment (one packed word read per step, ahead of its CAS);
//   * CountFilter: a scan of the table compacts the valid entries (ballot prefix) in place; a
//     rank sort by 256 key buckets gives each entry its output place; censoring looks the
//     neighbours up in the bucketed keys; terminal / isolated counts by ballots.
// A group with more than kWaveClaim distinct or kWaveValid valid k-mers moves to class 3
// (launched after this kernel): the outputs never depend on the path.
// The next group's descriptor and packed words are loaded into registers while the current
// group is processed (the descriptor two groups ahead), so a group waits on HBM only when
// its chunk of 64 groups starts.
// Two instances: 1024 slots (class 2), and 2048 (class 6) for the groups past class 2's
// claim bound or packed words (39..64 rows of 150 bases): at C3's UMI collision rate a group of 22-38 rows often holds
// 2-3 molecules' reads, past 768-832 distinct k-mers (~7% of the k_eff-16 work went to the
// workgroup kernel before the big instance)
constexpr int kWaveRows = 64;       // one row per lane
constexpr uint8_t kClsWaveBig = 6;  // the 2048-slot instance's class
template <int SLOTS>
struct WaveCfg {
    static constexpr int kSlots = SLOTS;          // table slots per wave (8 / 16 KB)
    static constexpr int kClaim = SLOTS * 13 / 16;  // distinct k-mers (checked every 2 trips: <= 15/16 of the slots)
    static constexpr int kValid = SLOTS / 2;      // valid k-mers (compacted to the front; keys bucketed behind them)
    static constexpr int kWords = SLOTS == 1024 ? 192 : 320;  // packed words (38 / 64 rows at stride 5)
    static constexpr int kWG = SLOTS == 1024 ? 2 : 1;          // waves per workgroup (8 workgroups per CU)
    static constexpr int kWPL = (kWords + 63) / 64;            // prefetched words per lane
    static constexpr uint8_t kCls = SLOTS == 1024 ? 2 : kClsWaveBig;
};
constexpr int kWaveWords = WaveCfg<1024>::kWords, kWaveBigWords = WaveCfg<2048>::kWords;
constexpr uint32_t kWEmpty = 0xFFFFFFFFu;  // an empty key slot (the all-T 16-mer has a counter of its own)

__device__ __forceinline__ void wave_lds_sync() {  // the wave's LDS writes before its reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int SLOTS>
__device__ __forceinline__ uint32_t wave_hash(uint32_t key) {
    // xor-fold + one 24-bit multiply (full rate; a 32-bit mul_lo is quarter rate, and this
    // kernel is bound by issue): k-mers of consecutive positions are shifts of each other
    // (the compiler turns __umul24 of a masked operand into a quarter-rate v_mul_lo_u32;
    // the 24-bit multiply is spelled out)
    const uint32_t x = key ^ (key >> 14) ^ (key >> 25);
    uint32_t m;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(m) : "v"(x), "v"(0x9E3779u));
    return (m >> 12) & (SLOTS - 1);
}

template <int SLOTS>
__global__ __launch_bounds__(64 * WaveCfg<SLOTS>::kWG) __attribute__((amdgpu_waves_per_eu(SLOTS == 1024 ? 4 : 2, 8))) void k_kmer_wave(const GroupDesc* __restrict__ gdesc, int64_t G,
                                                           uint8_t* __restrict__ gsmall, int K, int64_t min_cov,
                                                           const int32_t* __restrict__ row_len,
                                                           const int64_t* __restrict__ woff, int stride,
                                                           const uint64_t* __restrict__ packed,
                                                           const int64_t* __restrict__ cap_off,
                                                           uint64_t* __restrict__ t_kmer, uint8_t* __restrict__ t_ext,
                                                           uint16_t* __restrict__ t_cnt, int64_t* __restrict__ gcount,
                                                           unsigned long long* __restrict__ gstat, int lo_only) {
    using WC = WaveCfg<SLOTS>;
    constexpr int kWaveSlots = WC::kSlots, kWaveClaim = WC::kClaim, kWaveValid = WC::kValid, kWaveWG = WC::kWG,
                  kWaveWPL = WC::kWPL;
    constexpr int kBuf = WC::kWords;
    static_assert(2 * kWaveValid <= kWaveSlots, "entries + bucketed keys fit the key table");
    // per wave: keys TK[kWaveSlots + 1], then count | exts TV[kWaveSlots + 1]. Slot kWaveSlots
    // is the all-T key's at k_eff 16 (its key equals the empty mark): TK[kWaveSlots] stays
    // empty, so its CAS finds "empty" at once and its count lands in TV[kWaveSlots]
    constexpr int kTV = kWaveSlots + 4;
    __shared__ uint32_t s_tab[kWaveWG][kTV + kWaveSlots + 4];
    __shared__ __attribute__((aligned(16))) uint64_t s_buf[kWaveWG][kBuf + 2];
    static_assert((kBuf + 2) * 8 >= 256 * 4, "the rank sort's 256 bucket heads fit the words' LDS");
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* const TK = s_tab[wv];
    uint32_t* const TV = TK + kTV;
    uint64_t* const W = s_buf[wv];
    const uint32_t kmask = K >= 16 ? 0xFFFFFFFFu : (1u << (2 * K)) - 1u;
    // the rank sort's bucket: the key's top 8 bits, and never its last base (bsh >= 2)
    const int bsh = 2 * K - 8 >= 2 ? 2 * K - 8 : 2;
    for (int i = lane; i < kWaveSlots; i += 64) {
        TK[i] = kWEmpty;
        TV[i] = 0u;
    }
    if (lane == 0) {
        TK[kWaveSlots] = kWEmpty;
        TV[kWaveSlots] = 0u;
    }
    const int64_t n_chunks = (G + 63) >> 6;
    const int64_t nw = (int64_t)gridDim.x * kWaveWG;
    int64_t ch = (int64_t)blockIdx.x * kWaveWG + wv;
    uint64_t own = ch < n_chunks ? __ballot((ch << 6) + lane < G && gsmall[(ch << 6) + lane] == WC::kCls) : 0ull;
    // the next group of this class for this wave (-1: none); loads the chunk's classes as needed
    auto next_group = [&]() -> int64_t {
        while (true) {
            if (own) {
                const int i = __ffsll((unsigned long long)own) - 1;
                own &= own - 1;
                return (ch << 6) + i;
            }
            ch += nw;
            if (ch >= n_chunks) return -1;
            own = __ballot((ch << 6) + lane < G && gsmall[(ch << 6) + lane] == WC::kCls);
        }
    };
    // prefetch state of the next group: its row (lane) and packed words in registers
    int32_t p_len = 0, p_wo = 0;
    uint64_t p_words[kWaveWPL];
    auto load_group = [&](const GroupDesc& dd) {
        p_len = 0;
        p_wo = 0;
        if (lane < dd.nrows) {
            p_len = row_len[dd.r0 + lane];
            p_wo = stride ? lane * stride : (int32_t)(woff[dd.r0 + lane] - dd.w0);
        }
#pragma unroll
        for (int j = 0; j < kWaveWPL; ++j) {
            const int i = lane + 64 * j;
            p_words[j] = i < dd.nwords ? packed[dd.w0 + i] : 0ull;
        }
    };
    // descriptors by a VECTOR load (lane k < 6 takes dword k, readlane after): a scalar load
    // would share lgkmcnt with the LDS operations, and every LDS wait of the group before it
    // would wait for the prefetch too
    auto desc_load = [&](int64_t gg) -> uint32_t {
        return gg >= 0 && lane < 6 ? reinterpret_cast<const uint32_t*>(gdesc + gg)[lane] : 0u;
    };
    auto desc_get = [&](uint32_t dw) -> GroupDesc {
        GroupDesc o;
        o.r0 = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dw, 1) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)dw, 0));
        o.w0 = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dw, 3) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)dw, 2));
        o.nrows = __builtin_amdgcn_readlane((int)dw, 4);
        o.nwords = __builtin_amdgcn_readlane((int)dw, 5);
        return o;
    };
    static_assert(sizeof(GroupDesc) == 24, "GroupDesc: 6 dwords");
    int64_t g = next_group();
    GroupDesc d = desc_get(desc_load(g));
    if (g >= 0) load_group(d);
    int64_t g1 = g >= 0 ? next_group() : -1;
    uint32_t dw1 = desc_load(g1);
#ifdef ROGTK_KMER_TIMING
    const int tid = lane;
    unsigned long long kt_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, kt_last = wall_clock64();
#endif
    for (; g >= 0;) {
        const int nrows = d.nrows, nwords = d.nwords;
        // this group's rows: lane r holds row r's observation count, length and word offset
        const int c_len = p_len, c_wo = p_wo;
        const int c_nobs = lane < nrows && c_len ? max(c_len - K + 1, 0) : 0;
#pragma unroll
        for (int j = 0; j < kWaveWPL; ++j) {
            const int i = lane + 64 * j;
            if (i < nwords) W[i] = p_words[j];
        }
        if (lane == 0) W[nwords] = 0;  // the second word of a k-mer in the last word
        wave_lds_sync();
        // the next group's rows and words in flight while this group is processed, and the
        // descriptor of the one after it
        GroupDesc d1{0, 0, 0, 0};
        if (g1 >= 0) {
            d1 = desc_get(dw1);
            load_group(d1);
        }
        const int64_t g2 = g1 >= 0 ? next_group() : -1;
        const uint32_t dw2 = desc_load(g2);
        KT(0);
        // inserts, one pass: lane task = (row, segment), spr = floor(64 / rows) segments
        // per row of Ls = ceil(longest / spr) positions (a C3 group of ~12 rows of 135
        // observations: 60 lanes of 27 steps). Each lane starts its segment at a rotation of
        // its row (7 r mod its length) and wraps, so the rows' lanes - copies of one template -
        // insert different k-mers in a step instead of all hitting one slot
        int maxn = c_nobs;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) maxn = max(maxn, __shfl_xor(maxn, m));
        const int spr = nrows > 0 ? max(1, 64 / nrows) : 1;
        // (uniform: the trip loop and its exit stay scalar branches)
        const int Ls = __builtin_amdgcn_readfirstlane((maxn + spr - 1) / spr);
        const int r = lane / spr;
        const int seg = lane - r * spr;
        const int rs = r < nrows ? r : 0;
        const int nobs_r = __shfl(c_nobs, rs), len_r = __shfl(c_len, rs), wo_r = __shfl(c_wo, rs);
        const int pst = seg * Ls;
        const int nst = r < nrows ? min(max(nobs_r - pst, 0), Ls) : 0;
        const int rot = nst > 0 ? (7 * r) % nst : 0;
        // the base before the segment (left extension of its first k-mer) and the one before
        // the rotated start: later steps take the previous k-mer's first base
        auto base_at = [&](int q) -> uint32_t {  // base q of the lane's row (q >= 0)
            return (uint32_t)(W[wo_r + (q >> 5)] >> (62 - 2 * (q & 31))) & 3u;
        };
        auto win_at = [&](int q) -> uint64_t {  // bases q .. q + 31 of the lane's row
            const int wi = wo_r + (q >> 5);
            const uint64_t w0 = W[wi], w1 = W[wi + 1];
            const int o = 2 * (q & 31);
            return o ? (w0 << o) | (w1 >> (64 - o)) : w0;
        };
        // a rolling window: win holds the 32 bases from the lane's position p and nwd the
        // packed word that supplies base p + 32, so a step shifts one base in; the next
        // position's word is read before the trip's CAS, whose wait covers it (no LDS read
        // of its own on the trip's chain). The segment's start window is kept for the wrap.
        const uint32_t wrapb = nst > 0 && pst > 0 ? base_at(pst - 1) : 0u;
        uint32_t prevb = nst > 0 && pst + rot > 0 ? base_at(pst + rot - 1) : 0u;
        uint32_t key = 0u, key_s = 0u;
        uint64_t aw = 0;
        int p = pst + rot;
        if (nst > 0) {
            key_s = (uint32_t)(win_at(pst) >> (64 - 2 * K)) & kmask;
            key = rot ? (uint32_t)(win_at(p) >> (64 - 2 * K)) & kmask : key_s;
            aw = W[wo_r + ((p + K) >> 5)];
        }
        uint32_t claims = 0;
        bool over = false;
        // one insert step of the lane's segment; returns the wave's new claims
        auto step = [&](int t, auto check) -> uint32_t {
            uint32_t v = 0u, allt = 1u;  // (a lane past its segment claims nothing)
            if (!decltype(check)::value || t < nst) {
                const uint32_t rb = (uint32_t)(aw >> (62 - 2 * ((p + K) & 31))) & 3u;  // base p+K
                uint32_t e = p > 0 ? 1u << prevb : 0u;
                if (p + K < len_r) e |= 16u << rb;
                uint32_t h = wave_hash<SLOTS>(key);
                const bool wrap = p + 1 == pst + nst;
                const int pn = wrap ? pst : p + 1;
                const uint64_t aw_n = W[wo_r + ((pn + K) >> 5)];
                // claim or find the key's slot (a 32-bit CAS), then count it: a returning add
                // whose old value shows whether the extension bits are new (then an OR)
                allt = key == kWEmpty;
                h = allt ? (uint32_t)kWaveSlots : h;
                v = atomicCAS(&TK[h], kWEmpty, key);
                // one combined test (bitwise: no branch per condition)
                for (uint32_t miss = (uint32_t)(v != kWEmpty) & (uint32_t)(v != key); miss;
                     miss = (uint32_t)(v != kWEmpty) & (uint32_t)(v != key)) {
                    h = (h + 1) & (kWaveSlots - 1);
                    v = atomicCAS(&TK[h], kWEmpty, key);
                }
                const uint32_t old = atomicAdd(&TV[h], 1u << 8);
                atomicOr(&TV[h], e & ~old & 0xFFu);  // (no branch: an OR of 0 changes nothing)
                // the next position (a wrap restarts the segment): selects by masks, no branch
                prevb = wrap ? wrapb : key >> (2 * K - 2);
                key = wrap ? key_s : ((key << 2) | rb) & kmask;
                aw = aw_n;
                p = pn;
            }
            return (uint32_t)__popcll(__ballot((v == kWEmpty) & (allt == 0u)));
        };
        // the claim bound is checked every second step: <= 13/16 + 128 keys stay below the
        // table's 1024 slots, so probing always ends
        // trips every row's lanes take (the shortest segment of a row: its last one) run
        // inside one exec mask of the rows' lanes, without a per-trip segment test
        int lmin = r < nrows ? nst : 1 << 30;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) lmin = min(lmin, __shfl_xor(lmin, m));
        const int L0 = __builtin_amdgcn_readfirstlane(min(lmin, Ls)) & ~1;  // even: checks stay paired
        using kNoCheck = std::integral_constant<bool, false>;
        using kCheck = std::integral_constant<bool, true>;
        int t = 0;
        if (r < nrows) {
            for (; t < L0; t += 2) {
                claims += step(t, kNoCheck{});
                claims += step(t + 1, kNoCheck{});
                if (claims > (uint32_t)kWaveClaim) {
                    over = true;
                    break;
                }
            }
        }
        t = __builtin_amdgcn_readfirstlane(t);
        over = __builtin_amdgcn_readfirstlane((int)over) != 0;
        claims = __builtin_amdgcn_readfirstlane(claims);
        for (; !over && t < Ls; t += 2) {
            claims += step(t, kCheck{});
            if (t + 1 < Ls) claims += step(t + 1, kCheck{});
            if (claims > (uint32_t)kWaveClaim) {
                over = true;
                break;
            }
        }
        wave_lds_sync();
        KT(1);
        // CountFilter: the valid entries compacted IN PLACE to the front of the two arrays (key;
        // count | exts << 16; a chunk's 64 slots are read before any entry is written, and entries
        // only move down); the table is rebuilt empty after the group, and the censoring below
        // looks neighbours up in the bucketed keys instead of the hash table
        uint32_t nv = 0;
        if (!over) {
            for (int s0 = 0; s0 < kWaveSlots; s0 += 64) {
                const uint32_t k = TK[s0 + lane], v = TV[s0 + lane];
                const uint32_t cnt = v >> 8;
                const bool ok = k != kWEmpty && (int64_t)min(cnt, 0xFFFFu) >= min_cov;
                const uint64_t bm = __ballot(ok);
                const uint32_t at = nv + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
                if (ok && at < (uint32_t)kWaveValid) {
                    TK[at] = k;
                    TV[at] = min(cnt, 0xFFFFu) | ((v & 0xFFu) << 16);
                }
                nv += (uint32_t)__popcll(bm);
            }
            const uint32_t vt = TV[kWaveSlots];  // the all-T key (the largest key: it ranks last)
            if ((int64_t)min(vt >> 8, 0xFFFFu) >= min_cov && vt >= (1u << 8)) {
                if (lane == 0 && nv < (uint32_t)kWaveValid) {
                    TK[nv] = kWEmpty;
                    TV[nv] = min(vt >> 8, 0xFFFFu) | ((vt & 0xFFu) << 16);
                }
                ++nv;
            }
            if (nv > (uint32_t)kWaveValid) over = true;
        }
        uint32_t term = 0, iso = 0;
        if (!over && nv > 0) {
            // rank sort by buckets: the key's top 8 bits pick one of 256 buckets (an entry's
            // bucket holds ~1 key at C3's ~150 valid k-mers), an LDS atomic gives each entry its
            // place in its bucket (kept in the entry's bits 24..31), a wave scan the buckets'
            // starts; the bucketed keys K2 (behind the entries) give an entry's rank (its
            // bucket's start + the keys of its bucket below it) and the censoring's neighbour
            // lookups (a valid neighbour is one of K2's keys). bsh >= 2, so the four right
            // neighbours of a key share a bucket: one scan decides its four right bits.
            uint32_t* const K2 = TK + kWaveValid;
            uint32_t* const C = reinterpret_cast<uint32_t*>(W);  // the words are dead by now
            reinterpret_cast<uint4*>(C)[lane] = make_uint4(0u, 0u, 0u, 0u);
            wave_lds_sync();
            KT(2);
            bool deep = false;  // a bucket past 255 entries (adversarial keys): class 3
            for (uint32_t i = lane; i < nv; i += 64) {
                const uint32_t li = atomicAdd(&C[TK[i] >> bsh & 255u], 1u);
                deep |= li > 255u;
                TV[i] |= min(li, 255u) << 24;
            }
            if (__ballot(deep)) {
                over = true;
            } else {
                wave_lds_sync();
                const uint4 c4 = reinterpret_cast<const uint4*>(C)[lane];  // buckets 4 lane .. 4 lane + 3
                const uint32_t bc = c4.x + c4.y + c4.z + c4.w;
                uint32_t incl = bc;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t t = __shfl_up(incl, off);
                    if (lane >= off) incl += t;
                }
                // each bucket's start and count in LDS (the lookups below run under divergent
                // control flow, where a cross-lane read of an inactive lane is not defined)
                uint32_t st = incl - bc;
                uint4 o4;
                o4.x = st | (c4.x << 16);
                st += c4.x;
                o4.y = st | (c4.y << 16);
                st += c4.y;
                o4.z = st | (c4.z << 16);
                st += c4.z;
                o4.w = st | (c4.w << 16);
                reinterpret_cast<uint4*>(C)[lane] = o4;
                wave_lds_sync();
                for (uint32_t i = lane; i < nv; i += 64) {
                    const uint32_t k = TK[i];
                    K2[(C[k >> bsh & 255u] & 0xFFFFu) + (TV[i] >> 24)] = k;
                }
                wave_lds_sync();
                KT(3);
                const int64_t base = cap_off[g];
                const uint32_t kmask2 = kmask >> 2;
                for (uint32_t i0 = 0; i0 < nv; i0 += 64) {
                    const uint32_t i = i0 + lane;
                    const bool live = i < nv;
                    const uint32_t key = live ? TK[i] : 0u, v = live ? TV[i] : 0u;
                    bool tm = false, is = false;
                    if (live) {
                        const uint32_t ex = (uint32_t)(v >> 16) & 0xFFu;
                        // the three bucket heads first (independent reads), then the scans
                        const uint32_t q = C[key >> bsh & 255u];
                        const uint32_t qr = C[((key << 2) & kmask) >> bsh & 255u];
                        const uint32_t at = q & 0xFFFFu, bn = q >> 16;
                        uint32_t rank = at;
                        // the first 4 keys of a bucket by predicated reads (a bucket holds ~1
                        // key; the key table's pad keeps the reads in bounds), a loop past them
#pragma unroll
                        for (uint32_t m = 0; m < 4; ++m) rank += (uint32_t)(m < bn) & (uint32_t)(K2[at + m] < key);
                        for (uint32_t m = 4; m < bn; ++m) rank += K2[at + m] < key;
                        uint32_t nx = 0;
                        {
                            const uint32_t ar = qr & 0xFFFFu, nr = qr >> 16, lo = key & kmask2;
#pragma unroll
                            for (uint32_t m = 0; m < 4; ++m) {
                                const uint32_t k2 = K2[ar + m];
                                nx |= ((uint32_t)(m < nr) & (uint32_t)((k2 >> 2) == lo)) << (4 + (k2 & 3u));
                            }
                            for (uint32_t m = 4; m < nr; ++m) {
                                const uint32_t k2 = K2[ar + m];
                                if ((k2 >> 2) == lo) nx |= 16u << (k2 & 3u);
                            }
                            nx &= ex & 0xF0u;
                        }
                        // left neighbours: the first set bit (nearly always the only one)
                        // straight-line with predicated reads, any further bits by a loop
                        uint32_t lb = ex & 0xFu;
                        {
                            const uint32_t bb = (uint32_t)__builtin_ctz(lb | 0x10u) & 3u;
                            const uint32_t nb = (key >> 2) | (bb << (2 * K - 2));
                            const uint32_t q2 = C[nb >> bsh & 255u], a2 = q2 & 0xFFFFu;
                            const uint32_t n2 = lb ? q2 >> 16 : 0u;
                            uint32_t hit = 0u;
#pragma unroll
                            for (uint32_t m = 0; m < 4; ++m) hit |= (uint32_t)(m < n2) & (uint32_t)(K2[a2 + m] == nb);
                            for (uint32_t m = 4; m < n2; ++m) hit |= (uint32_t)(K2[a2 + m] == nb);
                            nx |= hit << bb;
                            lb &= lb - 1;
                        }
                        for (; lb; lb &= lb - 1) {
                            const uint32_t bb = (uint32_t)__builtin_ctz(lb);
                            const uint32_t nb = (key >> 2) | (bb << (2 * K - 2));
                            const uint32_t q2 = C[nb >> bsh & 255u], a2 = q2 & 0xFFFFu, n2 = q2 >> 16;
                            uint32_t hit = 0u;  // (no early exit: a bucket holds ~1 key)
                            for (uint32_t m = 0; m < n2; ++m) hit |= (uint32_t)(K2[a2 + m] == nb);
                            nx |= hit << bb;
                        }
                        const int64_t o = base + rank;
                        if (lo_only) {
                            t_kmer[o] = key;
                        } else {
                            t_kmer[2 * o] = 0;
                            t_kmer[2 * o + 1] = key;
                        }
                        t_ext[o] = (uint8_t)nx;
                        t_cnt[o] = (uint16_t)(v & 0xFFFFu);
                        const bool l0 = (nx & 0xFu) == 0, r0b = (nx >> 4) == 0;
                        tm = l0 || r0b;
                        is = l0 && r0b;
                    }
                    term += (uint32_t)__popcll(__ballot(tm));
                    iso += (uint32_t)__popcll(__ballot(is));
                }
            }
        }
        // more than this instance takes: the 2048-slot instance (launched next) or class 3 redoes it
        if (over && lane == 0) gsmall[g] = SLOTS == 1024 && nwords <= kWaveBigWords ? kClsWaveBig : 3;
        KT(4);
        if (lane == 0 && !over) {
            gcount[g] = nv;
            gstat[5 * g + 3] = term;
            gstat[5 * g + 4] = iso;
        }
        wave_lds_sync();
        for (int i = lane; i < kWaveSlots; i += 64) {
            TK[i] = kWEmpty;
            TV[i] = 0u;
        }
        if (lane == 0) TV[kWaveSlots] = 0u;
        wave_lds_sync();
        KT(5);
        g = g1;
        d = d1;
        g1 = g2;
        dw1 = dw2;
    }
#ifdef ROGTK_KMER_TIMING
    KT(6);
    if (lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&g_kmer_clk[k], kt_acc[k]);
#endif
}

// Per group of effective k K: observation, row and packed-word totals decide the path.
// 16 lanes per group (a C3 group has ~10 rows: a wave per group left most lanes idle);
// caps != NULL: also the group's output capacity (valid_cap of its observations)
constexpr int kClsLanes = 16;
// a group with nothing valid by the repeat certificate: no LDS kernel takes it, its rows
// leave the global path (k_drop_small_rows), its count and stats stay 0 (zeroed per call)
constexpr uint8_t kClsEmpty = 5;
__global__ __launch_bounds__(kBlock) void k_group_classify(const int64_t* __restrict__ go, int64_t G,
                                                           const uint8_t* __restrict__ gk, int K,
                                                           const int64_t* __restrict__ row_obs,
                                                           const int64_t* __restrict__ row_words,
                                                           const int64_t* __restrict__ woff, int stride,
                                                           uint8_t* __restrict__ gsmall, GroupDesc* __restrict__ gdesc,
                                                           int64_t* __restrict__ caps, int64_t min_cov,
                                                           const unsigned long long* __restrict__ gstat, int wave) {
    const int sub = threadIdx.x & (kClsLanes - 1);
    const int64_t step = (int64_t)gridDim.x * (kBlock / kClsLanes);
    // every segment of a wave runs the same number of trips (the shuffles need the lanes)
    const int64_t first = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kClsLanes;
    const int64_t wave_first = first - ((threadIdx.x & 63) / kClsLanes);
    for (int64_t base = wave_first; base < G; base += step) {
        const int64_t g = base + (first - wave_first);
        const bool live = g < G && gk[g] == K;
        int64_t obs = 0, words = 0, used = 0;
        if (live)
            for (int64_t r = go[g] + sub; r < go[g + 1]; r += kClsLanes) {
                const int64_t o = row_obs[r];
                obs += o;
                used += o > 0;
                if (!stride) words += row_words[r];
            }
        for (int m = kClsLanes / 2; m > 0; m >>= 1) {
            obs += __shfl_xor(obs, m);
            words += __shfl_xor(words, m);
            used += __shfl_xor(used, m);
        }
        if (sub != 0 || g >= G) continue;
        if (!live) {
            gsmall[g] = 0;
            if (caps) caps[g] = 0;
            continue;
        }
        const int64_t nrows = go[g + 1] - go[g];
        if (stride) words = nrows * stride;  // fixed-stride staging (k_row_gather)
        uint8_t cls = 0;
        // the repeat certificate (k_pack_reads): every row with observations certified and
        // fewer of them than min_cov -> no k-mer is counted min_cov times (K >= 31)
        const bool empty = gstat && K >= 31 && K <= 32 && min_cov >= 2 && used < min_cov && gstat[5 * g + 2] == 0;
        if (K <= 32 && obs > 0 && empty) {
            cls = kClsEmpty;
        } else if (K <= 32 && obs > 0) {
            if (wave && K <= 16 && nrows <= kWaveRows && words <= kWaveWords) cls = 2;
            else if (wave && K <= 16 && nrows <= kWaveRows && words <= kWaveBigWords) cls = kClsWaveBig;
            else if (wave && K <= 16 && nrows <= kWaveRows && words <= kWaveBigWords) cls = kClsWaveBig;
            else if (nrows <= LdsCfg<3>::kRows && words <= LdsCfg<3>::kWords) cls = 3;
            else if (nrows <= LdsCfg<1>::kRows && words <= LdsCfg<1>::kWords) cls = 1;
            else if (nrows <= LdsCfg<4>::kRows && words <= LdsCfg<4>::kWords) cls = 4;
        }
        gsmall[g] = cls;
        if (cls) gdesc[g] = GroupDesc{go[g], stride ? go[g] * stride : woff[go[g]], (int32_t)nrows, (int32_t)words};
        if (caps) caps[g] = cls == kClsEmpty ? 0 : obs / (min_cov > 1 ? min_cov : 1);  // valid_cap
    }
}

// The minimizer filter (below): on unless ROGTK_KMER_MZ=0 or rogtk_kmer_set_filter(0)
std::atomic<int> g_kmer_mz{-1};
// tests only (rogtk_kmer_debug_filter): per group of a call, the filter's decision
uint8_t* g_mz_debug = nullptr;
int64_t g_mz_debug_groups = 0;
inline bool kmer_mz_on() {
    int v = g_kmer_mz.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* e = getenv("ROGTK_KMER_MZ");
        v = e && e[0] == '0' ? 0 : 1;
        g_kmer_mz.store(v, std::memory_order_relaxed);
    }
    return v == 1;
}

// Round 4: the minimizer filter, a group-level certificate for class-3 groups whose rows
// are all certified (no K-mer twice in a row, K in {31, 32}; counting is stranded). A
// K-mer X counted min_cov times then occurs in min_cov distinct rows. Its minimizer m(X),
// the smallest of its W = K - 15 16-mers (2-bit codes compared as u32: lexicographic
// order), depends on X alone: every row that holds X has a window whose minimizer is
// m(X). Per group, each row adds its windows' minimizers to a count (once per run of
// consecutive windows that share one; one that returns after a gap is added again, which
// only over-counts): if no count reaches min_cov, no K-mer does, and the group has nothing
// valid (class kClsEmpty, as the row certificate gives it). About 13 distinct minimizers
// per 150-bp row are counted instead of 119 k-mer inserts.
// A lane per row: its 16-mers in blocks of 16 positions (one 32-bit half-word each),
// window minima as the suffix minimum of the first position's block and the prefix
// minimum of the last position's block (van Herk / Gil-Werman), the row's distinct
// minimizers appended to its own list in LDS; then the lists are counted in a table per
// wave, keyed by (group, minimizer). A wave takes consecutive candidate groups together
// (up to kMzG groups and 64 rows: ~2.5 C3 groups instead of one per wave pass); a group
// of more than 64 rows runs alone, 64 rows at a time. A group with a count of min_cov, or
// a row with more than kMzList minimizers, keeps its class; so does every group of a
// batch with more than kMzClaim distinct keys.
constexpr int kMzWaves = 2;    // waves per workgroup
constexpr int kMzSlots = 512;  // per wave: u64 key (batch group << 32 | minimizer) and u32 count
constexpr int kMzClaim = 384;  // distinct keys before the wave gives up (<= 448 claimed: never full)
constexpr int kMzList = 28;    // a row's distinct minimizers (its list in LDS, + a spare slot: 29, odd, so lanes spread over banks)
constexpr int kMzG = 8;        // groups per batch
// a batch of groups, spread over the lanes: lane i < ng holds group i's id; each lane
// holds its own row of the first pass (group index, row and word positions); uniform:
// the group and row counts, and group 0's row and word bases (passes past 64 rows)
struct MzBatch {
    int ng, rows;
    int64_t r00, w00;
    int64_t g;      // lane i < ng: group i
    int j;          // this lane's group in the batch
    int64_t ri, wi;  // this lane's row: row_len index, first word index
};
__global__ __launch_bounds__(64 * kMzWaves) void k_minimizer_filter(const GroupDesc* __restrict__ gdesc, int64_t G,
                                                                     uint8_t* __restrict__ gsmall, int K,
                                                                     int64_t min_cov,
                                                                     const int32_t* __restrict__ row_len, int stride,
                                                                     const uint64_t* __restrict__ packed,
                                                                     const unsigned long long* __restrict__ gstat,
                                                                     uint8_t* __restrict__ dbg) {
    constexpr int NW = 7;       // B = 8 blocks: at most 7 base words (224 bases) per row
    constexpr int NH = 2 * NW;  // 32-bit half-words: 16 positions each
    __shared__ unsigned long long s_key[kMzWaves][kMzSlots];
    __shared__ uint32_t s_cnt[kMzWaves][kMzSlots];
    __shared__ uint32_t s_list[kMzWaves][64 * (kMzList + 1)];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long* const key = s_key[wv];
    uint32_t* const cnt = s_cnt[wv];
    uint32_t* const lst = s_list[wv] + lane * (kMzList + 1);
    constexpr unsigned long long kNone = ~0ull;  // the empty key (a batch group index is < kMzG)
    for (int i = lane; i < kMzSlots; i += 64) {
        key[i] = kNone;
        cnt[i] = 0;
    }
    const bool w17 = K == 32;  // windows of 17 16-mers (K = 32) or 16 (K = 31)
    const uint32_t hit = (uint32_t)min_cov;
    // the candidate groups, in order: class-3 groups whose rows are all certified, in
    // chunks of 64 ids: a chunk's classes, certificate counts and descriptors are one
    // load per lane, issued a chunk ahead
    const int64_t n_chunks = (G + 63) >> 6;
    int64_t ch = (int64_t)blockIdx.x * kMzWaves + wv;
    const int64_t ch_step = (int64_t)gridDim.x * kMzWaves;
    struct Chunk {
        bool cand;
        int64_t r0, w0;
        int32_t nrows;
    };
    auto chunk_load = [&](int64_t c) {
        Chunk k{false, 0, 0, 0};
        const int64_t gl = (c << 6) + lane;
        if (c < n_chunks && gl < G) {
            const uint8_t cls = gsmall[gl];
            const unsigned long long unc = gstat[5 * gl + 2];
            const GroupDesc e = gdesc[gl];
            k.cand = cls == 3 && unc == 0;
            k.r0 = e.r0;
            k.w0 = e.w0;
            k.nrows = e.nrows;
        }
        return k;
    };
    auto rl64 = [](int64_t v, int i) {
        return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), i) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)v, i));
    };
    Chunk cur = chunk_load(ch), nxt = chunk_load(ch + ch_step);
    uint64_t own = ch < n_chunks ? __ballot(cur.cand) : 0;
    int64_t cur_base = ch << 6;
    bool done = ch >= n_chunks;
    // the next candidate group (wave-uniform); false when the wave's chunks are done
    auto next_group = [&](int64_t& g, int64_t& r0, int64_t& w0, int& nrows) {
        while (!own) {
            if (done) return false;
            ch += ch_step;
            if (ch >= n_chunks) {
                done = true;
                return false;
            }
            cur = nxt;
            cur_base = ch << 6;
            nxt = chunk_load(ch + ch_step);
            own = __ballot(cur.cand);
        }
        const int i = __ffsll((unsigned long long)own) - 1;
        own &= own - 1;
        g = cur_base + i;
        r0 = rl64(cur.r0, i);
        w0 = rl64(cur.w0, i);
        nrows = __builtin_amdgcn_readlane(cur.nrows, i);
        return true;
    };
    // batches: consecutive candidates while they fit 64 rows (a group of more rows alone)
    bool have_p = false;
    int64_t pg = 0, pr0 = 0, pw0 = 0;
    int pn = 0;
    auto form = [&](MzBatch& bt) {
        bt.ng = 0;
        bt.rows = 0;
        bt.g = -1;
        bt.j = 0;
        bt.ri = bt.wi = 0;
        while (true) {
            if (!have_p) have_p = next_group(pg, pr0, pw0, pn);
            if (!have_p) break;
            if (bt.ng > 0 && (bt.ng == kMzG || bt.rows + pn > 64)) break;
            if (bt.ng == 0) {
                bt.r00 = pr0;
                bt.w00 = pw0;
            }
            if (lane == bt.ng) bt.g = pg;
            if (lane >= bt.rows && lane < bt.rows + pn) {
                bt.j = bt.ng;
                bt.ri = pr0 + (lane - bt.rows);
                bt.wi = pw0 + (int64_t)(lane - bt.rows) * stride;
            }
            bt.rows += pn;
            ++bt.ng;
            have_p = false;
            if (bt.rows > 64) break;  // a group of more than 64 rows: alone
        }
        return bt.ng > 0;
    };
    // this lane's row of pass p of a batch: its length and words
    auto load = [&](const MzBatch& bt, int pass, uint64_t (&w)[NW], int& len) {
        const bool live = 64 * pass + lane < bt.rows;
        const int64_t ri = pass ? bt.r00 + 64 * pass + lane : bt.ri;
        const int64_t wi = pass ? bt.w00 + (int64_t)(64 * pass + lane) * stride : bt.wi;
        len = live ? row_len[ri] : 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) w[i] = live && i < stride ? packed[wi + i] : 0ull;
    };
    MzBatch cb, nb;
    uint64_t nw_[NW];
    int nlen = 0;
    bool have = form(cb);
    if (have) load(cb, 0, nw_, nlen);
    while (have) {
        uint64_t cw[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) cw[i] = nw_[i];
        int clen = nlen;
        const int cj = cb.j;  // pass 0's group; a multi-pass batch has one group (0)
        const bool have_n = form(nb);
        if (have_n) load(nb, 0, nw_, nlen);  // in flight while this batch is filtered
        bool gave_up = false, split = false;
        uint32_t claimed = 0, keep = 0;  // keep: groups with a row past kMzList minimizers
        uint32_t reach_split = 0;        // split batches: the groups that keep their class
        auto scan_reach_all = [&]() {
            uint32_t reach = 0;
            for (int i = lane; i < kMzSlots; i += 64)
                if (cnt[i] >= hit) reach |= 1u << (uint32_t)(key[i] >> 32);
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) reach |= (uint32_t)__shfl_xor((int)reach, m, 64);
            return (uint32_t)__builtin_amdgcn_readfirstlane((int)reach);
        };
        const int passes = (cb.rows + 63) >> 6;
        for (int pass = 0; pass < passes && !gave_up; ++pass) {
            if (pass) load(cb, pass, cw, clen);  // groups of more than 64 rows (rare)
            // this lane's row: its distinct window minimizers into its list
            const int nwin = clen >= K ? clen - K + 1 : 0;
            uint32_t hw[NH];
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                hw[2 * i] = (uint32_t)(cw[i] >> 32);
                hw[2 * i + 1] = (uint32_t)cw[i];
            }
            int nwmax = nwin;  // wave-uniform bound on the windows
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) nwmax = max(nwmax, __shfl_xor(nwmax, m, 64));
            nwmax = __builtin_amdgcn_readfirstlane(nwmax);
            int n = 0;
            uint32_t mprev = 0;
            // block b: windows 16 b .. 16 b + 15, from the suffix minima of block b's
            // 16-mers and the prefix minima of block b + 1's
            uint32_t suf[16];
            suf[0] = hw[0];
#pragma unroll
            for (int t = 1; t < 16; ++t) suf[t] = __builtin_amdgcn_alignbit(hw[0], hw[1], 32 - 2 * t);
#pragma unroll
            for (int t = 14; t >= 0; --t) suf[t] = min(suf[t], suf[t + 1]);
#pragma unroll
            for (int b = 0; b + 1 < NH; ++b) {
                if (16 * b >= nwmax) break;  // uniform
                const uint32_t lo = hw[b + 1], hi2 = b + 2 < NH ? hw[b + 2] : 0u;
                uint32_t pre[16], nsuf[16];
                pre[0] = lo;
#pragma unroll
                for (int t = 1; t < 16; ++t) pre[t] = __builtin_amdgcn_alignbit(lo, hi2, 32 - 2 * t);
#pragma unroll
                for (int t = 0; t < 16; ++t) nsuf[t] = pre[t];
#pragma unroll
                for (int t = 1; t < 16; ++t) pre[t] = min(pre[t], pre[t - 1]);
#pragma unroll
                for (int t = 14; t >= 0; --t) nsuf[t] = min(nsuf[t], nsuf[t + 1]);
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    const int p = 16 * b + t;
                    const uint32_t m = w17 ? min(suf[t], pre[t]) : t ? min(suf[t], pre[t - 1]) : suf[0];
                    const bool f = p < nwin && (p == 0 || m != mprev);
                    lst[min(n, kMzList)] = m;  // kept only when f (n moves on; n = kMzList: the spare slot): no branch
                    n += f;
                    mprev = m;
                }
#pragma unroll
                for (int t = 0; t < 16; ++t) suf[t] = nsuf[t];
            }
            // a row with too many minimizers: its group keeps its class
            const uint64_t over = __ballot(n > kMzList);
            if (over) {
#pragma unroll
                for (int i = 0; i < kMzG; ++i)
                    if (__ballot(n > kMzList && cj == i)) keep |= 1u << i;
            }
            const int nn = min(n, kMzList);
            int nmax = nn, total = nn;
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) {
                nmax = max(nmax, __shfl_xor(nmax, m, 64));
                total += __shfl_xor(total, m, 64);
            }
            nmax = __builtin_amdgcn_readfirstlane(nmax);
            total = __builtin_amdgcn_readfirstlane(total);
            // the lists of the lanes in `sel` into the table; with a cap on the claims
            // (none is needed while the keys inserted stay within kMzClaim)
            // each lane walks its list from its own rotation: the rows of one group (copies of
            // one molecule) hold the same minimizers in the same order, and lanes adding the
            // same key in one step serialise on its slot
            const int rot = nn > 0 ? (5 * lane) % nn : 0;
            auto insert = [&](bool sel, bool capped) {
                uint32_t claimed_here = 0;
                for (int k = 0; k < nmax; ++k) {
                    bool fresh = false;
                    if (sel && k < nn) {
                        const int kk0 = k + rot;
                        const uint32_t m = lst[kk0 >= nn ? kk0 - nn : kk0];
                        const unsigned long long kk = ((unsigned long long)cj << 32) | m;
                        uint32_t slot = ((m ^ (uint32_t)cj * 0x85EBCA77u) * 0x9E3779B1u) >> 23;  // 512 slots
                        while (true) {
                            const unsigned long long prev = atomicCAS(&key[slot], kNone, kk);
                            if (prev == kNone || prev == kk) {
                                fresh = prev == kNone;
                                break;
                            }
                            slot = (slot + 1) & (kMzSlots - 1);
                        }
                        atomicAdd(&cnt[slot], 1u);
                    }
                    if (capped) {
                        claimed_here += (uint32_t)__popcll(__ballot(fresh));
                        if (claimed + claimed_here > (uint32_t)kMzClaim) return claimed_here;
                    }
                }
                return claimed_here;
            };
            auto scan_reach = [&]() {  // the table's groups with a count of min_cov
                uint32_t reach = 0;
                for (int i = lane; i < kMzSlots; i += 64)
                    if (cnt[i] >= hit) reach |= 1u << (uint32_t)(key[i] >> 32);
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) reach |= (uint32_t)__shfl_xor((int)reach, m, 64);
                return (uint32_t)__builtin_amdgcn_readfirstlane((int)reach);
            };
            auto reset = [&]() {
                __builtin_amdgcn_wave_barrier();
                for (int i = lane; i < kMzSlots; i += 64) {
                    key[i] = kNone;
                    cnt[i] = 0;
                }
                __builtin_amdgcn_wave_barrier();
            };
            if (cb.ng == 1) {  // one group (of up to 3 passes): claims capped over its passes
                claimed += insert(true, true);
                if (claimed > (uint32_t)kMzClaim) gave_up = true;
            } else if (total <= kMzClaim || insert(true, true) <= (uint32_t)kMzClaim) {
                // the whole batch in one table (inserted above when it may pass the cap)
                if (total <= kMzClaim) insert(true, false);
            } else {  // too many distinct keys for one table: the batch's groups one at a time
                reset();
                split = true;
                for (int i = 0; i < cb.ng; ++i) {
                    claimed = 0;
                    claimed = insert(cj == i, true);
                    __builtin_amdgcn_wave_barrier();
                    if (claimed > (uint32_t)kMzClaim) reach_split |= 1u << i;  // gave up: keeps its class
                    else reach_split |= scan_reach() & (1u << i);
                    reset();
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (!gave_up) {
            const uint32_t reach = (split ? reach_split : scan_reach_all()) | keep;
            if (lane < cb.ng && !((reach >> lane) & 1u)) gsmall[cb.g] = kClsEmpty;
            if (dbg && lane < cb.ng) dbg[cb.g] = ((reach >> lane) & 1u) ? 2 : 1;  // tests: kept / emptied
        } else if (dbg && lane < cb.ng) {
            dbg[cb.g] = 3;  // gave up: kept
        }
        for (int i = lane; i < kMzSlots; i += 64) {  // the table for the next batch
            key[i] = kNone;
            cnt[i] = 0;
        }
        __builtin_amdgcn_wave_barrier();
        have = have_n;
        cb = nb;
    }
}

// rogtk_kmer_path_stats: groups of effective k K on the LDS path (gsmall != 0 after the
// LDS kernels) and on the global path, counted on the device (no G-byte copy to the host)
__global__ __launch_bounds__(kBlock) void k_path_counts(const uint8_t* __restrict__ gk, int K, int64_t G,
                                                        const uint8_t* __restrict__ gsmall,
                                                        const GroupDesc* __restrict__ gdesc,
                                                        unsigned long long* __restrict__ out2) {
    unsigned long long lds = 0, glob = 0, cert = 0, lrows = 0;
    for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < G; g += (int64_t)gridDim.x * kBlock) {
        if (gk[g] != K) continue;
        if (gsmall && gsmall[g]) ++lds;
        else ++glob;
        if (gsmall && gsmall[g] == kClsEmpty) ++cert;
        else if (gsmall && gsmall[g]) lrows += (unsigned long long)gdesc[g].nrows;  // rows the LDS kernels insert
    }
    for (int m = 32; m > 0; m >>= 1) {
        lds += __shfl_xor(lds, m);
        glob += __shfl_xor(glob, m);
        cert += __shfl_xor(cert, m);
        lrows += __shfl_xor(lrows, m);
    }
    // one atomic per workgroup and counter (per wave, 3 x 16K atomics on the same three
    // words serialised at L2: 0.4 ms at 8.17M groups)
    __shared__ unsigned long long s3[kWavesPerBlock][4];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s3[wv][0] = lds;
        s3[wv][1] = glob;
        s3[wv][2] = cert;
        s3[wv][3] = lrows;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned long long v = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) v += s3[w][threadIdx.x];
        if (v) atomicAdd(out2 + threadIdx.x, v);  // out2[2]: of the LDS ones, empty by a certificate
    }
}

// rows of LDS-path groups leave the global path
__global__ __launch_bounds__(kBlock) void k_drop_small_rows(const uint32_t* __restrict__ row_group,
                                                            const uint8_t* __restrict__ gsmall, int64_t n_rows,
                                                            int64_t* __restrict__ row_obs) {
    for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < n_rows; r += (int64_t)gridDim.x * kBlock)
        if (gsmall[row_group[r]]) row_obs[r] = 0;
}

// Per-group capacity: the group's k-mer observations are at most O = sum over its rows
// of max(0, len - 3) (k_eff >= 4), and every valid k-mer takes at least min_cov of them
// (count >= min_cov; the u16 count saturates only above that), so at most
// O / max(min_cov, 1) entries are valid (20x less temporary and output space than O at
// the usual floor of 20, so one call covers 100M reads)
__device__ __host__ __forceinline__ int64_t valid_cap(int64_t obs, int64_t min_cov) {
    return obs / (min_cov > 1 ? min_cov : 1);
}

__global__ __launch_bounds__(kBlock) void k_group_caps(const int64_t* __restrict__ offsets,
                                                       const int64_t* __restrict__ rows,
                                                       const int64_t* __restrict__ go, int64_t G,
                                                       int64_t* __restrict__ caps, int64_t min_cov) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t g = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); g < G; g += waves) {
        int64_t t = 0;
        for (int64_t r = go[g] + lane; r < go[g + 1]; r += 64) {
            const int64_t pr = rows ? rows[r] : r;
            const int64_t len = offsets[pr + 1] - offsets[pr];
            if (len >= 4) t += len - 3;
        }
        for (int m = 32; m > 0; m >>= 1) t += __shfl_xor(t, m);
        if (lane == 0) caps[g] = valid_cap(t, min_cov);
    }
}

// Per-group capacity from the staged rows' observation counts (contiguous per group): at
// most obs / max(min_cov, 1) k-mers of a group are valid (valid_cap). The block path
// computes it here, after staging, instead of by a gather of every row's length first.
__global__ __launch_bounds__(kBlock) void k_group_caps_obs(const int64_t* __restrict__ go, int64_t G,
                                                           const int64_t* __restrict__ row_obs, int64_t min_cov,
                                                           int64_t* __restrict__ caps) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t g = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); g < G; g += waves) {
        int64_t t = 0;
        for (int64_t r = go[g] + lane; r < go[g + 1]; r += 64) t += row_obs[r];
        for (int m = 32; m > 0; m >>= 1) t += __shfl_xor(t, m);
        if (lane == 0) caps[g] = valid_cap(t, min_cov);
    }
}

__global__ void k_tail_sum(const int64_t* __restrict__ pre, const int64_t* __restrict__ vals, int64_t G,
                           int64_t* __restrict__ out_last) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *out_last = G ? pre[G - 1] + vals[G - 1] : 0;
}

__global__ __launch_bounds__(kBlock) void k_group_stats_out(const unsigned long long* __restrict__ gstat,
                                                            const int64_t* __restrict__ gcount, int64_t G, int K,
                                                            int64_t* __restrict__ out) {
    for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < G; g += (int64_t)gridDim.x * kBlock) {
        out[5 * g + 0] = K;
        out[5 * g + 1] = K ? (int64_t)gstat[5 * g + 1] : 0;
        out[5 * g + 2] = gcount[g];
        out[5 * g + 3] = (int64_t)gstat[5 * g + 3];
        out[5 * g + 4] = (int64_t)gstat[5 * g + 4];
    }
}

__global__ __launch_bounds__(kBlock) void k_key_heads(const uint32_t* __restrict__ k, int64_t n,
                                                      uint32_t* __restrict__ head) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        head[i] = (i == 0 || k[i] != k[i - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void k_iota32(uint32_t* __restrict__ out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        out[i] = (uint32_t)i;
}

// the largest key (the radix sort then covers only its significant bits); *mx zeroed before
__global__ __launch_bounds__(kBlock) void k_key_max(const uint32_t* __restrict__ k, int64_t n,
                                                    uint32_t* __restrict__ mx) {
    uint32_t m = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        m = max(m, k[i]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
    __shared__ uint32_t s_m[kWavesPerBlock];  // one atomic per workgroup (not per wave)
    if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kWavesPerBlock; ++w) m = max(m, s_m[w]);
        if (m) atomicMax(mx, m);
    }
}

// the group offsets (an exclusive scan of the heads: a head's group = gid; row i's group =
// gid + head - 1) and the sorted u32 row indices widened to int64
__global__ __launch_bounds__(kBlock) void k_key_offsets_rows(const uint32_t* __restrict__ head,
                                                             const uint32_t* __restrict__ gid,
                                                             const uint32_t* __restrict__ rows32, int64_t n,
                                                             int64_t* __restrict__ go, int64_t* __restrict__ rows) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const uint32_t h = head[i];
        rows[i] = rows32[i];
        if (h) go[gid[i]] = i;
        if (i == n - 1) go[gid[i] + h] = n;
    }
}

int grid_for(int64_t n, int cap = 8192) {
    int64_t g = (n + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

// ---------------------------------------------------------------- host side
int estimate_k_host(const std::vector<int64_t>& lens) {  // fracture.rs:24-54 over the non-null rows
    if (lens.empty()) return 31;
    uint64_t total = 0, count = 0;
    for (int64_t l : lens)
        if (l > 0) {
            total += (uint64_t)l;
            count += 1;
        }
    if (count == 0) return 31;
    const double mean = (double)total / (double)count;
    const int64_t k = (int64_t)std::round(mean / 3.0);
    uint64_t ku = (k % 2 == 0) ? (uint64_t)k - 1 : (uint64_t)k;  // 0 - 1 wraps (release build)
    if (ku < 11) ku = 11;
    if (ku > 63) ku = 63;
    return (int)ku;
}

int effective_k(int k) { return k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : k <= 32 ? 32 : 64; }

struct KmerCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    DevBuf offsets, values, validity, go, gk, cap_off, gstat, gstart, gcount, out_off;
    DevBuf row_group, row_obs, obs_off, row_len, row_words, woff, packed, row_st, raw_len, gdesc;
    DevBuf key_lo, key_hi, ext, grp, idx, perm_a, perm_b, tmp_u64, tmp_u32;
    DevBuf s_lo, s_hi, s_ext, s_grp, head, rid, r_valid, r_first, r_ext, r_cnt, vpos;
    DevBuf v_lo, v_hi, v_grp, v_ext, v_cnt, t_kmer, t_ext, t_cnt, o_kmer, o_ext, o_cnt, cub, gsmall, caps, scal;
    DevBuf long_rows;  // block path: grouped rows longer than the staging stride (an error)
    bool lds_path = true;  // rogtk_kmer_set_path(): tests force the global path
    bool wave_path = true;  // rogtk_kmer_set_path(2): the LDS path without class 2 (tests)
    // the staged k-mers of this call: one word per entry (every group's k_eff <= 32: the
    // high word is 0 and k_pack writes it) or two (a group of k_eff 64 in the call)
    bool lo_only = true;
    int64_t last_lds_groups = 0, last_global_groups = 0;  // rogtk_kmer_path_stats()
    int64_t last_cert_groups = 0;                         // rogtk_kmer_certified_groups()
    int64_t last_lds_rows = 0;                            // rogtk_kmer_lds_rows()
    // the retired allocations of every buffer; a device-wide sync first when there are any
    // (an earlier call's kernels may still read them on another stream; buffers regrow only
    // while the calls' sizes grow, so steady-state calls find nothing to free)
    void reclaim() {
        DevBuf* const all[] = {&offsets, &values, &validity, &go, &gk, &cap_off, &gstat, &gstart, &gcount, &out_off,
                               &row_group, &row_obs, &obs_off, &row_len, &row_words, &woff, &packed, &row_st,
                               &raw_len, &gdesc, &key_lo, &key_hi, &ext, &grp, &idx, &perm_a, &perm_b, &tmp_u64,
                               &tmp_u32, &s_lo, &s_hi, &s_ext, &s_grp, &head, &rid, &r_valid, &r_first, &r_ext,
                               &r_cnt, &vpos, &v_lo, &v_hi, &v_grp, &v_ext, &v_cnt, &t_kmer, &t_ext, &t_cnt,
                               &o_kmer, &o_ext, &o_cnt, &cub, &gsmall, &caps, &scal, &long_rows};
        bool any = false;
        for (DevBuf* b : all) any |= !b->retired.empty();
        if (!any) return;
        (void)hipDeviceSynchronize();
        for (DevBuf* b : all) b->reclaim();
    }
    ~KmerCtx() {
        if (stream) hipStreamDestroy(stream);
    }
};
thread_local std::unique_ptr<KmerCtx> t_kctx;

int kmer_ctx(KmerCtx** out) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_error("no HIP device available (librogtk_hip needs an MI355X / gfx950 GPU)");
        return ROGTK_E_NODEVICE;
    }
    int dev = 0;
    ROGTK_HIP_CHECK(hipGetDevice(&dev));
    if (!t_kctx || t_kctx->device != dev) {
        t_kctx.reset(new KmerCtx());
        t_kctx->device = dev;
        ROGTK_HIP_CHECK(hipStreamCreateWithFlags(&t_kctx->stream, hipStreamNonBlocking));
    }
    *out = t_kctx.get();
    return ROGTK_OK;
}

// hipcub helpers with grow-only temp storage
int cub_exsum_i64(KmerCtx* c, const int64_t* in, int64_t* out, int64_t n, hipStream_t s) {
    size_t bytes = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, (int)n, s));
    if (int rc = c->cub.ensure(bytes)) return rc;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(c->cub.p, bytes, in, out, (int)n, s));
    return ROGTK_OK;
}
int cub_exsum_u32(KmerCtx* c, const uint32_t* in, uint32_t* out, int64_t n, hipStream_t s) {
    size_t bytes = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, (int)n, s));
    if (int rc = c->cub.ensure(bytes)) return rc;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(c->cub.p, bytes, in, out, (int)n, s));
    return ROGTK_OK;
}
template <class K>
int cub_sort(KmerCtx* c, const K* kin, K* kout, const uint32_t* vin, uint32_t* vout, int64_t n, int end_bit,
             hipStream_t s) {
    size_t bytes = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, kin, kout, vin, vout, (int)n, 0, end_bit, s));
    if (int rc = c->cub.ensure(bytes)) return rc;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(c->cub.p, bytes, kin, kout, vin, vout, (int)n, 0, end_bit, s));
    return ROGTK_OK;
}

int bits_for(uint64_t v) {
    int b = 1;
    while (b < 64 && (v >> b)) ++b;
    return b;
}

// Inputs / per-group outputs of one spectrum call (device pointers). Offsets are
// int64; rows (optional) maps grouped row r to its physical row.
struct KIn {
    const int64_t* offsets;
    const uint8_t* values;
    const uint8_t* validity;
    int64_t voff;
    const int64_t* rows;
    const int64_t* go;
    const uint8_t* gk;
    const int64_t* cap_off;
    unsigned long long* gstat;  // G x 5
    int64_t* gcount;            // G
    const uint64_t* blocks = nullptr;  // the column as B-word 2-bit blocks (k_pack_reads), or NULL
    int B = 0;                         // words per block
    int S = 0;                         // 2-bit words per row to stage: ceil(max_len / 32) <= B - 1
    int64_t* cap_fill = nullptr;       // != NULL: per-group capacities computed here (into this
                                       // scratch, then cap_off) from the staged rows' observations
    bool fused = false;                // stage from the ASCII bytes by k_pack_gather (S words per row)
    int64_t vlen = 0;                  // fused: readable bytes of values
};

template <int OW, bool WIDE>
int run_class(KmerCtx* c, const KIn& in, int64_t n_rows, int64_t G, int K, int64_t min_cov, hipStream_t s,
              const std::vector<uint8_t>* gk_host) {
    const int64_t* go = in.go;
    unsigned long long* gstat = in.gstat;
    if (int rc = c->row_group.ensure(n_rows * 4)) return rc;
    if (int rc = c->row_obs.ensure(n_rows * 8)) return rc;
    if (int rc = c->row_len.ensure(n_rows * 4)) return rc;
    if (int rc = c->row_words.ensure(n_rows * 8)) return rc;
    if (int rc = c->woff.ensure(n_rows * 8)) return rc;
    if (int rc = c->row_st.ensure(n_rows * 8)) return rc;
    if (int rc = c->raw_len.ensure(n_rows * 4)) return rc;
    if (int rc = c->obs_off.ensure(n_rows * 8)) return rc;
    const int wgrid = grid_for((n_rows + kWavesPerBlock - 1) / kWavesPerBlock * kBlock, 16384);
    hipLaunchKernelGGL(k_row_groups, dim3(grid_for(G * 16, 16384)), dim3(kBlock), 0, s, go, G,
                       c->row_group.as<uint32_t>());
    const int stride = (in.blocks || in.fused) ? in.S : 0;  // staged words per row (0: compact, woff)
    if (in.fused) {
        // round 5: packed from the ASCII bytes in group order (k_pack_gather), no block column
        if (int rc = c->packed.ensure((size_t)std::max<int64_t>(n_rows * stride, 1) * 8)) return rc;
        ProfScope prof(K_PACK_GATHER, s, true);
        const int pgrid = (int)std::min<int64_t>((n_rows + 63) / 64, (int64_t)8192 * 256 / 64);
#define ROGTK_PG(NW)                                                                                              \
    hipExtLaunchKernelGGL(k_pack_gather<NW>, dim3(pgrid), dim3(64), 0, s, prof.start(), prof.stop(), 0, in.offsets,  \
                          in.values, in.validity, in.voff, in.vlen, in.rows, n_rows, K, stride, in.gk,                \
                          c->row_group.as<uint32_t>(), c->packed.as<uint64_t>(), c->row_obs.as<int64_t>(),            \
                          c->row_len.as<int32_t>(), gstat, c->long_rows.as<unsigned long long>())
        if (stride <= 5) ROGTK_PG(5);
        else ROGTK_PG(7);
#undef ROGTK_PG
    } else if (in.blocks) {
        // stage from the packed column: each grouped row's block as whole lines, its bases
        // at a fixed stride (row r at packed[r * S]: no offsets, no scan)
        if (int rc = c->packed.ensure((size_t)std::max<int64_t>(n_rows * stride, 1) * 8)) return rc;
        const int ggrid = grid_for((n_rows + 63) / 64 * 64 / kWavesPerBlock, 16384);
        ProfScope prof(K_ROW_GATHER, s, true);
#define ROGTK_GATHER(BW)                                                                                       \
    hipExtLaunchKernelGGL(k_row_gather<BW>, dim3(ggrid), dim3(kBlock), 0, s, prof.start(), prof.stop(), 0,      \
                       in.blocks, in.rows, n_rows, K, stride, in.gk, c->row_group.as<uint32_t>(), c->packed.as<uint64_t>(), c->row_obs.as<int64_t>(),  \
                       c->row_len.as<int32_t>(), gstat, c->long_rows.as<unsigned long long>())
        if (in.B == 8) ROGTK_GATHER(8);
        else if (in.B == 16) ROGTK_GATHER(16);
        else ROGTK_GATHER(32);
#undef ROGTK_GATHER
    } else {
        // stage: row spans -> word offsets -> one pass over the bytes (check + pack + counts)
        hipLaunchKernelGGL((k_row_meta<OW>), dim3(grid_for(n_rows)), dim3(kBlock), 0, s, in.offsets, in.validity,
                           in.voff, in.rows, n_rows, in.gk, K, c->row_group.as<uint32_t>(), c->row_st.as<int64_t>(),
                           c->raw_len.as<int32_t>(), c->row_words.as<int64_t>());
        if (int rc = cub_exsum_i64(c, c->row_words.as<int64_t>(), c->woff.as<int64_t>(), n_rows, s)) return rc;
        {
            int64_t wl[2] = {0, 0};
            ROGTK_HIP_CHECK(hipMemcpyAsync(&wl[0], c->woff.as<int64_t>() + n_rows - 1, 8, hipMemcpyDeviceToHost, s));
            ROGTK_HIP_CHECK(
                hipMemcpyAsync(&wl[1], c->row_words.as<int64_t>() + n_rows - 1, 8, hipMemcpyDeviceToHost, s));
            ROGTK_HIP_CHECK(hipStreamSynchronize(s));
            if (int rc = c->packed.ensure((size_t)std::max<int64_t>(wl[0] + wl[1], 1) * 8)) return rc;
        }
        hipLaunchKernelGGL(k_row_stage, dim3(wgrid), dim3(kBlock), 0, s, in.values, n_rows, K,
                           c->row_group.as<uint32_t>(), c->row_st.as<int64_t>(), c->raw_len.as<int32_t>(),
                           c->woff.as<int64_t>(), c->packed.as<uint64_t>(), c->row_obs.as<int64_t>(),
                           c->row_len.as<int32_t>(), gstat);
    }
    ROGTK_HIP_CHECK(hipGetLastError());
    const bool lds = c->lds_path && K <= 32;
    if (lds) {
        // size classes (and, on the block path, the capacities from the staged rows)
        if (int rc = c->gsmall.ensure((size_t)G)) return rc;
        if (int rc = c->gdesc.ensure((size_t)G * sizeof(GroupDesc))) return rc;
        hipLaunchKernelGGL(k_group_classify, dim3(grid_for(G * kClsLanes, 16384)), dim3(kBlock), 0, s, go, G, in.gk,
                           K, c->row_obs.as<int64_t>(), c->row_words.as<int64_t>(), c->woff.as<int64_t>(), stride,
                           c->gsmall.as<uint8_t>(), c->gdesc.as<GroupDesc>(), in.cap_fill, min_cov,
                           stride && kmer_cert_on() ? gstat : nullptr, (int)(c->wave_path && K <= 16));
    } else if (in.cap_fill) {
        hipLaunchKernelGGL(k_group_caps_obs, dim3(grid_for(G * 64, 16384)), dim3(kBlock), 0, s, go, G,
                           c->row_obs.as<int64_t>(), min_cov, in.cap_fill);
    }
    if (in.cap_fill) {  // capacity offsets from the staged observation counts (before any output)
        int64_t* co = const_cast<int64_t*>(in.cap_off);
        if (int rc = cub_exsum_i64(c, in.cap_fill, co, G, s)) return rc;
        hipLaunchKernelGGL(k_tail_sum, dim3(1), dim3(64), 0, s, co, in.cap_fill, G, co + G);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    if (lds && stride && gstat && kmer_cert_on() && kmer_mz_on() && (K == 31 || K == 32) && min_cov >= 2) {
        ProfScope prof(K_KMER_MZ, s, true);
        const int64_t chunks = (G + 63) / 64;
        hipExtLaunchKernelGGL(k_minimizer_filter, dim3((unsigned)std::min<int64_t>((chunks + kMzWaves - 1) / kMzWaves, 4096)),
                              dim3(64 * kMzWaves), 0, s, prof.start(), prof.stop(), 0, c->gdesc.as<GroupDesc>(), G,
                              c->gsmall.as<uint8_t>(), K, min_cov, c->row_len.as<int32_t>(), stride,
                              c->packed.as<uint64_t>(), gstat, g_mz_debug_groups >= G ? g_mz_debug : nullptr);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    if (lds && c->wave_path && K <= 16) {
        // classes 2 and 6 first: their overflowing groups become class 3 for the launch below
        const int64_t chunks = (G + 63) / 64;
        ROGTK_TIMED_LAUNCH(K_KMER_WAVE, k_kmer_wave<1024>,
                           dim3((unsigned)std::min<int64_t>((chunks + WaveCfg<1024>::kWG - 1) / WaveCfg<1024>::kWG, 65536)),
                           dim3(64 * WaveCfg<1024>::kWG), 0, s, c->gdesc.as<GroupDesc>(), G, c->gsmall.as<uint8_t>(), K,
                           min_cov, c->row_len.as<int32_t>(), c->woff.as<int64_t>(), stride, c->packed.as<uint64_t>(),
                           in.cap_off, c->t_kmer.as<uint64_t>(), c->t_ext.as<uint8_t>(), c->t_cnt.as<uint16_t>(),
                           in.gcount, gstat, c->lo_only ? 1 : 0);
        ROGTK_TIMED_LAUNCH(K_KMER_WAVE, k_kmer_wave<2048>, dim3((unsigned)std::min<int64_t>(chunks, 16384)),
                           dim3(64 * WaveCfg<2048>::kWG), 0, s, c->gdesc.as<GroupDesc>(), G, c->gsmall.as<uint8_t>(), K,
                           min_cov, c->row_len.as<int32_t>(), c->woff.as<int64_t>(), stride, c->packed.as<uint64_t>(),
                           in.cap_off, c->t_kmer.as<uint64_t>(), c->t_ext.as<uint8_t>(), c->t_cnt.as<uint16_t>(),
                           in.gcount, gstat, c->lo_only ? 1 : 0);
    }
    if (lds) {
        ProfScope prof(K_KMER_LDS, s, true);
        hipExtLaunchKernelGGL((k_kmer_lds<3, kLdsBlock>), dim3((unsigned)std::min<int64_t>((G + 63) / 64, 65536)),
                              dim3(kLdsBlock), 0, s, prof.start(), prof.stop(), 0, c->gdesc.as<GroupDesc>(), G,
                              c->gsmall.as<uint8_t>(), K, min_cov, c->row_len.as<int32_t>(),
                              c->woff.as<int64_t>(), stride, c->packed.as<uint64_t>(), in.cap_off, c->t_kmer.as<uint64_t>(),
                              c->t_ext.as<uint8_t>(), c->t_cnt.as<uint16_t>(), in.gcount, gstat, c->lo_only ? 1 : 0);
    }
    if (lds) {
        // one workgroup per small group, straight from the packed rows
        ROGTK_TIMED_LAUNCH(K_KMER_LDS, (k_kmer_lds<1, kLdsBlock>), dim3((unsigned)std::min<int64_t>((G + 63) / 64, 65536)), dim3(kLdsBlock), 0, s,
                           c->gdesc.as<GroupDesc>(), G,
                           c->gsmall.as<uint8_t>(), K, min_cov, c->row_len.as<int32_t>(),
                           c->woff.as<int64_t>(), stride, c->packed.as<uint64_t>(), in.cap_off, c->t_kmer.as<uint64_t>(),
                           c->t_ext.as<uint8_t>(), c->t_cnt.as<uint16_t>(), in.gcount, gstat, c->lo_only ? 1 : 0);
        ROGTK_TIMED_LAUNCH(K_KMER_LDS, (k_kmer_lds<4, kLdsBlock>), dim3((unsigned)std::min<int64_t>((G + 63) / 64, 8192)), dim3(kLdsBlock), 0, s,
                           c->gdesc.as<GroupDesc>(), G,
                           c->gsmall.as<uint8_t>(), K, min_cov, c->row_len.as<int32_t>(),
                           c->woff.as<int64_t>(), stride, c->packed.as<uint64_t>(), in.cap_off, c->t_kmer.as<uint64_t>(),
                           c->t_ext.as<uint8_t>(), c->t_cnt.as<uint16_t>(), in.gcount, gstat, c->lo_only ? 1 : 0);
    }
    // the groups per path first: with none on the global path (the usual C3 call, every
    // group in LDS or certified empty) its row drop and observation scan are skipped
    if (int rc = c->scal.ensure(64)) return rc;
    ROGTK_HIP_CHECK(hipMemsetAsync(c->scal.p, 0, 32, s));
    hipLaunchKernelGGL(k_path_counts, dim3(grid_for(G, 1024)), dim3(kBlock), 0, s, in.gk, K, G,
                       (c->lds_path && K <= 32) ? c->gsmall.as<uint8_t>() : nullptr,
                       (c->lds_path && K <= 32) ? c->gdesc.as<GroupDesc>() : nullptr,
                       c->scal.as<unsigned long long>());
    int64_t last[6] = {0, 0, 0, 0, 0, 0};
    ROGTK_HIP_CHECK(hipMemcpyAsync(&last[2], c->scal.p, 32, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    c->reclaim();
    c->last_lds_groups += last[2];
    c->last_global_groups += last[3];
    c->last_cert_groups += last[4];
    c->last_lds_rows += last[5];
    if (last[3] == 0) return ROGTK_OK;
    if (lds) {
        hipLaunchKernelGGL(k_drop_small_rows, dim3(grid_for(n_rows)), dim3(kBlock), 0, s, c->row_group.as<uint32_t>(),
                           c->gsmall.as<uint8_t>(), n_rows, c->row_obs.as<int64_t>());
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    if (int rc = cub_exsum_i64(c, c->row_obs.as<int64_t>(), c->obs_off.as<int64_t>(), n_rows, s)) return rc;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&last[0], c->obs_off.as<int64_t>() + n_rows - 1, 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(&last[1], c->row_obs.as<int64_t>() + n_rows - 1, 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    const int64_t T = last[0] + last[1];
    if (T == 0) return ROGTK_OK;
    ROGTK_REQUIRE(T <= kMaxObsPerLaunch, ROGTK_E_UNSUPPORTED,
                  "kmer: %lld k-mer observations in one call (max %lld); split the groups over calls",
                  (long long)T, (long long)kMaxObsPerLaunch);
    for (DevBuf* b : {&c->key_lo, &c->key_hi, &c->tmp_u64, &c->s_lo, &c->s_hi, &c->v_lo, &c->v_hi})
        if (int rc = b->ensure((size_t)T * 8)) return rc;
    for (DevBuf* b : {&c->grp, &c->idx, &c->perm_a, &c->perm_b, &c->tmp_u32, &c->s_grp, &c->head, &c->rid,
                      &c->r_valid, &c->r_first, &c->vpos, &c->v_grp})
        if (int rc = b->ensure((size_t)T * 4)) return rc;
    for (DevBuf* b : {&c->ext, &c->s_ext, &c->r_ext, &c->v_ext})
        if (int rc = b->ensure((size_t)T)) return rc;
    for (DevBuf* b : {&c->r_cnt, &c->v_cnt})
        if (int rc = b->ensure((size_t)T * 2)) return rc;

    hipLaunchKernelGGL((k_kmer_emit<OW, WIDE>), dim3(wgrid), dim3(kBlock), 0, s, in.offsets, in.values, in.rows,
                       n_rows, K, c->row_group.as<uint32_t>(), c->row_obs.as<int64_t>(),
                       c->obs_off.as<int64_t>(), c->key_lo.as<uint64_t>(), c->key_hi.as<uint64_t>(),
                       c->ext.as<uint8_t>(), c->grp.as<uint32_t>(), c->idx.as<uint32_t>());
    ROGTK_HIP_CHECK(hipGetLastError());
    // LSD: key lo, [key hi], group (hipcub radix sort is stable)
    const int g = grid_for(T);
    const int lo_bits = WIDE ? 64 : 2 * K;
    if (int rc = cub_sort<uint64_t>(c, c->key_lo.as<uint64_t>(), c->tmp_u64.as<uint64_t>(), c->idx.as<uint32_t>(),
                                    c->perm_a.as<uint32_t>(), T, lo_bits, s))
        return rc;
    uint32_t* perm = c->perm_a.as<uint32_t>();
    uint32_t* other = c->perm_b.as<uint32_t>();
    if (WIDE) {
        hipLaunchKernelGGL(k_gather<uint64_t>, dim3(g), dim3(kBlock), 0, s, c->key_hi.as<uint64_t>(), perm, T,
                           c->s_hi.as<uint64_t>());
        if (int rc = cub_sort<uint64_t>(c, c->s_hi.as<uint64_t>(), c->tmp_u64.as<uint64_t>(), perm, other, T, 64, s))
            return rc;
        std::swap(perm, other);
    }
    if (G > 1) {
        hipLaunchKernelGGL(k_gather<uint32_t>, dim3(g), dim3(kBlock), 0, s, c->grp.as<uint32_t>(), perm, T,
                           c->s_grp.as<uint32_t>());
        if (int rc = cub_sort<uint32_t>(c, c->s_grp.as<uint32_t>(), c->tmp_u32.as<uint32_t>(), perm, other, T,
                                        bits_for((uint64_t)G - 1), s))
            return rc;
        std::swap(perm, other);
    }
    hipLaunchKernelGGL(k_gather<uint64_t>, dim3(g), dim3(kBlock), 0, s, c->key_lo.as<uint64_t>(), perm, T,
                       c->s_lo.as<uint64_t>());
    if (WIDE)
        hipLaunchKernelGGL(k_gather<uint64_t>, dim3(g), dim3(kBlock), 0, s, c->key_hi.as<uint64_t>(), perm, T,
                           c->s_hi.as<uint64_t>());
    hipLaunchKernelGGL(k_gather<uint8_t>, dim3(g), dim3(kBlock), 0, s, c->ext.as<uint8_t>(), perm, T,
                       c->s_ext.as<uint8_t>());
    hipLaunchKernelGGL(k_gather<uint32_t>, dim3(g), dim3(kBlock), 0, s, c->grp.as<uint32_t>(), perm, T,
                       c->s_grp.as<uint32_t>());
    ROGTK_HIP_CHECK(hipGetLastError());
    // runs + CountFilter
    hipLaunchKernelGGL((k_heads<WIDE>), dim3(g), dim3(kBlock), 0, s, c->s_lo.as<uint64_t>(), c->s_hi.as<uint64_t>(),
                       c->s_grp.as<uint32_t>(), T, c->head.as<uint32_t>());
    if (int rc = cub_exsum_u32(c, c->head.as<uint32_t>(), c->rid.as<uint32_t>(), T, s)) return rc;
    uint32_t lastu[2] = {0, 0};
    ROGTK_HIP_CHECK(hipMemcpyAsync(&lastu[0], c->rid.as<uint32_t>() + T - 1, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(&lastu[1], c->head.as<uint32_t>() + T - 1, 4, hipMemcpyDeviceToHost, s));
    hipLaunchKernelGGL((k_runs<WIDE>), dim3(g), dim3(kBlock), 0, s, c->s_lo.as<uint64_t>(), c->s_hi.as<uint64_t>(),
                       c->s_grp.as<uint32_t>(), c->s_ext.as<uint8_t>(), c->head.as<uint32_t>(),
                       c->rid.as<uint32_t>(), T, min_cov, c->r_valid.as<uint32_t>(), c->r_first.as<uint32_t>(),
                       c->r_ext.as<uint8_t>(), c->r_cnt.as<uint16_t>());
    ROGTK_HIP_CHECK(hipGetLastError());
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    const int64_t n_runs = (int64_t)lastu[0] + lastu[1];
    if (int rc = cub_exsum_u32(c, c->r_valid.as<uint32_t>(), c->vpos.as<uint32_t>(), n_runs, s)) return rc;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&lastu[0], c->vpos.as<uint32_t>() + n_runs - 1, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(&lastu[1], c->r_valid.as<uint32_t>() + n_runs - 1, 4, hipMemcpyDeviceToHost, s));
    const int gr = grid_for(n_runs);
    hipLaunchKernelGGL((k_compact_valid<WIDE>), dim3(gr), dim3(kBlock), 0, s, c->r_valid.as<uint32_t>(),
                       c->vpos.as<uint32_t>(), c->r_first.as<uint32_t>(), c->r_ext.as<uint8_t>(),
                       c->r_cnt.as<uint16_t>(), n_runs, c->s_lo.as<uint64_t>(), c->s_hi.as<uint64_t>(),
                       c->s_grp.as<uint32_t>(), c->v_lo.as<uint64_t>(), c->v_hi.as<uint64_t>(),
                       c->v_grp.as<uint32_t>(), c->v_ext.as<uint8_t>(), c->v_cnt.as<uint16_t>());
    ROGTK_HIP_CHECK(hipGetLastError());
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    const int64_t nv = (int64_t)lastu[0] + lastu[1];
    if (nv == 0) return ROGTK_OK;
    const int gv = grid_for(nv);
    hipLaunchKernelGGL(k_group_ranges, dim3(gv), dim3(kBlock), 0, s, c->v_grp.as<uint32_t>(), nv,
                       c->gstart.as<int64_t>(), in.gcount);
    hipLaunchKernelGGL(k_group_counts, dim3(grid_for(G)), dim3(kBlock), 0, s, in.gk, K, G,
                       (c->lds_path && K <= 32) ? c->gsmall.as<uint8_t>() : nullptr, c->gstart.as<int64_t>(),
                       in.gcount);
    hipLaunchKernelGGL((k_censor<WIDE>), dim3(gv), dim3(kBlock), 0, s, c->v_lo.as<uint64_t>(),
                       c->v_hi.as<uint64_t>(), c->v_grp.as<uint32_t>(), c->v_ext.as<uint8_t>(),
                       c->v_cnt.as<uint16_t>(), nv, K, c->gstart.as<int64_t>(), in.gcount,
                       in.cap_off, c->t_kmer.as<uint64_t>(), c->t_ext.as<uint8_t>(),
                       c->t_cnt.as<uint16_t>(), gstat, c->lo_only ? 1 : 0);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

template <int OW>
int run_any(KmerCtx* c, const KIn& in, int64_t n_rows, int64_t G, int K, int64_t min_cov, hipStream_t s,
            const std::vector<uint8_t>* gk) {
    return K == 64 ? run_class<OW, true>(c, in, n_rows, G, K, min_cov, s, gk)
                   : run_class<OW, false>(c, in, n_rows, G, K, min_cov, s, gk);
}

}  // namespace
}  // namespace rogtk

using namespace rogtk;

extern "C" {

int rogtk_kmer_set_path(int lds_small_groups) {
    KmerCtx* c = nullptr;
    if (int rc = kmer_ctx(&c)) return rc;
    c->lds_path = lds_small_groups != 0;
    c->wave_path = lds_small_groups == 1;
    return ROGTK_OK;
}

int rogtk_kmer_set_filter(int minimizer_filter) {
    g_kmer_mz.store(minimizer_filter ? 1 : 0, std::memory_order_relaxed);
    return ROGTK_OK;
}

#ifdef ROGTK_KMER_TIMING
// experiment builds only: reads and clears the per-phase clocks (100 MHz ticks summed over workgroups)
extern "C" int rogtk_kmer_timing(unsigned long long* out8) {
    hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_kmer_clk), 8 * sizeof(unsigned long long));
    unsigned long long z[8] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_kmer_clk), z, sizeof(z));
    return ROGTK_OK;
}
#endif

int rogtk_kmer_certified_groups(int64_t* out) {
    ROGTK_REQUIRE(out, ROGTK_E_INVALID, "kmer_certified_groups: NULL");
    KmerCtx* c = nullptr;
    if (int rc = kmer_ctx(&c)) return rc;
    *out = c->last_cert_groups;
    return ROGTK_OK;
}

int rogtk_kmer_lds_rows(int64_t* out) {
    ROGTK_REQUIRE(out, ROGTK_E_INVALID, "kmer_lds_rows: NULL");
    KmerCtx* c = nullptr;
    if (int rc = kmer_ctx(&c)) return rc;
    *out = c->last_lds_rows;
    return ROGTK_OK;
}

int rogtk_kmer_debug_filter(uint8_t* decisions, int64_t n_groups) {
    ROGTK_REQUIRE(!decisions == !n_groups && n_groups >= 0, ROGTK_E_INVALID, "kmer_debug_filter: buffer and size");
    g_mz_debug = decisions;
    g_mz_debug_groups = n_groups;
    return ROGTK_OK;
}

int rogtk_kmer_path_stats(int64_t* out2) {
    ROGTK_REQUIRE(out2, ROGTK_E_INVALID, "kmer_path_stats: NULL");
    KmerCtx* c = nullptr;
    if (int rc = kmer_ctx(&c)) return rc;
    out2[0] = c->last_lds_groups;
    out2[1] = c->last_global_groups;
    return ROGTK_OK;
}

int rogtk_kmer_capacity(const void* offsets, int offset_width, int64_t n_rows, int64_t* capacity) {
    ROGTK_REQUIRE(capacity && (n_rows == 0 || offsets), ROGTK_E_INVALID, "kmer_capacity: NULL argument");
    ROGTK_REQUIRE(offset_width == 4 || offset_width == 8, ROGTK_E_INVALID, "offset_width must be 4 or 8");
    int64_t t = 0;
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t len = offset_width == 4
                                ? (int64_t)((const int32_t*)offsets)[r + 1] - ((const int32_t*)offsets)[r]
                                : ((const int64_t*)offsets)[r + 1] - ((const int64_t*)offsets)[r];
        if (len >= 4) t += len - 3;
    }
    *capacity = t;
    return ROGTK_OK;
}

int rogtk_kmer_spectrum_host(const void* offsets, int offset_width, const uint8_t* values, int64_t values_len,
                             const uint8_t* validity, int64_t validity_offset, int64_t n_rows,
                             const int64_t* group_offsets, int64_t n_groups, int k, int auto_k,
                             int64_t min_coverage, int64_t capacity, uint64_t* kmers, uint8_t* exts,
                             uint16_t* counts, int64_t* entry_offsets, int64_t* group_stats) {
    ROGTK_REQUIRE(offset_width == 4 || offset_width == 8, ROGTK_E_INVALID, "offset_width must be 4 or 8");
    ROGTK_REQUIRE(n_rows >= 0 && (n_rows == 0 || offsets), ROGTK_E_INVALID, "kmer: bad offsets / n_rows");
    ROGTK_REQUIRE(values_len >= 0 && (values_len == 0 || values), ROGTK_E_INVALID, "kmer: bad values");
    ROGTK_REQUIRE(entry_offsets && group_stats, ROGTK_E_INVALID, "kmer: entry_offsets / group_stats are NULL");
    ROGTK_REQUIRE(capacity >= 0 && (capacity == 0 || (kmers && exts && counts)), ROGTK_E_INVALID,
                  "kmer: output arrays are NULL");
    ROGTK_REQUIRE(min_coverage >= 0, ROGTK_E_INVALID, "kmer: min_coverage must be >= 0");
    // groups: contiguous row ranges covering [0, n_rows)
    std::vector<int64_t> go;
    if (group_offsets && n_groups > 0) {
        go.assign(group_offsets, group_offsets + n_groups + 1);
        ROGTK_REQUIRE(go.front() == 0 && go.back() == n_rows, ROGTK_E_INVALID,
                      "kmer: group_offsets must start at 0 and end at n_rows");
        for (int64_t g = 0; g < n_groups; ++g)
            ROGTK_REQUIRE(go[g] <= go[g + 1], ROGTK_E_INVALID, "kmer: group_offsets must be non-decreasing");
    } else {
        go = {0, n_rows};
    }
    const int64_t G = (int64_t)go.size() - 1;
    ROGTK_REQUIRE(G < (int64_t)0xFFFFFFFF, ROGTK_E_UNSUPPORTED, "kmer: too many groups");
    auto row_len = [&](int64_t r) -> int64_t {
        return offset_width == 4 ? (int64_t)((const int32_t*)offsets)[r + 1] - ((const int32_t*)offsets)[r]
                                 : ((const int64_t*)offsets)[r + 1] - ((const int64_t*)offsets)[r];
    };
    auto row_ok = [&](int64_t r) -> bool {
        if (!validity) return true;
        const int64_t b = validity_offset + r;
        return (validity[b >> 3] >> (b & 7)) & 1;
    };
    // per-group effective k (0 = no output: k > 64), capacity offsets
    std::vector<uint8_t> gk(G);
    std::vector<int64_t> cap_off(G + 1, 0);
    bool present[65] = {false};
    for (int64_t g = 0; g < G; ++g) {
        int kg = k;
        if (auto_k) {
            std::vector<int64_t> lens;
            for (int64_t r = go[g]; r < go[g + 1]; ++r)
                if (row_ok(r)) lens.push_back(row_len(r));
            kg = estimate_k_host(lens);
        }
        gk[g] = (uint8_t)(kg > 64 ? 0 : effective_k(kg));
        if (gk[g]) present[gk[g]] = true;
        int64_t cap = 0;
        for (int64_t r = go[g]; r < go[g + 1]; ++r) {
            const int64_t len = row_len(r);
            if (len >= 4) cap += len - 3;
        }
        cap_off[g + 1] = cap_off[g] + valid_cap(cap, min_coverage);
    }
    KmerCtx* c = nullptr;
    if (int rc = kmer_ctx(&c)) return rc;
    hipStream_t s = c->stream;
    // normalise offsets to start at 0 so only the referenced values travel
    const int64_t base = n_rows ? (offset_width == 4 ? ((const int32_t*)offsets)[0] : ((const int64_t*)offsets)[0]) : 0;
    const int64_t vend = n_rows ? (offset_width == 4 ? ((const int32_t*)offsets)[n_rows] : ((const int64_t*)offsets)[n_rows]) : 0;
    ROGTK_REQUIRE(vend <= values_len, ROGTK_E_INVALID, "kmer: offsets exceed values_len");
    std::vector<int64_t> offs(n_rows + 1);
    for (int64_t r = 0; r <= n_rows; ++r)
        offs[r] = (offset_width == 4 ? (int64_t)((const int32_t*)offsets)[r] : ((const int64_t*)offsets)[r]) - base;
    std::vector<uint8_t> vbits;
    if (validity) {
        vbits.assign((size_t)(n_rows + 7) / 8, 0);
        for (int64_t r = 0; r < n_rows; ++r)
            if (row_ok(r)) vbits[r >> 3] |= (uint8_t)(1u << (r & 7));
    }
    if (int rc = c->offsets.ensure((size_t)(n_rows + 1) * 8)) return rc;
    if (int rc = c->values.ensure((size_t)std::max<int64_t>(vend - base, 1))) return rc;
    if (int rc = c->go.ensure((size_t)(G + 1) * 8)) return rc;
    if (int rc = c->gk.ensure((size_t)G)) return rc;
    if (int rc = c->cap_off.ensure((size_t)(G + 1) * 8)) return rc;
    if (int rc = c->gstat.ensure((size_t)G * 5 * 8)) return rc;
    if (int rc = c->gstart.ensure((size_t)G * 8)) return rc;
    if (int rc = c->gcount.ensure((size_t)G * 8)) return rc;
    if (int rc = c->out_off.ensure((size_t)(G + 1) * 8)) return rc;
    const int64_t tcap = std::max<int64_t>(cap_off[G], 1);
    if (int rc = c->t_kmer.ensure((size_t)tcap * 16)) return rc;
    if (int rc = c->t_ext.ensure((size_t)tcap)) return rc;
    if (int rc = c->t_cnt.ensure((size_t)tcap * 2)) return rc;
    if (validity) {
        if (int rc = c->validity.ensure(vbits.size())) return rc;
    }
    ROGTK_HIP_CHECK(hipMemcpyAsync(c->offsets.p, offs.data(), (n_rows + 1) * 8, hipMemcpyHostToDevice, s));
    if (vend > base)
        ROGTK_HIP_CHECK(hipMemcpyAsync(c->values.p, values + base, vend - base, hipMemcpyHostToDevice, s));
    if (validity)
        ROGTK_HIP_CHECK(hipMemcpyAsync(c->validity.p, vbits.data(), vbits.size(), hipMemcpyHostToDevice, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(c->go.p, go.data(), (G + 1) * 8, hipMemcpyHostToDevice, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(c->gk.p, gk.data(), G, hipMemcpyHostToDevice, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(c->cap_off.p, cap_off.data(), (G + 1) * 8, hipMemcpyHostToDevice, s));
    ROGTK_HIP_CHECK(hipMemsetAsync(c->gstat.p, 0, G * 5 * 8, s));
    ROGTK_HIP_CHECK(hipMemsetAsync(c->gcount.p, 0, G * 8, s));
    c->last_lds_groups = c->last_global_groups = c->last_cert_groups = c->last_lds_rows = 0;
    const KIn in{c->offsets.as<int64_t>(), c->values.as<uint8_t>(), validity ? c->validity.as<uint8_t>() : nullptr,
                 0, nullptr, c->go.as<int64_t>(), c->gk.as<uint8_t>(), c->cap_off.as<int64_t>(),
                 c->gstat.as<unsigned long long>(), c->gcount.as<int64_t>()};
    c->lo_only = !present[64];
    for (int K : {4, 8, 16, 32, 64}) {
        if (!present[K] || n_rows == 0) continue;
        if (int rc = run_any<8>(c, in, n_rows, G, K, min_coverage, s, &gk)) return rc;
    }
    // dense packing by group
    std::vector<int64_t> gcount(G);
    ROGTK_HIP_CHECK(hipMemcpyAsync(gcount.data(), c->gcount.p, G * 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    entry_offsets[0] = 0;
    for (int64_t g = 0; g < G; ++g) entry_offsets[g + 1] = entry_offsets[g] + gcount[g];
    const int64_t total = entry_offsets[G];
    ROGTK_REQUIRE(total <= capacity, ROGTK_E_OVERFLOW, "kmer: %lld entries exceed capacity %lld",
                  (long long)total, (long long)capacity);
    if (total > 0) {
        if (int rc = c->o_kmer.ensure((size_t)total * 16)) return rc;
        if (int rc = c->o_ext.ensure((size_t)total)) return rc;
        if (int rc = c->o_cnt.ensure((size_t)total * 2)) return rc;
        ROGTK_HIP_CHECK(hipMemcpyAsync(c->out_off.p, entry_offsets, (G + 1) * 8, hipMemcpyHostToDevice, s));
        auto pack = c->lo_only ? k_pack<true, true> : k_pack<true, false>;
        hipLaunchKernelGGL(pack, dim3(grid_for(G * 64, 16384)), dim3(kBlock), 0, s, c->t_kmer.as<uint64_t>(),
                           c->t_ext.as<uint8_t>(), c->t_cnt.as<uint16_t>(), G, c->cap_off.as<int64_t>(),
                           c->gcount.as<int64_t>(), c->out_off.as<int64_t>(), c->o_kmer.as<uint64_t>(),
                           c->o_ext.as<uint8_t>(), c->o_cnt.as<uint16_t>());
        ROGTK_HIP_CHECK(hipGetLastError());
        ROGTK_HIP_CHECK(hipMemcpyAsync(kmers, c->o_kmer.p, total * 16, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipMemcpyAsync(exts, c->o_ext.p, total, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipMemcpyAsync(counts, c->o_cnt.p, total * 2, hipMemcpyDeviceToHost, s));
    }
    std::vector<unsigned long long> st((size_t)G * 5);
    ROGTK_HIP_CHECK(hipMemcpyAsync(st.data(), c->gstat.p, G * 5 * 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    for (int64_t g = 0; g < G; ++g) {
        group_stats[5 * g + 0] = gk[g];
        group_stats[5 * g + 1] = (int64_t)st[5 * g + 1];
        group_stats[5 * g + 2] = gcount[g];
        group_stats[5 * g + 3] = (int64_t)st[5 * g + 3];
        group_stats[5 * g + 4] = (int64_t)st[5 * g + 4];
    }
    return ROGTK_OK;
}

int rogtk_group_by_key(const uint32_t* keys, int64_t n, int64_t* rows_out, int64_t* group_offsets_out,
                       int64_t* n_groups, void* stream) {
    ROGTK_REQUIRE(n_groups && (n == 0 || (keys && rows_out && group_offsets_out)), ROGTK_E_INVALID,
                  "group_by_key: NULL argument");
    ROGTK_REQUIRE(n >= 0 && n < (int64_t)0x7FFFFFFF, ROGTK_E_UNSUPPORTED, "group_by_key: n must be < 2^31");
    *n_groups = 0;
    if (n == 0) return ROGTK_OK;
    KmerCtx* c = nullptr;
    if (int rc = kmer_ctx(&c)) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (int rc = c->tmp_u32.ensure((size_t)n * 4)) return rc;
    if (int rc = c->head.ensure((size_t)n * 4)) return rc;
    if (int rc = c->rid.ensure((size_t)n * 4)) return rc;
    if (int rc = c->obs_off.ensure((size_t)n * 8)) return rc;  // the u32 row indices, in and out
    if (int rc = c->scal.ensure(64)) return rc;
    const int g = grid_for(n);
    // round 4: u32 row indices through the sort (16 instead of 24 B per row and pass) and
    // only the keys' significant bits (C3: ids < 2^23, 3 onesweep passes instead of 4)
    uint32_t* const iota = c->obs_off.as<uint32_t>();
    uint32_t* const rows32 = iota + n;
    ROGTK_HIP_CHECK(hipMemsetAsync(c->scal.p, 0, 4, s));
    hipLaunchKernelGGL(k_key_max, dim3(std::min(g, 1024)), dim3(kBlock), 0, s, keys, n, c->scal.as<uint32_t>());
    hipLaunchKernelGGL(k_iota32, dim3(g), dim3(kBlock), 0, s, iota, n);
    uint32_t kmax = 0;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&kmax, c->scal.p, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    const int end_bit = kmax ? 32 - __builtin_clz(kmax) : 1;
    size_t bytes = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, keys, c->tmp_u32.as<uint32_t>(), iota, rows32,
                                                       (int)n, 0, end_bit, s));
    if (int rc = c->cub.ensure(bytes)) return rc;
    ROGTK_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(c->cub.p, bytes, keys, c->tmp_u32.as<uint32_t>(), iota, rows32,
                                                       (int)n, 0, end_bit, s));
    hipLaunchKernelGGL(k_key_heads, dim3(g), dim3(kBlock), 0, s, c->tmp_u32.as<uint32_t>(), n, c->head.as<uint32_t>());
    if (int rc = cub_exsum_u32(c, c->head.as<uint32_t>(), c->rid.as<uint32_t>(), n, s)) return rc;
    hipLaunchKernelGGL(k_key_offsets_rows, dim3(g), dim3(kBlock), 0, s, c->head.as<uint32_t>(), c->rid.as<uint32_t>(),
                       rows32, n, group_offsets_out, rows_out);
    ROGTK_HIP_CHECK(hipGetLastError());
    uint32_t last[2];
    ROGTK_HIP_CHECK(hipMemcpyAsync(&last[0], c->rid.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(&last[1], c->head.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    *n_groups = (int64_t)last[0] + last[1];
    return ROGTK_OK;
}

}  // extern "C"

namespace rogtk {
namespace {
int spectrum_dev(const int64_t* offsets, const uint8_t* values, const uint8_t* validity, int64_t validity_offset,
                 const int64_t* rows, int64_t n_rows, const int64_t* group_offsets, int64_t n_groups, int k,
                 int64_t min_coverage, int64_t capacity, uint64_t* kmers, uint8_t* exts, uint16_t* counts,
                 int64_t* entry_offsets, int64_t* group_stats, int64_t* n_entries, void* stream,
                 const uint64_t* blocks, int B, int S, bool fused = false, int64_t vlen = 0) {
    ROGTK_REQUIRE(offsets && values && group_offsets && entry_offsets && group_stats && n_entries, ROGTK_E_INVALID,
                  "kmer_dev: NULL argument");
    ROGTK_REQUIRE(n_rows >= 0 && n_groups >= 1 && min_coverage >= 0, ROGTK_E_INVALID,
                  "kmer_dev: n_rows >= 0, n_groups >= 1, min_coverage >= 0");
    ROGTK_REQUIRE(n_groups < (int64_t)0xFFFFFFFF, ROGTK_E_UNSUPPORTED, "kmer_dev: too many groups");
    KmerCtx* c = nullptr;
    if (int rc = kmer_ctx(&c)) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t G = n_groups;
    const int K = k > 64 ? 0 : effective_k(k);
    for (DevBuf* b : {&c->caps, &c->cap_off, &c->gcount, &c->gstart})
        if (int rc = b->ensure((size_t)(G + 1) * 8)) return rc;
    if (int rc = c->gk.ensure((size_t)G)) return rc;
    if (int rc = c->gstat.ensure((size_t)G * 5 * 8)) return rc;
    if (int rc = c->scal.ensure(64)) return rc;
    ROGTK_HIP_CHECK(hipMemsetAsync(c->gk.p, K, G, s));
    ROGTK_HIP_CHECK(hipMemsetAsync(c->gstat.p, 0, G * 5 * 8, s));
    ROGTK_HIP_CHECK(hipMemsetAsync(c->gcount.p, 0, G * 8, s));
    if (int rc = c->long_rows.ensure(8)) return rc;
    ROGTK_HIP_CHECK(hipMemsetAsync(c->long_rows.p, 0, 8, s));
    unsigned long long long_rows = 0;
    int64_t tcap = 0;
    if (blocks || fused) {
        // block path: a row holds at most 32 S bases, so at most 32 S - K + 1 observations;
        // the per-group capacities follow from the staged rows (run_class, cap_fill)
        tcap = valid_cap(n_rows * std::max<int64_t>(0, 32 * (int64_t)S - (K ? K : 64) + 1), min_coverage);
    } else {
        hipLaunchKernelGGL(k_group_caps, dim3(grid_for(G * 64, 16384)), dim3(kBlock), 0, s, offsets, rows,
                           group_offsets, G, c->caps.as<int64_t>(), min_coverage);
        if (int rc = cub_exsum_i64(c, c->caps.as<int64_t>(), c->cap_off.as<int64_t>(), G, s)) return rc;
        hipLaunchKernelGGL(k_tail_sum, dim3(1), dim3(64), 0, s, c->cap_off.as<int64_t>(), c->caps.as<int64_t>(), G,
                           c->cap_off.as<int64_t>() + G);
        ROGTK_HIP_CHECK(hipMemcpyAsync(&tcap, c->cap_off.as<int64_t>() + G, 8, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    }
    tcap = std::max<int64_t>(tcap, 1);
    if (int rc = c->t_kmer.ensure((size_t)tcap * 16)) return rc;
    if (int rc = c->t_ext.ensure((size_t)tcap)) return rc;
    if (int rc = c->t_cnt.ensure((size_t)tcap * 2)) return rc;
    c->last_lds_groups = c->last_global_groups = c->last_cert_groups = c->last_lds_rows = 0;
    if (K && n_rows > 0) {
        KIn in{offsets, values, validity, validity_offset, rows, group_offsets, c->gk.as<uint8_t>(),
               c->cap_off.as<int64_t>(), c->gstat.as<unsigned long long>(), c->gcount.as<int64_t>()};
        in.blocks = blocks;
        in.B = B;
        in.S = S;
        in.fused = fused;
        in.vlen = vlen;
        if (blocks || fused) in.cap_fill = c->caps.as<int64_t>();
        c->lo_only = K <= 32;
        if (int rc = run_any<8>(c, in, n_rows, G, K, min_coverage, s, nullptr)) return rc;
    }
    if (int rc = cub_exsum_i64(c, c->gcount.as<int64_t>(), entry_offsets, G, s)) return rc;
    hipLaunchKernelGGL(k_tail_sum, dim3(1), dim3(64), 0, s, entry_offsets, c->gcount.as<int64_t>(), G,
                       entry_offsets + G);
    ROGTK_HIP_CHECK(hipMemcpyAsync(n_entries, entry_offsets + G, 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(&long_rows, c->long_rows.p, 8, hipMemcpyDeviceToHost, s));
    hipLaunchKernelGGL(k_group_stats_out, dim3(grid_for(G)), dim3(kBlock), 0, s, c->gstat.as<unsigned long long>(),
                       c->gcount.as<int64_t>(), G, K, group_stats);
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    ROGTK_REQUIRE(long_rows == 0, ROGTK_E_INVALID,
                  "kmer_blocks: %llu row(s) longer than max_len %d (the packed column's bound)", long_rows, 32 * S);
    ROGTK_REQUIRE(*n_entries <= capacity, ROGTK_E_OVERFLOW, "kmer_dev: %lld entries exceed capacity %lld",
                  (long long)*n_entries, (long long)capacity);
    if (*n_entries > 0) {
        ROGTK_REQUIRE(kmers && exts && counts, ROGTK_E_INVALID, "kmer_dev: output arrays are NULL");
        // the caller's k-mer array may sit at any 8-B offset of its buffer
        const bool v16 = ((uintptr_t)kmers & 15u) == 0;
        auto pack = c->lo_only ? (v16 ? k_pack<true, true> : k_pack<false, true>)
                               : (v16 ? k_pack<true, false> : k_pack<false, false>);
        hipLaunchKernelGGL(pack, dim3(grid_for(G * 64, 16384)), dim3(kBlock), 0, s, c->t_kmer.as<uint64_t>(),
                           c->t_ext.as<uint8_t>(), c->t_cnt.as<uint16_t>(), G, c->cap_off.as<int64_t>(),
                           c->gcount.as<int64_t>(), entry_offsets, kmers, exts, counts);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    return ROGTK_OK;
}
}  // namespace
}  // namespace rogtk

extern "C" {

int rogtk_kmer_spectrum_dev(const int64_t* offsets, const uint8_t* values, const uint8_t* validity,
                            int64_t validity_offset, const int64_t* rows, int64_t n_rows,
                            const int64_t* group_offsets, int64_t n_groups, int k, int64_t min_coverage,
                            int64_t capacity, uint64_t* kmers, uint8_t* exts, uint16_t* counts,
                            int64_t* entry_offsets, int64_t* group_stats, int64_t* n_entries, void* stream) {
    return spectrum_dev(offsets, values, validity, validity_offset, rows, n_rows, group_offsets, n_groups, k,
                        min_coverage, capacity, kmers, exts, counts, entry_offsets, group_stats, n_entries, stream,
                        nullptr, 0, 0);
}

int rogtk_read_block_words(int64_t max_len) {
    if (max_len < 0) return 0;
    const int64_t words = 1 + (max_len + 31) / 32;  // meta + bases
    return words <= 8 ? 8 : words <= 16 ? 16 : words <= 32 ? 32 : 0;
}

int rogtk_pack_reads(const int64_t* offsets, const uint8_t* values, const uint8_t* validity, int64_t validity_offset,
                     int64_t n, int block_words, uint64_t* blocks, int64_t* max_len, void* stream) {
    ROGTK_REQUIRE(n >= 0 && (n == 0 || (offsets && values && blocks)), ROGTK_E_INVALID, "pack_reads: NULL argument");
    ROGTK_REQUIRE(block_words == 8 || block_words == 16 || block_words == 32, ROGTK_E_INVALID,
                  "pack_reads: block_words must be 8, 16 or 32 (rogtk_read_block_words)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (max_len) ROGTK_HIP_CHECK(hipMemsetAsync(max_len, 0, 8, s));
    if (n == 0) return ROGTK_OK;
    constexpr int kRows = 64;  // one wave per workgroup (k_pack_reads)
    const int g = (int)std::min<int64_t>((n + kRows - 1) / kRows, (int64_t)8192 * 256 / kRows);
    ProfScope prof(K_PACK_READS, s, true);
#define ROGTK_PACK_LAUNCH(BW)                                                                                       \
    hipExtLaunchKernelGGL((k_pack_reads<BW, kRows>), dim3(g), dim3(kRows), 0, s, prof.start(), prof.stop(), 0, offsets, \
                          values, validity, validity_offset, n, blocks, (unsigned long long*)max_len)
    if (block_words == 8)
        ROGTK_PACK_LAUNCH(8);
    else if (block_words == 16)
        ROGTK_PACK_LAUNCH(16);
    else
        ROGTK_PACK_LAUNCH(32);
#undef ROGTK_PACK_LAUNCH
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

int rogtk_max_row_len(const int64_t* offsets, int64_t n, int64_t* max_len, void* stream) {
    ROGTK_REQUIRE(max_len && n >= 0 && (n == 0 || offsets), ROGTK_E_INVALID, "max_row_len: NULL argument");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    KmerCtx* c = nullptr;
    if (int rc = kmer_ctx(&c)) return rc;
    if (int rc = c->scal.ensure(64)) return rc;
    ROGTK_HIP_CHECK(hipMemsetAsync(c->scal.p, 0, 8, s));
    if (n > 0)
        hipLaunchKernelGGL(k_max_row_len, dim3((unsigned)std::min<int64_t>((n + kBlock - 1) / kBlock, 4096)),
                           dim3(kBlock), 0, s, offsets, n, c->scal.as<unsigned long long>());
    unsigned long long m = 0;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&m, c->scal.p, 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    *max_len = (int64_t)m;
    return ROGTK_OK;
}

int rogtk_kmer_spectrum_fused(const int64_t* offsets, const uint8_t* values, int64_t values_len,
                              const uint8_t* validity, int64_t validity_offset, const int64_t* rows, int64_t n_rows,
                              const int64_t* group_offsets, int64_t n_groups, int k, int64_t min_coverage,
                              int64_t capacity, uint64_t* kmers, uint8_t* exts, uint16_t* counts,
                              int64_t* entry_offsets, int64_t* group_stats, int64_t* n_entries, int64_t max_len,
                              int64_t n_column, void* stream) {
    ROGTK_REQUIRE(offsets && values && values_len >= 0, ROGTK_E_INVALID, "kmer_fused: NULL argument");
    ROGTK_REQUIRE(((uintptr_t)values & 15u) == 0, ROGTK_E_UNSUPPORTED,
                  "kmer_fused: values must be 16-byte aligned (16-B loads; use the block column)");
    if (max_len < 0) {  // the column's longest row: one pass over its offsets and one 8-byte read
        ROGTK_REQUIRE(n_column >= 0, ROGTK_E_INVALID, "kmer_fused: max_len < 0 needs n_column");
        if (int rc = rogtk_max_row_len(offsets, n_column, &max_len, stream)) return rc;
    }
    ROGTK_REQUIRE(max_len <= 224, ROGTK_E_UNSUPPORTED,
                  "kmer_fused: rows up to %lld bases; the fused staging takes <= 224 (use the block column)",
                  (long long)max_len);
    return spectrum_dev(offsets, values, validity, validity_offset, rows, n_rows, group_offsets, n_groups, k,
                        min_coverage, capacity, kmers, exts, counts, entry_offsets, group_stats, n_entries, stream,
                        nullptr, 8, (int)std::max<int64_t>(1, (max_len + 31) / 32), true, values_len);
}

int rogtk_kmer_spectrum_blocks(const uint64_t* blocks, int block_words, int64_t max_len, const int64_t* offsets,
                               const uint8_t* values, const uint8_t* validity, int64_t validity_offset,
                               const int64_t* rows, int64_t n_rows, const int64_t* group_offsets, int64_t n_groups,
                               int k, int64_t min_coverage, int64_t capacity, uint64_t* kmers, uint8_t* exts,
                               uint16_t* counts, int64_t* entry_offsets, int64_t* group_stats, int64_t* n_entries,
                               void* stream) {
    ROGTK_REQUIRE(blocks, ROGTK_E_INVALID, "kmer_blocks: NULL blocks");
    ROGTK_REQUIRE(block_words == rogtk_read_block_words(max_len) && block_words > 0, ROGTK_E_INVALID,
                  "kmer_blocks: block_words %d does not match max_len %lld", block_words, (long long)max_len);
    return spectrum_dev(offsets, values, validity, validity_offset, rows, n_rows, group_offsets, n_groups, k,
                        min_coverage, capacity, kmers, exts, counts, entry_offsets, group_stats, n_entries, stream,
                        blocks, block_words, (int)std::max<int64_t>(1, (max_len + 31) / 32));
}

}  // extern "C"
