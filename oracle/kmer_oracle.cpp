// =============================================================================
// kmer_oracle.cpp — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT PATH.
//
// CPU restatement of rogtk's k-mer front end of fracture assembly (SURVEY.md §8a
// H4.1-H4.2), used only by tests/ and bench tooling as the checker.
//
// Reference call path (per group of reads, i.e. per polars group_by group):
//   expressions.rs:739-744   sequences = column.into_iter().flatten() (nulls skipped)
//   fracture.rs:200-208      auto_k -> estimate_k (fracture.rs:24-54)
//   fracture.rs:211-214      k > 64 -> no output
//   fracture.rs:217-229      to_uppercase, drop any sequence with a non-ACGT byte
//   fracture.rs:246-256      effective k = 4 / 8 / 16 / 32 / 64 (Kmer4..Kmer64)
//   fracture.rs:105-116      filter_kmers::<K>(seqs, CountFilter::new(min_cov),
//                            stranded = true, report_all_kmers = true, memory_size = 4)
//   fracture.rs:118-146      node / terminal / isolated counts
// The arithmetic below filter_kmers lives in the third-party crate
// debruijn = "0.3.4" (Cargo.toml:51; no lockfile, crate sources absent here). Its
// published algorithm, restated (crate, unverified against its sources):
//   * iter_kmer_exts: every k-mer of a sequence with a 1-base extension on each
//     side; the sequence's own exts are empty (fracture.rs:238-240), so the first
//     k-mer has no left and the last k-mer no right extension. Exts is a u8: low
//     nibble = left bases, high nibble = right bases (bit = base A0 C1 G2 T3).
//   * stranded -> no reverse-complement canonicalisation.
//   * bucket by the k-mer's top byte (its first 4 bases), sort each bucket, group
//     equal k-mers; buckets are visited in order, so the output is sorted.
//   * CountFilter: count = number of observations (u16, saturating), exts = OR of
//     the observations' exts, valid iff count >= min_cov.
//   * remove_censored_exts: an extension survives only if the extended k-mer
//     (extend_left: base + kmer[0..k-1]; extend_right: kmer[1..k] + base) is
//     itself valid (binary search over the sorted valid list).
//   * BoomHashMap2 then reorders the entries by MPHF slot: that order is not
//     reproducible without the crate sources, so parity is on the sorted
//     (kmer, exts, count) set ("parity unpinned" for the MPHF order).
// K-mers are 2-bit codes, first base most significant (A0 C1 G2 T3), so numeric
// order == the crate's Kmer Ord == lexicographic order.
// =============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

typedef unsigned __int128 u128;

inline bool row_valid(const uint8_t* validity, int64_t bit_offset, int64_t i) {
    if (!validity) return true;
    int64_t b = bit_offset + i;
    return (validity[b >> 3] >> (b & 7)) & 1;
}

inline void row_span(const void* offsets, int offset_width, int64_t i, int64_t* start, int64_t* len) {
    if (offset_width == 4) {
        const int32_t* o = (const int32_t*)offsets;
        *start = o[i];
        *len = (int64_t)o[i + 1] - o[i];
    } else {
        const int64_t* o = (const int64_t*)offsets;
        *start = o[i];
        *len = o[i + 1] - o[i];
    }
}

// ---- fracture.rs:24-54 -------------------------------------------------------
int estimate_k(const std::vector<std::string>& seqs) {
    if (seqs.empty()) return 31;
    uint64_t total = 0, count = 0;
    for (const auto& s : seqs) {
        if (!s.empty()) {
            total += s.size();
            count += 1;
        }
    }
    if (count == 0) return 31;
    const double mean = (double)total / (double)count;
    int64_t k = (int64_t)std::round(mean / 3.0);  // f64::round: half away from zero
    // k even -> k - 1; usize 0 - 1 wraps in a release build (clamped to 63 below)
    uint64_t ku = (k % 2 == 0) ? (uint64_t)k - 1 : (uint64_t)k;
    if (ku < 11) ku = 11;
    if (ku > 63) ku = 63;
    return (int)ku;
}

int effective_k(int k) {
    return k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : k <= 32 ? 32 : 64;
}

int base_code(char c) {
    switch (c) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        default: return 3;  // 'T' (sequences were validated)
    }
}

struct Obs {
    u128 kmer;
    uint8_t exts;
};

}  // namespace

extern "C" {

// One group: rows [row_begin, row_end) of an Arrow string column. Writes up to
// `cap` valid entries sorted by k-mer: kmers_hilo[2i] = high 64 bits (k = 64 only),
// kmers_hilo[2i+1] = low 64 bits. stats5 = {k_eff (0 when k > 64), n_sequences,
// node_count, terminal_count, isolated_count}. Returns the entry count, -1 when
// cap is too small.
int64_t oracle_kmer_spectrum(const void* offsets, int offset_width, const uint8_t* values,
                             const uint8_t* validity, int64_t validity_offset, int64_t row_begin,
                             int64_t row_end, int k, int auto_k, int64_t min_cov, uint64_t* kmers_hilo,
                             uint8_t* exts_out, uint16_t* counts_out, int64_t cap, int64_t* stats5) {
    for (int i = 0; i < 5; ++i) stats5[i] = 0;
    // expressions.rs:739-744: nulls are skipped
    std::vector<std::string> raw;
    for (int64_t r = row_begin; r < row_end; ++r) {
        if (!row_valid(validity, validity_offset, r)) continue;
        int64_t st, len;
        row_span(offsets, offset_width, r, &st, &len);
        raw.emplace_back((const char*)values + st, (size_t)len);
    }
    if (auto_k) k = estimate_k(raw);
    if (k > 64) return 0;  // fracture.rs:211-214
    // fracture.rs:217-229 (ASCII uppercase: no non-ASCII scalar uppercases to A/C/G/T)
    std::vector<std::string> seqs;
    for (auto& s : raw) {
        bool ok = true;
        for (auto& ch : s) {
            if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
            if (ch != 'A' && ch != 'C' && ch != 'G' && ch != 'T') ok = false;
        }
        if (ok) seqs.push_back(s);
    }
    const int K = effective_k(k);
    stats5[0] = K;
    stats5[1] = (int64_t)seqs.size();
    if (seqs.empty()) return 0;

    const u128 mask = K == 64 ? ~(u128)0 : (((u128)1 << (2 * K)) - 1);
    // filter_kmers: one bucket per top byte (memory_size 4 GB -> a single slice here)
    std::vector<std::vector<Obs>> buckets(256);
    for (const auto& s : seqs) {
        const int64_t n = (int64_t)s.size();
        if (n < K) continue;
        u128 km = 0;
        for (int i = 0; i < K; ++i) km = (km << 2) | (u128)base_code(s[i]);
        for (int64_t i = 0; i + K <= n; ++i) {
            if (i > 0) km = ((km << 2) | (u128)base_code(s[i + K - 1])) & mask;
            uint8_t e = 0;
            if (i > 0) e |= (uint8_t)(1u << base_code(s[i - 1]));           // left ext
            if (i + K < n) e |= (uint8_t)(1u << (4 + base_code(s[i + K])));  // right ext
            const int bucket = (int)((km >> (2 * K - 8)) & 0xFF);
            buckets[bucket].push_back({km, e});
        }
    }
    std::vector<u128> vk;
    std::vector<uint8_t> ve;
    std::vector<uint16_t> vc;
    for (auto& b : buckets) {
        std::stable_sort(b.begin(), b.end(), [](const Obs& x, const Obs& y) { return x.kmer < y.kmer; });
        size_t i = 0;
        while (i < b.size()) {
            size_t j = i;
            uint16_t count = 0;
            uint8_t e = 0;
            while (j < b.size() && b[j].kmer == b[i].kmer) {
                if (count < 0xFFFF) count += 1;  // saturating_add
                e |= b[j].exts;
                ++j;
            }
            if ((int64_t)count >= min_cov) {
                vk.push_back(b[i].kmer);
                ve.push_back(e);
                vc.push_back(count);
            }
            i = j;
        }
    }
    // remove_censored_exts (stranded): keep an ext only if the neighbour is valid
    std::vector<uint8_t> ne(vk.size(), 0);
    for (size_t i = 0; i < vk.size(); ++i) {
        for (int dir = 0; dir < 2; ++dir) {
            for (int b = 0; b < 4; ++b) {
                if (!((ve[i] >> (4 * dir + b)) & 1)) continue;
                const u128 nb = dir == 0 ? ((vk[i] >> 2) | ((u128)b << (2 * K - 2)))  // extend_left
                                         : (((vk[i] << 2) | (u128)b) & mask);         // extend_right
                if (std::binary_search(vk.begin(), vk.end(), nb)) ne[i] |= (uint8_t)(1u << (4 * dir + b));
            }
        }
    }
    if ((int64_t)vk.size() > cap) return -1;
    int64_t terminal = 0, isolated = 0;
    for (size_t i = 0; i < vk.size(); ++i) {
        kmers_hilo[2 * i] = (uint64_t)(vk[i] >> 64);
        kmers_hilo[2 * i + 1] = (uint64_t)vk[i];
        exts_out[i] = ne[i];
        counts_out[i] = vc[i];
        const bool l0 = (ne[i] & 0xF) == 0, r0 = (ne[i] >> 4) == 0;
        if (l0 || r0) terminal += 1;  // fracture.rs:134-139
        if (l0 && r0) isolated += 1;
    }
    stats5[2] = (int64_t)vk.size();
    stats5[3] = terminal;
    stats5[4] = isolated;
    return (int64_t)vk.size();
}

// Upper bound on the valid entries of rows [row_begin, row_end) for effective k K:
// the number of k-mer observations (every row counted, no filtering).
int64_t oracle_kmer_observations(const void* offsets, int offset_width, int64_t row_begin, int64_t row_end, int K) {
    int64_t t = 0;
    for (int64_t r = row_begin; r < row_end; ++r) {
        int64_t st, len;
        row_span(offsets, offset_width, r, &st, &len);
        if (len >= K) t += len - K + 1;
    }
    return t;
}

}  // extern "C"
