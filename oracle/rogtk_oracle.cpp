// =============================================================================
// rogtk_oracle.cpp — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT PATH.
//
// CPU restatement of the reference (tzeitim/rogtk) algorithms on the UMI
// score + cluster hot path. Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library, and only as the checker / the CPU
// baseline; the product (rogtk_amd + librogtk_hip.so) never links or calls it.
//
// Parity pinning: the reference is Rust (no cargo/rustc in this image) and has
// no tests or golden vectors for these functions. The
// restatement is pinned by (1) the hand-derived known answers of SURVEY.md
// Appendix A, (2) an independent pure-Python restatement (oracle/pyoracle.py),
// and (3) the golden vectors it generated, committed under tests/golden/.
//
// Data structures deliberately mirror the reference (per-UMI hash maps, serial
// row loop) so this also serves as the "port" CPU baseline of bench.py.
//
// Deliberate, documented deviation: dinucleotide_entropy sums its terms in
// ascending (byte0, byte1) order. The reference sums in Rust HashMap
// iteration order (RandomState, different in every process), so the reference
// itself is not bit-reproducible there (≤2 ULP spread).
// `dinuc_order = 1` selects first-occurrence order (the order Appendix A's
// printed values used) for the KAT check.
//
// Build: see oracle/Makefile (g++ -O2 -ffp-contract=off, glibc log2).
// =============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <iterator>
#include <map>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

// ---- umi_score.rs:45-73 ------------------------------------------------------
double shannon_entropy(const uint8_t* s, size_t n) {
    uint32_t counts[4] = {0, 0, 0, 0};
    uint32_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        total += 1;  // every byte counts toward total (:50), incl. N / lowercase
        switch (s[i]) {
            case 'A': counts[0] += 1; break;
            case 'C': counts[1] += 1; break;
            case 'G': counts[2] += 1; break;
            case 'T': counts[3] += 1; break;
            default: break;
        }
    }
    if (total == 0) return 0.0;
    double entropy = 0.0;
    for (int b = 0; b < 4; ++b) {  // fixed A,C,G,T order (:65)
        if (counts[b] > 0) {
            double p = (double)counts[b] / (double)total;
            entropy -= p * std::log2(p);
        }
    }
    return entropy;
}

// ---- umi_score.rs:77-93 ------------------------------------------------------
double linguistic_complexity(const uint8_t* s, size_t n) {
    if (n < 3) return 0.0;
    const size_t k = 3;
    std::unordered_map<uint32_t, int> kmers;  // key = the 3-byte window
    for (size_t i = 0; i + k <= n; ++i) {
        uint32_t key = ((uint32_t)s[i] << 16) | ((uint32_t)s[i + 1] << 8) | s[i + 2];
        kmers[key] += 1;
    }
    double unique_kmers = (double)kmers.size();
    double max_possible = (double)std::min<size_t>(n - k + 1, 64);  // 4^3 (:90)
    return unique_kmers / max_possible;
}

// ---- umi_score.rs:96-121 -----------------------------------------------------
double homopolymer_fraction(const uint8_t* s, size_t n) {
    if (n == 0) return 0.0;
    size_t in_homopolymer = 0, i = 0;
    while (i < n) {
        uint8_t current = s[i];
        size_t run_length = 1;
        while (i + run_length < n && s[i + run_length] == current) run_length += 1;
        if (run_length >= 3) in_homopolymer += run_length;
        i += run_length;
    }
    return (double)in_homopolymer / (double)n;
}

// ---- umi_score.rs:124-146 ----------------------------------------------------
double dinucleotide_entropy(const uint8_t* s, size_t n, int order) {
    if (n < 2) return 0.0;
    const double total = (double)(n - 1);
    double entropy = 0.0;
    if (order == 0) {
        // canonical: ascending (byte0, byte1) — std::map iterates in key order
        std::map<std::pair<uint8_t, uint8_t>, int> counts;
        for (size_t i = 0; i + 2 <= n; ++i) counts[{s[i], s[i + 1]}] += 1;
        for (const auto& kv : counts) {
            double p = (double)kv.second / total;
            entropy -= p * std::log2(p);
        }
    } else {
        // first-occurrence order (SURVEY.md Appendix A convention)
        std::vector<std::pair<uint16_t, int>> counts;
        for (size_t i = 0; i + 2 <= n; ++i) {
            uint16_t key = (uint16_t)((s[i] << 8) | s[i + 1]);
            auto it = std::find_if(counts.begin(), counts.end(),
                                   [&](const std::pair<uint16_t, int>& e) { return e.first == key; });
            if (it == counts.end()) counts.push_back({key, 1});
            else it->second += 1;
        }
        for (const auto& kv : counts) {
            double p = (double)kv.second / total;
            entropy -= p * std::log2(p);
        }
    }
    return entropy / 4.0;
}

// ---- umi_score.rs:149-168 ----------------------------------------------------
size_t longest_homopolymer_run(const uint8_t* s, size_t n) {
    if (n == 0) return 0;
    size_t max_run = 1, current_run = 1;
    for (size_t i = 1; i < n; ++i) {
        if (s[i] == s[i - 1]) {
            current_run += 1;
            max_run = std::max(max_run, current_run);
        } else {
            current_run = 1;
        }
    }
    return max_run;
}

// ---- umi_score.rs:171-200 ----------------------------------------------------
double dust_score(const uint8_t* s, size_t n, size_t window_size) {
    if (n < window_size) return 0.0;
    double total_score = 0.0;
    for (size_t i = 0; i + window_size <= n; ++i) {
        const uint8_t* w = s + i;
        std::unordered_map<uint32_t, int> triplet_counts;
        for (size_t j = 0; j + 3 <= window_size; ++j) {
            uint32_t key = ((uint32_t)w[j] << 16) | ((uint32_t)w[j + 1] << 8) | w[j + 2];
            triplet_counts[key] += 1;
        }
        double window_score = 0.0;
        for (const auto& kv : triplet_counts) {
            int count = kv.second;
            if (count > 1) window_score += (double)(count * (count - 1)) / 2.0;
        }
        total_score += window_score;
    }
    return total_score / (double)(n - window_size + 1);
}

struct Score {
    double shannon, linguistic, homopolymer, dinuc, dust, combined;
    uint32_t longest;
};

// ---- umi_score.rs:17-43 ------------------------------------------------------
Score calculate_umi_complexity(const uint8_t* s, size_t n, int order) {
    Score r;
    r.shannon = shannon_entropy(s, n);
    r.linguistic = linguistic_complexity(s, n);
    r.homopolymer = homopolymer_fraction(s, n);
    r.dinuc = dinucleotide_entropy(s, n, order);
    size_t longest = longest_homopolymer_run(s, n);
    r.dust = dust_score(s, n, 64);
    // evaluated left to right, no contraction (built with -ffp-contract=off)
    r.combined = 0.25 * r.shannon
               + 0.25 * r.linguistic
               + 0.15 * (1.0 - r.homopolymer)
               + 0.15 * r.dinuc
               + 0.10 * (1.0 - ((double)longest / (double)n))
               + 0.10 * (1.0 - std::fmin(r.dust, 1.0));
    r.longest = (uint32_t)longest;  // exported as UInt32 (expressions.rs:1254)
    return r;
}

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

// Decode one UTF-8 scalar (input is a valid Rust &str / Arrow utf8 value).
inline size_t utf8_next(const uint8_t* s, size_t n, size_t i, uint32_t* cp) {
    uint8_t c = s[i];
    size_t w = c < 0x80 ? 1 : (c >> 5) == 0x6 ? 2 : (c >> 4) == 0xE ? 3 : 4;
    if (i + w > n) w = n - i;
    uint32_t v = w == 1 ? c : w == 2 ? (c & 0x1F) : w == 3 ? (c & 0x0F) : (c & 0x07);
    for (size_t k = 1; k < w; ++k) v = (v << 6) | (s[i + k] & 0x3F);
    *cp = v;
    return i + w;
}

// ---- expressions.rs:1054-1069: byte-length check, then chars().zip() ----------
uint32_t hamming_one(const uint8_t* s, size_t n, const uint8_t* t, size_t tn) {
    if (n != tn) return UINT32_MAX;
    uint32_t d = 0;
    size_t i = 0, j = 0;
    while (i < n && j < tn) {
        uint32_t a, b;
        i = utf8_next(s, n, i, &a);
        j = utf8_next(t, tn, j, &b);
        if (a != b) d += 1;
    }
    return d;
}

}  // namespace

extern "C" {

const char* oracle_version(void) { return "rogtk-oracle 1 (umi_score.rs/expressions.rs restatement)"; }

// One UMI. out6 = {shannon, linguistic, homopolymer, dinuc, dust, combined}.
void oracle_umi_complexity(const uint8_t* s, int64_t n, int dinuc_order, double* out6, uint32_t* longest) {
    Score r = calculate_umi_complexity(s, (size_t)n, dinuc_order);
    out6[0] = r.shannon; out6[1] = r.linguistic; out6[2] = r.homopolymer;
    out6[3] = r.dinuc;   out6[4] = r.dust;       out6[5] = r.combined;
    *longest = r.longest;
}

// Row loop of umi_complexity_all_expr (expressions.rs:1246-1268). Null rows are
// skipped (their outputs are left untouched; validity = input validity).
void oracle_umi_complexity_batch(const void* offsets, int offset_width, const uint8_t* values,
                                 const uint8_t* validity, int64_t validity_offset, int64_t n,
                                 int dinuc_order, double* shannon, double* linguistic,
                                 double* homopolymer, double* dinuc, uint32_t* longest,
                                 double* dust, double* combined) {
    for (int64_t i = 0; i < n; ++i) {
        if (!row_valid(validity, validity_offset, i)) continue;
        int64_t st, len;
        row_span(offsets, offset_width, i, &st, &len);
        Score r = calculate_umi_complexity(values + st, (size_t)len, dinuc_order);
        if (shannon) shannon[i] = r.shannon;
        if (linguistic) linguistic[i] = r.linguistic;
        if (homopolymer) homopolymer[i] = r.homopolymer;
        if (dinuc) dinuc[i] = r.dinuc;
        if (longest) longest[i] = r.longest;
        if (dust) dust[i] = r.dust;
        if (combined) combined[i] = r.combined;
    }
}

// hamming_distance_expr (expressions.rs:1048-1073) / hamming_within_expr
// (:1075-1101). dist: u32::MAX on byte-length mismatch; within: dist <= max.
void oracle_hamming_batch(const void* offsets, int offset_width, const uint8_t* values,
                          const uint8_t* validity, int64_t validity_offset, int64_t n,
                          const uint8_t* target, int64_t target_len, uint32_t max_distance,
                          uint32_t* dist, uint8_t* within) {
    for (int64_t i = 0; i < n; ++i) {
        if (!row_valid(validity, validity_offset, i)) continue;
        int64_t st, len;
        row_span(offsets, offset_width, i, &st, &len);
        uint32_t d = hamming_one(values + st, (size_t)len, target, (size_t)target_len);
        if (dist) dist[i] = d;
        if (within) within[i] = (d != UINT32_MAX && d <= max_distance) ? 1 : 0;
    }
}

// ---- H3: UMI cluster assignment (spec owned by this build) ----
// Regular rows (byte length == L <= 32, all of A/C/G/T) are packed 2 bits/base, first
// base most significant (A=0,C=1,G=2,T=3), so code order == lexicographic order. Every
// other non-null row is irregular (N, lowercase, other lengths, any bytes).
// max_distance 0: clusters = distinct strings. max_distance 1: connected components of
// the graph over ALL distinct non-null strings with an edge wherever the H2.1 distance
// (expressions.rs:1054-1069: equal byte length, then mismatches) is 1, compared byte by
// byte (N and lowercase are ordinary bytes, distinct from A/C/G/T).
// An irregular string can thus join a regular cluster (ACGTNACGTACG ~ ACGTAACGTACG) and
// bridge two of them.
// Ids are dense: components holding a regular UMI first, in order of their smallest
// regular code; then components of irregular strings only, in byte-lexicographic order of
// their smallest string. Null rows get no id (out_valid = 0).
// umi_len <= 0: L = byte length of the first non-null row.
// Returns the number of clusters, or -1 on bad arguments. oracle_umi_cluster_mt splits the
// row passes and the edge search over `threads` host threads (same result for any count).
int64_t oracle_umi_cluster_mt(const void* offsets, int offset_width, const uint8_t* values,
                              const uint8_t* validity, int64_t validity_offset, int64_t n, int umi_len,
                              int max_distance, uint32_t* cluster_id, uint8_t* out_valid, int* resolved_len,
                              int threads) {
    if (max_distance < 0 || max_distance > 1) return -1;
    if (threads < 1) threads = 1;
    int L = umi_len;
    if (L <= 0) {
        L = 0;
        for (int64_t i = 0; i < n; ++i)
            if (row_valid(validity, validity_offset, i)) {
                int64_t st, len;
                row_span(offsets, offset_width, i, &st, &len);
                L = (int)len;
                break;
            }
    }
    if (resolved_len) *resolved_len = L;
    const bool packable = L >= 1 && L <= 32;
    // row chunks / index ranges per thread (results do not depend on the split: every
    // union-find root is its component's smallest vertex)
    auto parallel = [&](int64_t count, auto&& fn) {
        const int t = (int)std::max<int64_t>(1, std::min<int64_t>(threads, count / 4096 + 1));
        std::vector<std::thread> pool;
        for (int k = 0; k < t; ++k)
            pool.emplace_back([&, k] { fn(k, count * k / t, count * (k + 1) / t); });
        for (auto& th : pool) th.join();
        return t;
    };
    std::vector<uint64_t> codes((size_t)n, 0);
    std::vector<uint8_t> cls((size_t)n, 0);  // 0 null, 1 regular, 2 irregular
    std::vector<std::vector<uint64_t>> part((size_t)threads);
    const int tp = parallel(n, [&](int k, int64_t lo, int64_t hi) {
        std::vector<uint64_t>& mine = part[(size_t)k];
        for (int64_t i = lo; i < hi; ++i) {
            if (!row_valid(validity, validity_offset, i)) continue;
            int64_t st, len;
            row_span(offsets, offset_width, i, &st, &len);
            const uint8_t* s = values + st;
            bool reg = packable && len == L;
            uint64_t c = 0;
            for (int64_t j = 0; reg && j < len; ++j) {
                int b = s[j] == 'A' ? 0 : s[j] == 'C' ? 1 : s[j] == 'G' ? 2 : s[j] == 'T' ? 3 : -1;
                if (b < 0) reg = false;
                c = (c << 2) | (uint64_t)(b & 3);
            }
            cls[(size_t)i] = reg ? 1 : 2;
            if (reg) {
                codes[(size_t)i] = c;
                mine.push_back(c);
            }
        }
        std::sort(mine.begin(), mine.end());
        mine.erase(std::unique(mine.begin(), mine.end()), mine.end());
    });
    // merge the sorted per-thread sets pairwise
    for (int width = 1; width < tp; width *= 2) {
        std::vector<std::thread> pool;
        for (int k = 0; k + width < tp; k += 2 * width)
            pool.emplace_back([&, k, width] {
                std::vector<uint64_t> m;
                m.reserve(part[(size_t)k].size() + part[(size_t)(k + width)].size());
                std::set_union(part[(size_t)k].begin(), part[(size_t)k].end(), part[(size_t)(k + width)].begin(),
                               part[(size_t)(k + width)].end(), std::back_inserter(m));
                part[(size_t)k].swap(m);
                std::vector<uint64_t>().swap(part[(size_t)(k + width)]);
            });
        for (auto& th : pool) th.join();
    }
    std::vector<uint64_t> distinct;
    distinct.swap(part[0]);
    const size_t D = distinct.size();
    std::vector<uint32_t> parent(D);
    for (size_t i = 0; i < D; ++i) parent[i] = (uint32_t)i;
    auto find = [&](uint32_t x) {
        while (parent[x] != x) { parent[x] = parent[parent[x]]; x = parent[x]; }
        return x;
    };
    auto unite = [&](uint32_t x, uint32_t y) {
        uint32_t a = find(x), b = find(y);
        if (a == b) return;
        if (a < b) std::swap(a, b);
        parent[a] = b;  // hook larger root under smaller: root = smallest vertex
    };
    if (max_distance == 1) {
        // regular ~ regular: the Hamming-1 neighbours of every distinct code (edges found
        // in parallel, united serially)
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> edges((size_t)threads);
        parallel((int64_t)D, [&](int k, int64_t lo, int64_t hi) {
            auto& e = edges[(size_t)k];
            for (int64_t i = lo; i < hi; ++i) {
                const uint64_t c = distinct[(size_t)i];
                for (int p = 0; p < L; ++p)
                    for (uint64_t d = 1; d <= 3; ++d) {
                        uint64_t nb = c ^ (d << (2 * p));
                        if (nb >= c) continue;
                        auto it = std::lower_bound(distinct.begin(), distinct.end(), nb);
                        if (it == distinct.end() || *it != nb) continue;
                        e.emplace_back((uint32_t)i, (uint32_t)(it - distinct.begin()));
                    }
            }
        });
        for (auto& e : edges)
            for (auto& pr : e) unite(pr.first, pr.second);
    }
    // irregular distinct strings, byte-lexicographic: vertices D + j
    std::map<std::string, uint32_t> irregular;
    for (int64_t i = 0; i < n; ++i)
        if (cls[(size_t)i] == 2) {
            int64_t st, len;
            row_span(offsets, offset_width, i, &st, &len);
            irregular.emplace(std::string((const char*)values + st, (size_t)len), 0);
        }
    std::vector<const std::string*> istr;
    for (auto& kv : irregular) {
        kv.second = (uint32_t)istr.size();
        istr.push_back(&kv.first);
    }
    const size_t I = istr.size();
    parent.resize(D + I);
    for (size_t j = 0; j < I; ++j) parent[D + j] = (uint32_t)(D + j);
    if (max_distance == 1) {
        // irregular ~ irregular: equal length, equal except at one position p -> same
        // (p, string without byte p) key; link each to the first string seen
        std::map<std::pair<size_t, std::string>, uint32_t> first;
        for (size_t j = 0; j < I; ++j) {
            const std::string& s = *istr[j];
            for (size_t p = 0; p < s.size(); ++p) {
                std::string key = s.substr(0, p) + s.substr(p + 1);
                auto it = first.emplace(std::make_pair(p, std::move(key)), (uint32_t)j);
                if (!it.second) unite((uint32_t)(D + it.first->second), (uint32_t)(D + j));
            }
        }
        // irregular ~ regular: length L with exactly one non-ACGT byte at p -> the codes
        // with A/C/G/T at p
        for (size_t j = 0; packable && j < I; ++j) {
            const std::string& s = *istr[j];
            if ((int)s.size() != L) continue;
            int bad = -1, nbad = 0;
            uint64_t c = 0;
            for (int q = 0; q < L; ++q) {
                const char ch = s[(size_t)q];
                int b = ch == 'A' ? 0 : ch == 'C' ? 1 : ch == 'G' ? 2 : ch == 'T' ? 3 : -1;
                if (b < 0) {
                    ++nbad;
                    bad = q;
                    b = 0;
                }
                c = (c << 2) | (uint64_t)b;
            }
            if (nbad != 1) continue;
            const int sh = 2 * (L - 1 - bad);
            for (uint64_t x = 0; x < 4; ++x) {
                const uint64_t nb = (c & ~(3ull << sh)) | (x << sh);
                auto it = std::lower_bound(distinct.begin(), distinct.end(), nb);
                if (it != distinct.end() && *it == nb)
                    unite((uint32_t)(D + j), (uint32_t)(it - distinct.begin()));
            }
        }
    }
    std::vector<uint32_t> label(D + I);
    uint32_t next = 0;
    for (size_t i = 0; i < D + I; ++i) {  // roots in vertex order
        uint32_t r = find((uint32_t)i);
        if (r == i) label[i] = next++;
        else label[i] = label[r];  // r < i already labelled
    }
    parallel(n, [&](int, int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i) {
            if (out_valid) out_valid[i] = cls[(size_t)i] != 0;
            if (cls[(size_t)i] == 0) {
                cluster_id[i] = 0;
            } else if (cls[(size_t)i] == 1) {
                size_t idx = (size_t)(std::lower_bound(distinct.begin(), distinct.end(), codes[(size_t)i]) -
                                      distinct.begin());
                cluster_id[i] = label[idx];
            } else {
                int64_t st, len;
                row_span(offsets, offset_width, i, &st, &len);
                cluster_id[i] = label[D + irregular.at(std::string((const char*)values + st, (size_t)len))];
            }
        }
    });
    return (int64_t)next;
}

int64_t oracle_umi_cluster(const void* offsets, int offset_width, const uint8_t* values,
                           const uint8_t* validity, int64_t validity_offset, int64_t n,
                           int umi_len, int max_distance, uint32_t* cluster_id, uint8_t* out_valid,
                           int* resolved_len) {
    return oracle_umi_cluster_mt(offsets, offset_width, values, validity, validity_offset, n, umi_len, max_distance,
                                 cluster_id, out_valid, resolved_len, 1);
}

// Entropy term table entry as the reference computes it: p = c/t; p*log2(p).
double oracle_plogp(uint32_t c, uint32_t t) {
    double p = (double)c / (double)t;
    return p * std::log2(p);
}

}  // extern "C"
