// assembly.cpp — H4.4 + H5: de Bruijn assembly of one read group (host C++).
//
// The reference runs this per polars group on the CPU (Rust + debruijn 0.3.4 +
// petgraph 0.7.1); so does this build, natively, fed by the GPU k-mer spectrum:
//   spectrum   rogtk_kmer_spectrum_host at min_coverage 0, once per effective k and
//              call: every observed k-mer with its count and the OR of its exts (an
//              ext always names an observed k-mer, so nothing is censored at 0).
//              Each (k, min_coverage) probe then applies CountFilter + censoring on
//              the host, so sweep / optimize never recount k-mers.
//   graph      nodes = valid k-mers in ascending order (the reference adds them in
//              BoomHashMap2 MPHF order, which cannot be reproduced: every choice the
//              node order decides is "parity unpinned" and documented below)
//   methods    fracture.rs:351-464
//     compression         compress_graph(stranded, SimpleCompress(sum)): maximal
//                         unambiguous paths from each still-available seed, left
//                         then right (debruijn compression, restated)
//     shortest_path       djfind.rs:78-304: petgraph DiGraph over the k-mer nodes,
//                         edge weight -ln((cov_from + cov_to) / 2), Dijkstra (petgraph
//                         visited-on-pop semantics, std BinaryHeap sift order),
//                         backtrack with eps 1e-9, path -> first + next[k-1..]
//     shortest_path_auto  djfind.rs:309-492: degree/coverage endpoint candidates,
//                         <= 100 pairs, score 0.6 len + 0.4 cov
//   assemble   fracture.rs:188-280 (auto_k, k > 64, min_length, only_largest =
//              max_by_key: the LAST longest contig in node order)
//   sweep      expressions.rs:880-955;  optimize  fracture_opt.rs:120-282
// Graph export (DOT / CSV files, export_graphs) is a file side effect and out of scope.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <map>
#include <set>
#include <thread>
#include <string>
#include <utility>
#include <vector>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

typedef unsigned __int128 u128;

int effective_k_h(int k) { return k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : k <= 32 ? 32 : 64; }

// fracture.rs:24-54 (usize 0 - 1 wraps in a release build and is clamped to 63)
int estimate_k_h(const std::vector<std::string>& seqs) {
    if (seqs.empty()) return 31;
    uint64_t total = 0, count = 0;
    for (const auto& s : seqs)
        if (!s.empty()) {
            total += s.size();
            count += 1;
        }
    if (count == 0) return 31;
    const int64_t k = (int64_t)std::round(((double)total / (double)count) / 3.0);
    uint64_t ku = (k % 2 == 0) ? (uint64_t)k - 1 : (uint64_t)k;
    return (int)std::min<uint64_t>(std::max<uint64_t>(ku, 11), 63);
}

// One group's column, kept on the host for spectra at several k.
struct GroupCol {
    std::vector<int64_t> offsets;
    std::vector<uint8_t> values;
    std::vector<uint8_t> validity;  // empty = all valid
    int64_t n = 0;
    std::vector<std::string> raw;   // non-null rows (expressions.rs:739-744)
};

struct Spectrum {
    int K = 0;
    int64_t nseq = 0;
    std::vector<u128> kmer;
    std::vector<uint8_t> ext;
    std::vector<uint16_t> cnt;
};

int load_group(const void* offsets, int ow, const uint8_t* values, int64_t values_len, const uint8_t* validity,
               int64_t voff, int64_t n, GroupCol* g) {
    ROGTK_REQUIRE(ow == 4 || ow == 8, ROGTK_E_INVALID, "offset_width must be 4 or 8");
    ROGTK_REQUIRE(n >= 0 && (n == 0 || offsets), ROGTK_E_INVALID, "assemble: bad offsets / n_rows");
    auto off = [&](int64_t r) -> int64_t {
        return ow == 4 ? (int64_t)((const int32_t*)offsets)[r] : ((const int64_t*)offsets)[r];
    };
    const int64_t base = n ? off(0) : 0, end = n ? off(n) : 0;
    ROGTK_REQUIRE(end <= values_len && base <= end, ROGTK_E_INVALID, "assemble: offsets exceed values_len");
    g->n = n;
    g->offsets.resize(n + 1);
    for (int64_t r = 0; r <= n; ++r) g->offsets[r] = n ? off(r) - base : 0;
    g->values.assign(values ? values + base : nullptr, values ? values + end : nullptr);
    if (g->values.empty()) g->values.push_back(0);
    g->validity.clear();
    if (validity) {
        g->validity.assign((size_t)(n + 7) / 8, 0);
        for (int64_t r = 0; r < n; ++r) {
            const int64_t b = voff + r;
            if ((validity[b >> 3] >> (b & 7)) & 1) g->validity[r >> 3] |= (uint8_t)(1u << (r & 7));
        }
    }
    g->raw.clear();
    for (int64_t r = 0; r < n; ++r) {
        if (!g->validity.empty() && !((g->validity[r >> 3] >> (r & 7)) & 1)) continue;
        g->raw.emplace_back((const char*)g->values.data() + g->offsets[r], (size_t)(g->offsets[r + 1] - g->offsets[r]));
    }
    return ROGTK_OK;
}

// GPU spectrum at min_coverage 0 for effective k K
int spectrum(const GroupCol& g, int K, Spectrum* out) {
    int64_t cap = 0;
    for (int64_t r = 0; r < g.n; ++r) {
        const int64_t len = g.offsets[r + 1] - g.offsets[r];
        if (len >= 4) cap += len - 3;
    }
    cap = std::max<int64_t>(cap, 1);
    std::vector<uint64_t> km((size_t)cap * 2);
    std::vector<uint8_t> ex((size_t)cap);
    std::vector<uint16_t> cn((size_t)cap);
    int64_t eo[2] = {0, 0}, st[5] = {0, 0, 0, 0, 0};
    if (int rc = rogtk_kmer_spectrum_host(g.offsets.data(), 8, g.values.data(), (int64_t)g.values.size(),
                                          g.validity.empty() ? nullptr : g.validity.data(), 0, g.n, nullptr, 0, K,
                                          0, 0, cap, km.data(), ex.data(), cn.data(), eo, st))
        return rc;
    const int64_t m = eo[1];
    out->K = K;
    out->nseq = st[1];
    out->kmer.resize(m);
    out->ext.assign(ex.begin(), ex.begin() + m);
    out->cnt.assign(cn.begin(), cn.begin() + m);
    for (int64_t i = 0; i < m; ++i) out->kmer[i] = ((u128)km[2 * i] << 64) | km[2 * i + 1];
    return ROGTK_OK;
}

// The preliminary graph of fracture.rs:343-348 for one min_coverage: valid k-mers
// (CountFilter) with exts censored to valid neighbours (remove_censored_exts).
struct Graph {
    int K = 0;
    u128 mask = 0;
    std::vector<u128> km;
    std::vector<uint8_t> ex;
    std::vector<uint16_t> cov;

    int64_t find(u128 x) const {
        auto it = std::lower_bound(km.begin(), km.end(), x);
        return (it != km.end() && *it == x) ? (int64_t)(it - km.begin()) : -1;
    }
    u128 ext_left(u128 x, int b) const { return (x >> 2) | ((u128)b << (2 * K - 2)); }
    u128 ext_right(u128 x, int b) const { return ((x << 2) | (u128)b) & mask; }
    std::string seq(int64_t i) const {
        std::string s((size_t)K, 'A');
        for (int j = 0; j < K; ++j) s[j] = "ACGT"[(int)((km[i] >> (2 * (K - 1 - j))) & 3)];
        return s;
    }
    int64_t size() const { return (int64_t)km.size(); }
};

Graph make_graph(const Spectrum& s, int64_t min_cov) {
    Graph g;
    g.K = s.K;
    g.mask = s.K == 64 ? ~(u128)0 : (((u128)1 << (2 * s.K)) - 1);
    for (size_t i = 0; i < s.kmer.size(); ++i)
        if ((int64_t)s.cnt[i] >= min_cov) {
            g.km.push_back(s.kmer[i]);
            g.ex.push_back(s.ext[i]);
            g.cov.push_back(s.cnt[i]);
        }
    for (int64_t i = 0; i < g.size(); ++i) {
        uint8_t ne = 0;
        for (int bit = 0; bit < 8; ++bit) {
            if (!((g.ex[i] >> bit) & 1)) continue;
            const u128 nb = bit < 4 ? g.ext_left(g.km[i], bit) : g.ext_right(g.km[i], bit - 4);
            if (g.find(nb) >= 0) ne |= (uint8_t)(1u << bit);
        }
        g.ex[i] = ne;
    }
    return g;
}

inline int popc4(unsigned x) { return __builtin_popcount(x & 0xFu); }
inline int ctz4(unsigned x) { return __builtin_ctz(x & 0xFu); }

// compress()'s walks without building every contig: the last longest path of at least
// min_len bases (assemble_graph's min_length + only_largest: max_by_key keeps the last
// maximum), as a string; false when none qualifies. Scratch buffers are per thread (the
// batched H5 calls it once per group). Same seeds, same order, same walks as compress().
// Neighbours by an open-addressing table of the group's k-mers (built once per group)
// instead of Graph::find's binary search: the walks look up ~2 neighbours per node.
struct KmerIndex {
    std::vector<u128> key;
    std::vector<int32_t> at;  // -1: empty
    uint64_t mask = 0;
    static uint64_t hash(u128 x) {
        const uint64_t h = (uint64_t)x ^ (uint64_t)(x >> 64) * 0x9E3779B97F4A7C15ull;
        return (h ^ (h >> 29)) * 0xBF58476D1CE4E5B9ull;
    }
    void build(const Graph& g) {
        size_t cap = 16;
        while (cap < 2 * (size_t)g.size()) cap <<= 1;
        key.resize(cap);
        at.assign(cap, -1);
        mask = cap - 1;
        for (int64_t i = 0; i < g.size(); ++i) {
            uint64_t h = hash(g.km[i]) & mask;
            while (at[h] >= 0) h = (h + 1) & mask;
            key[h] = g.km[i];
            at[h] = (int32_t)i;
        }
    }
    int64_t find(u128 x) const {
        for (uint64_t h = hash(x) & mask;; h = (h + 1) & mask) {
            if (at[h] < 0) return -1;
            if (key[h] == x) return at[h];
        }
    }
};

bool compress_largest(const Graph& g, int64_t min_len, std::string* out) {
    thread_local std::vector<char> avail;
    thread_local std::vector<int64_t> lpath, rpath, best;
    thread_local KmerIndex ix;
    const int64_t n = g.size();
    avail.assign((size_t)n, 1);
    ix.build(g);
    int64_t best_len = -1;
    for (int64_t seed = 0; seed < n; ++seed) {
        if (!avail[seed]) continue;
        avail[seed] = 0;
        lpath.clear();
        rpath.clear();
        for (int64_t cur = seed;;) {  // extend left
            const unsigned l = g.ex[cur] & 0xFu;
            if (popc4(l) != 1) break;
            const int64_t nx = ix.find(g.ext_left(g.km[cur], ctz4(l)));
            if (nx < 0 || !avail[nx] || popc4(g.ex[nx] >> 4) != 1) break;
            avail[nx] = 0;
            lpath.push_back(nx);
            cur = nx;
        }
        for (int64_t cur = seed;;) {  // extend right
            const unsigned r = g.ex[cur] >> 4;
            if (popc4(r) != 1) break;
            const int64_t nx = ix.find(g.ext_right(g.km[cur], ctz4(r)));
            if (nx < 0 || !avail[nx] || popc4(g.ex[nx] & 0xFu) != 1) break;
            avail[nx] = 0;
            rpath.push_back(nx);
            cur = nx;
        }
        const int64_t len = g.K + (int64_t)(lpath.size() + rpath.size());
        if (len < min_len || len < best_len) continue;
        best_len = len;
        best.assign(lpath.rbegin(), lpath.rend());
        best.push_back(seed);
        best.insert(best.end(), rpath.begin(), rpath.end());
    }
    if (best_len < 0) return false;
    *out = g.seq(best[0]);
    for (size_t i = 1; i < best.size(); ++i) out->push_back("ACGT"[(int)(g.km[best[i]] & 3)]);
    return true;
}

// ---------------------------------------------------- compression (fracture.rs:351-383)
std::vector<std::string> compress(const Graph& g) {
    const int64_t n = g.size();
    std::vector<char> avail((size_t)n, 1);
    std::vector<std::string> contigs;
    for (int64_t seed = 0; seed < n; ++seed) {
        if (!avail[seed]) continue;
        avail[seed] = 0;
        std::vector<int64_t> lpath, rpath;
        for (int64_t cur = seed;;) {  // extend left
            const unsigned l = g.ex[cur] & 0xFu;
            if (popc4(l) != 1) break;
            const int64_t nx = g.find(g.ext_left(g.km[cur], ctz4(l)));
            if (nx < 0 || !avail[nx] || popc4(g.ex[nx] >> 4) != 1) break;
            avail[nx] = 0;
            lpath.push_back(nx);
            cur = nx;
        }
        for (int64_t cur = seed;;) {  // extend right
            const unsigned r = g.ex[cur] >> 4;
            if (popc4(r) != 1) break;
            const int64_t nx = g.find(g.ext_right(g.km[cur], ctz4(r)));
            if (nx < 0 || !avail[nx] || popc4(g.ex[nx] & 0xFu) != 1) break;
            avail[nx] = 0;
            rpath.push_back(nx);
            cur = nx;
        }
        std::vector<int64_t> path(lpath.rbegin(), lpath.rend());
        path.push_back(seed);
        path.insert(path.end(), rpath.begin(), rpath.end());
        std::string s = g.seq(path[0]);
        for (size_t i = 1; i < path.size(); ++i) s.push_back("ACGT"[(int)(g.km[path[i]] & 3)]);
        if ((int64_t)s.size() >= g.K) contigs.push_back(std::move(s));
    }
    return contigs;
}

// --------------------------------------------- petgraph view (djfind.rs:78-121)
// Edges are added per node in ascending base order; petgraph iterates a node's
// outgoing and incoming edges newest-first, which the lists below reproduce.
struct PetGraph {
    std::vector<std::string> seq;
    std::vector<std::vector<std::pair<int64_t, double>>> out, in;  // newest first
};

PetGraph to_petgraph(const Graph& g) {
    PetGraph pg;
    const int64_t n = g.size();
    pg.seq.resize(n);
    pg.out.assign(n, {});
    pg.in.assign(n, {});
    for (int64_t i = 0; i < n; ++i) pg.seq[i] = g.seq(i);
    for (int64_t from = 0; from < n; ++from) {
        for (int b = 0; b < 4; ++b) {
            if (!((g.ex[from] >> (4 + b)) & 1)) continue;
            const int64_t to = g.find(g.ext_right(g.km[from], b));
            if (to < 0) continue;
            const double w = -std::log(((double)g.cov[from] + (double)g.cov[to]) / 2.0);
            pg.out[from].insert(pg.out[from].begin(), {to, w});
            pg.in[to].insert(pg.in[to].begin(), {from, w});
        }
    }
    return pg;
}

// petgraph::algo::dijkstra with std::collections::BinaryHeap<MinScored> (max-heap of
// reversed scores; push = sift_up, pop = swap last to root + sift_down_to_bottom)
struct MinHeap {
    std::vector<std::pair<double, int64_t>> d;
    static bool le(const std::pair<double, int64_t>& a, const std::pair<double, int64_t>& b) {
        return a.first >= b.first;  // a <= b in MinScored order
    }
    void sift_up(size_t start, size_t pos) {
        auto elem = d[pos];
        while (pos > start) {
            const size_t parent = (pos - 1) / 2;
            if (le(elem, d[parent])) break;
            d[pos] = d[parent];
            pos = parent;
        }
        d[pos] = elem;
    }
    void push(double s, int64_t v) {
        d.push_back({s, v});
        sift_up(0, d.size() - 1);
    }
    std::pair<double, int64_t> pop() {
        auto item = d.back();
        d.pop_back();
        if (!d.empty()) {
            std::swap(item, d[0]);
            const size_t end = d.size();
            size_t pos = 0, child = 1;
            auto elem = d[0];
            while (end >= 2 && child <= end - 2) {
                child += le(d[child], d[child + 1]) ? 1 : 0;
                d[pos] = d[child];
                pos = child;
                child = 2 * pos + 1;
            }
            if (child == end - 1) {
                d[pos] = d[child];
                pos = child;
            }
            d[pos] = elem;
            sift_up(0, pos);
        }
        return item;
    }
};

std::map<int64_t, double> dijkstra(const PetGraph& pg, int64_t start) {
    std::map<int64_t, double> scores;
    std::vector<char> visited(pg.seq.size(), 0);
    MinHeap h;
    scores[start] = 0.0;
    h.push(0.0, start);
    while (!h.d.empty()) {
        const auto [score, node] = h.pop();
        if (visited[node]) continue;
        for (const auto& [next, w] : pg.out[node]) {
            if (visited[next]) continue;
            const double ns = score + w;
            auto it = scores.find(next);
            if (it != scores.end()) {
                if (ns < it->second) {
                    it->second = ns;
                    h.push(ns, next);
                }
            } else {
                scores[next] = ns;
                h.push(ns, next);
            }
        }
        visited[node] = 1;
    }
    return scores;
}

// djfind.rs:157-247
bool shortest_path(const PetGraph& pg, const std::vector<int64_t>& starts, const std::vector<int64_t>& ends,
                   std::vector<int64_t>* best_path, double* best_weight) {
    bool found = false;
    double min_total = INFINITY;
    for (int64_t start : starts) {
        const auto dist = dijkstra(pg, start);
        for (int64_t end : ends) {
            auto de = dist.find(end);
            if (de == dist.end()) continue;
            const double total = de->second;
            if (!(total < min_total)) continue;
            std::vector<int64_t> path{end};
            int64_t current = end;
            bool valid = false;
            int iterations = 0;
            while (current != start) {
                if (++iterations > 1000) break;
                int64_t best_prev = -1;
                double best_dist = INFINITY;
                const double cur_dist = dist.at(current);
                for (const auto& [nb, w] : pg.in[current]) {
                    auto dn = dist.find(nb);
                    if (dn == dist.end()) continue;
                    // find_edge(nb, current): the first (newest) outgoing edge of nb to current
                    double ew = w;
                    for (const auto& [t2, w2] : pg.out[nb])
                        if (t2 == current) {
                            ew = w2;
                            break;
                        }
                    if (std::fabs(dn->second + ew - cur_dist) < 1e-9 && dn->second < best_dist) {
                        best_dist = dn->second;
                        best_prev = nb;
                    }
                }
                if (best_prev < 0) break;
                path.push_back(best_prev);
                current = best_prev;
                if (current == start) valid = true;
            }
            // start == end: the reference's loop never runs and the path stays invalid
            if (valid) {
                std::reverse(path.begin(), path.end());
                *best_path = path;
                *best_weight = total;
                min_total = total;
                found = true;
            }
        }
    }
    return found;
}

std::string concat_path(const PetGraph& pg, const std::vector<int64_t>& path, int K) {
    if (path.empty()) return std::string();
    std::string s = pg.seq[path[0]];
    for (size_t i = 1; i < path.size(); ++i) s += pg.seq[path[i]].substr((size_t)K - 1);
    return s;
}

// djfind.rs:257-304 (errors -> no contig, fracture.rs:414-417)
bool path_assembly(const Graph& g, const PetGraph& pg, const std::string& sa, const std::string& ea, std::string* out) {
    std::vector<int64_t> starts, ends;
    for (int64_t i = 0; i < (int64_t)pg.seq.size(); ++i) {
        const std::string& s = pg.seq[i];
        if (s.compare(0, sa.size(), sa) == 0 && s.size() >= sa.size()) starts.push_back(i);
        if (s.size() >= ea.size() && s.compare(s.size() - ea.size(), ea.size(), ea) == 0) ends.push_back(i);
    }
    if (starts.empty() || ends.empty()) return false;
    std::vector<int64_t> path;
    double w = 0;
    if (!shortest_path(pg, starts, ends, &path, &w)) return false;
    *out = concat_path(pg, path, g.K);
    return true;
}

// djfind.rs:309-492
bool auto_path_assembly(const Graph& g, const PetGraph& pg, std::string* out) {
    const int64_t n = g.size();
    double sum = 0;
    for (int64_t i = 0; i < n; ++i) sum += (double)g.cov[i];
    const double avg = sum / (double)n;  // NaN for an empty graph (no candidates follow)
    const double thr_f = std::fmax(avg * 0.1, 1.0);
    const uint16_t thr = (uint16_t)std::min(65535.0, std::max(0.0, std::floor(thr_f)));
    std::vector<int64_t> sc, ec;
    for (int64_t i = 0; i < n; ++i) {
        if (g.cov[i] < thr) continue;
        const int in_deg = (int)pg.in[i].size(), out_deg = (int)pg.out[i].size();
        if (in_deg == 0 && out_deg > 0) sc.push_back(i);
        if (out_deg == 0 && in_deg > 0) ec.push_back(i);
    }
    if (sc.empty() || ec.empty()) return false;
    if (sc.size() == 1 && ec.size() == 1) return path_assembly(g, pg, pg.seq[sc[0]], pg.seq[ec[0]], out);
    int evaluated = 0;
    bool have = false;
    double best_score = 0;
    for (int64_t s : sc) {
        for (int64_t e : ec) {
            if (evaluated >= 100) break;
            ++evaluated;
            // nodes whose sequence contains the candidate's (all length K: equality)
            std::vector<int64_t> starts{s}, ends{e};
            std::vector<int64_t> path;
            double w = 0;
            if (!shortest_path(pg, starts, ends, &path, &w)) continue;
            double plen = 0;
            for (int64_t v : path) plen += (double)pg.seq[v].size();
            const double mean_cov = 1.0 / (w / (double)path.size());
            const double score = 0.6 * std::fmin(plen / 5000.0, 1.0) + 0.4 * std::fmin(mean_cov / 100.0, 1.0);
            if (!have || score > best_score) {
                have = true;
                best_score = score;
                *out = concat_path(pg, path, g.K);
            }
        }
    }
    return have;
}

enum Method { M_COMPRESSION = 0, M_SHORTEST = 1, M_AUTO = 2 };

// AssemblyMethod::from_str (djfind.rs:32-58) + the expr-level checks
int parse_method(const char* method, const char* sa, const char* ea, int* out) {
    ROGTK_REQUIRE(method, ROGTK_E_INVALID, "method is NULL");
    const std::string m(method);
    if (m == "compression") {
        ROGTK_REQUIRE(!sa && !ea, ROGTK_E_INVALID, "Anchor sequences should not be provided for compression method");
        *out = M_COMPRESSION;
    } else if (m == "shortest_path") {
        ROGTK_REQUIRE(sa && ea, ROGTK_E_INVALID, "Both start_anchor and end_anchor are required for shortest_path method");
        *out = M_SHORTEST;
    } else if (m == "shortest_path_auto") {
        ROGTK_REQUIRE(!sa && !ea, ROGTK_E_INVALID,
                      "Anchor sequences should not be provided for shortest_path_auto method");
        *out = M_AUTO;
    } else {
        set_error("Invalid assembly method. Must be 'compression', 'shortest_path', or 'shortest_path_auto'");
        return ROGTK_E_INVALID;
    }
    return ROGTK_OK;
}

// fracture.rs:343-464 from the preliminary graph on: the method's contigs, min_length,
// only_largest (max_by_key: the last longest)
void assemble_graph(const Graph& g, int method, const std::string& sa, const std::string& ea, int only_largest,
                    int64_t min_length, std::vector<std::string>* out) {
    out->clear();
    std::vector<std::string> cs;
    if (method == M_COMPRESSION) {
        cs = compress(g);
    } else {
        const PetGraph pg = to_petgraph(g);
        std::string c;
        const bool ok = method == M_SHORTEST ? path_assembly(g, pg, sa, ea, &c) : auto_path_assembly(g, pg, &c);
        if (ok) cs.push_back(c);
    }
    for (auto& c : cs)
        if ((int64_t)c.size() >= std::max<int64_t>(min_length, 0)) out->push_back(c);
    if (out->empty() || !only_largest) return;
    size_t best = 0;  // max_by_key: the last maximum
    for (size_t i = 1; i < out->size(); ++i)
        if ((*out)[i].size() >= (*out)[best].size()) best = i;
    std::string keep = (*out)[best];
    out->assign(1, keep);
}

// assemble_sequences (fracture.rs:188-280) over a prepared group with a spectrum cache
struct Assembler {
    GroupCol col;
    std::map<int, Spectrum> cache;

    int contigs(int k, int64_t min_cov, int method, const std::string& sa, const std::string& ea, int only_largest,
                int64_t min_length, int auto_k, std::vector<std::string>* out) {
        out->clear();
        if (auto_k) k = estimate_k_h(col.raw);
        if (k > 64) return ROGTK_OK;  // fracture.rs:211-214
        const int K = effective_k_h(k);
        auto it = cache.find(K);
        if (it == cache.end()) {
            Spectrum s;
            if (int rc = spectrum(col, K, &s)) return rc;
            it = cache.emplace(K, std::move(s)).first;
        }
        const Spectrum& s = it->second;
        if (s.nseq == 0) return ROGTK_OK;  // no valid sequences
        assemble_graph(make_graph(s, min_cov), method, sa, ea, only_largest, min_length, out);
        return ROGTK_OK;
    }
};

int copy_out(const std::string& s, char* out, int64_t cap, int64_t* len) {
    *len = (int64_t)s.size();
    ROGTK_REQUIRE((int64_t)s.size() <= cap || !out, ROGTK_E_OVERFLOW, "output buffer of %lld bytes < %lld",
                  (long long)cap, (long long)s.size());
    if (out && !s.empty()) std::memcpy(out, s.data(), s.size());
    return ROGTK_OK;
}

// The batched H5 result (rogtk_assemble_groups_host): one string per group, the group's
// contigs joined by '\n' (assemble_sequences_expr's output row, expressions.rs:695-760).
struct AssemblyResult {
    std::vector<int64_t> offsets;  // n_groups + 1
    std::string values;
    std::vector<int64_t> n_contigs;  // per group
};

}  // namespace
}  // namespace rogtk

using namespace rogtk;

extern "C" {

int rogtk_assemble_host(const void* offsets, int offset_width, const uint8_t* values, int64_t values_len,
                        const uint8_t* validity, int64_t validity_offset, int64_t n_rows, int k,
                        int64_t min_coverage, const char* method, const char* start_anchor, const char* end_anchor,
                        int only_largest, int64_t min_length, int auto_k, char* out, int64_t out_cap,
                        int64_t* out_len, int64_t* n_contigs) {
    ROGTK_REQUIRE(out_len && n_contigs, ROGTK_E_INVALID, "assemble: out_len / n_contigs are NULL");
    ROGTK_REQUIRE(k >= 0 && min_coverage >= 0, ROGTK_E_INVALID, "assemble: k and min_coverage must be >= 0");
    int m = 0;
    if (int rc = parse_method(method, start_anchor, end_anchor, &m)) return rc;
    Assembler a;
    if (int rc = load_group(offsets, offset_width, values, values_len, validity, validity_offset, n_rows, &a.col))
        return rc;
    std::vector<std::string> cs;
    if (int rc = a.contigs(k, min_coverage, m, start_anchor ? start_anchor : "", end_anchor ? end_anchor : "",
                           only_largest, min_length, auto_k, &cs))
        return rc;
    std::string joined;
    for (size_t i = 0; i < cs.size(); ++i) {
        if (i) joined.push_back('\n');
        joined += cs[i];
    }
    *n_contigs = (int64_t)cs.size();
    return copy_out(joined, out, out_cap, out_len);
}

int rogtk_assembly_sweep_host(const void* offsets, int offset_width, const uint8_t* values, int64_t values_len,
                              const uint8_t* validity, int64_t validity_offset, int64_t n_rows, int64_t k_start,
                              int64_t k_end, int64_t k_step, int64_t cov_start, int64_t cov_end, int64_t cov_step,
                              const char* method, const char* start_anchor, const char* end_anchor, int64_t cap,
                              int64_t* out_k, int64_t* out_cov, int64_t* out_len, int64_t* n_out) {
    ROGTK_REQUIRE(n_out, ROGTK_E_INVALID, "sweep: n_out is NULL");
    ROGTK_REQUIRE(k_step > 0 && cov_step > 0, ROGTK_E_INVALID, "sweep: step_by(0)");
    int m = 0;
    if (int rc = parse_method(method, start_anchor, end_anchor, &m)) {
        set_error("Invalid assembly method: %s", rogtk_last_error());
        return rc;
    }
    Assembler a;
    if (int rc = load_group(offsets, offset_width, values, values_len, validity, validity_offset, n_rows, &a.col))
        return rc;
    int64_t n = 0;
    for (int64_t k = k_start; k <= k_end; k += k_step) {
        for (int64_t c = cov_start; c <= cov_end; c += cov_step) {
            std::vector<std::string> cs;
            int64_t len = 0;
            if (int rc = a.contigs((int)std::min<int64_t>(k, 0x7FFFFFFF), c, m, start_anchor ? start_anchor : "",
                                   end_anchor ? end_anchor : "", 1, -1, 0, &cs))
                return rc;  // a device failure, not an assembly outcome
            if (!cs.empty()) len = (int64_t)cs[0].size();
            if (n < cap && out_k && out_cov && out_len) {
                out_k[n] = k;
                out_cov[n] = c;
                out_len[n] = len;
            }
            ++n;
        }
    }
    *n_out = n;
    ROGTK_REQUIRE(n <= cap, ROGTK_E_OVERFLOW, "sweep: %lld rows exceed capacity %lld", (long long)n, (long long)cap);
    return ROGTK_OK;
}

int rogtk_assembly_optimize_host(const void* offsets, int offset_width, const uint8_t* values, int64_t values_len,
                                 const uint8_t* validity, int64_t validity_offset, int64_t n_rows,
                                 const char* method, const char* start_anchor, const char* end_anchor,
                                 int64_t start_k, int64_t start_min_coverage, int64_t max_iterations, int explore_k,
                                 int prioritize_length, char* contig, int64_t contig_cap, int64_t* contig_len,
                                 uint32_t* out4) {
    ROGTK_REQUIRE(contig_len && out4, ROGTK_E_INVALID, "optimize: contig_len / out4 are NULL");
    ROGTK_REQUIRE(start_anchor, ROGTK_E_INVALID, "start_anchor is required");
    ROGTK_REQUIRE(end_anchor, ROGTK_E_INVALID, "end_anchor is required");
    int m = 0;
    if (int rc = parse_method(method, start_anchor, end_anchor, &m)) return rc;
    Assembler a;
    if (int rc = load_group(offsets, offset_width, values, values_len, validity, validity_offset, n_rows, &a.col))
        return rc;
    const std::string sa(start_anchor), ea(end_anchor);
    const uint32_t nin = (uint32_t)a.col.raw.size();
    struct Res {
        std::string contig;
        int64_t k, cov;
        bool anchors;
    };
    auto run = [&](int64_t k, int64_t c, Res* r) -> int {
        std::vector<std::string> cs;
        if (int rc = a.contigs((int)std::min<int64_t>(k, 0x7FFFFFFF), c, m, sa, ea, 1, -1, 0, &cs)) return rc;
        r->contig = cs.empty() ? std::string() : cs[0];
        r->k = k;
        r->cov = c;
        r->anchors = r->contig.find(sa) != std::string::npos && r->contig.find(ea) != std::string::npos;
        return ROGTK_OK;
    };
    // fracture_opt.rs:120-228
    std::set<std::pair<int64_t, int64_t>> tested{{start_k, start_min_coverage}};
    bool have_anch = false, have_len = false, done = false;
    Res best_anch, best_len, cur;
    int rc = run(start_k, start_min_coverage, &cur);
    if (rc == ROGTK_OK) {
        if (cur.anchors) {
            best_anch = cur;
            have_anch = true;
        }
        best_len = cur;
        have_len = true;
        struct PathS {
            int64_t k, cov, length, steps;
        };
        std::vector<PathS> paths{{cur.k, cur.cov, (int64_t)cur.contig.size(), 0}};
        const int ndirs = explore_k ? 4 : 2;  // West, East, North, South
        for (int64_t it = 0; it < max_iterations && !done && rc == ROGTK_OK; ++it) {
            std::vector<PathS> next;
            for (const auto& p : paths) {
                if (done || rc) break;
                for (int d = 0; d < ndirs; ++d) {
                    int64_t k = p.k, c = p.cov;
                    if (d == 0) {
                        if (c <= 1) continue;
                        c -= 1;
                    } else if (d == 1) {
                        c += 1;
                    } else if (d == 2) {
                        if (k <= 4) continue;
                        k -= 1;
                    } else {
                        if (k >= 64) continue;
                        k += 1;
                    }
                    if (tested.count({k, c})) continue;
                    tested.insert({k, c});
                    Res r;
                    if ((rc = run(k, c, &r))) break;
                    if (r.anchors && (!have_anch || r.contig.size() > best_anch.contig.size())) {
                        best_anch = r;
                        have_anch = true;
                    }
                    if (!have_len || r.contig.size() > best_len.contig.size()) {
                        best_len = r;
                        have_len = true;
                    }
                    if (r.anchors && !prioritize_length) {  // early return
                        best_anch = r;
                        have_anch = true;
                        done = true;
                        break;
                    }
                    if (!r.contig.empty()) {
                        const int64_t len = (int64_t)r.contig.size();
                        next.push_back({k, c, len, len > p.length ? 0 : p.steps + 1});
                    }
                }
            }
            if (done || rc) break;
            if (next.empty()) break;
            std::stable_sort(next.begin(), next.end(), [](const PathS& x, const PathS& y) {
                return x.length != y.length ? x.length > y.length : x.steps < y.steps;
            });
            if (next.size() > 4) next.resize(4);
            paths = next;
        }
    }
    if (rc) return rc;  // a device failure, not an assembly outcome
    const bool ok = done || (prioritize_length ? have_len : have_anch);
    const Res& r = done ? best_anch : (prioritize_length ? best_len : best_anch);
    if (!ok) {  // Ok(None) | Err(_) -> empty row with the input count
        out4[0] = out4[1] = out4[2] = 0;
        out4[3] = nin;
        return copy_out(std::string(), contig, contig_cap, contig_len);
    }
    out4[0] = (uint32_t)r.k;
    out4[1] = (uint32_t)r.cov;
    out4[2] = (uint32_t)r.contig.size();
    out4[3] = nin;
    return copy_out(r.contig, contig, contig_cap, contig_len);
}

// Round 6: H5 over every group of a spectrum call at once. The device spectra at the
// call's min_coverage are the preliminary graphs (CountFilter + exts censored to valid
// neighbours = make_graph of the min_coverage 0 spectrum, fracture.rs:343-348), so each
// group's graph is its entry slice; groups are assembled on n_threads host threads
// (atomic work counter, 64 groups per take), each writing its own string.
int rogtk_assemble_groups_host(const uint64_t* kmers, const uint8_t* exts, const uint16_t* counts,
                               const int64_t* entry_offsets, const int64_t* group_stats, int64_t n_groups,
                               const char* method, const char* start_anchor, const char* end_anchor,
                               int only_largest, int64_t min_length, int n_threads, void** result) {
    ROGTK_REQUIRE(result, ROGTK_E_INVALID, "assemble_groups: result is NULL");
    *result = nullptr;
    ROGTK_REQUIRE(n_groups >= 0 && (n_groups == 0 || (entry_offsets && group_stats)), ROGTK_E_INVALID,
                  "assemble_groups: bad groups");
    const int64_t total = n_groups ? entry_offsets[n_groups] : 0;
    ROGTK_REQUIRE(total == 0 || (kmers && exts && counts), ROGTK_E_INVALID, "assemble_groups: NULL spectrum arrays");
    int m = 0;
    if (int rc = parse_method(method, start_anchor, end_anchor, &m)) return rc;
    const std::string sa(start_anchor ? start_anchor : ""), ea(end_anchor ? end_anchor : "");
    std::vector<std::string> per((size_t)n_groups);
    std::vector<int64_t> nc((size_t)n_groups, 0);
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        std::vector<std::string> cs;
        Graph gr;  // reused across the thread's groups (no allocation once grown)
        for (;;) {
            const int64_t g0 = next.fetch_add(64);
            if (g0 >= n_groups) return;
            for (int64_t g = g0; g < std::min<int64_t>(n_groups, g0 + 64); ++g) {
                const int K = (int)group_stats[5 * g];
                if (K <= 0 || group_stats[5 * g + 1] == 0) continue;  // k > 64 / no valid sequences
                gr.K = K;
                gr.mask = K == 64 ? ~(u128)0 : (((u128)1 << (2 * K)) - 1);
                const int64_t a = entry_offsets[g], b = entry_offsets[g + 1];
                gr.km.resize((size_t)(b - a));
                for (int64_t i = a; i < b; ++i) gr.km[i - a] = ((u128)kmers[2 * i] << 64) | kmers[2 * i + 1];
                gr.ex.assign(exts + a, exts + b);
                gr.cov.assign(counts + a, counts + b);
                if (m == M_COMPRESSION && only_largest) {  // the expression's default: one string
                    std::string& o = per[g];
                    nc[g] = compress_largest(gr, std::max<int64_t>(min_length, 0), &o) ? 1 : 0;
                    continue;
                }
                assemble_graph(gr, m, sa, ea, only_largest, min_length, &cs);
                nc[g] = (int64_t)cs.size();
                std::string& o = per[g];
                for (size_t i = 0; i < cs.size(); ++i) {
                    if (i) o.push_back('\n');
                    o += cs[i];
                }
            }
        }
    };
    const int T = std::max(1, std::min<int>(n_threads > 0 ? n_threads : 16, (int)((n_groups + 63) / 64)));
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
    auto* r = new AssemblyResult();
    r->offsets.resize((size_t)n_groups + 1);
    r->offsets[0] = 0;
    for (int64_t g = 0; g < n_groups; ++g) r->offsets[g + 1] = r->offsets[g] + (int64_t)per[g].size();
    r->values.reserve((size_t)r->offsets[n_groups]);
    for (auto& x : per) r->values += x;
    r->n_contigs = std::move(nc);
    *result = r;
    return ROGTK_OK;
}

int rogtk_assembly_result_sizes(const void* result, int64_t* n_groups, int64_t* values_len) {
    ROGTK_REQUIRE(result && n_groups && values_len, ROGTK_E_INVALID, "assembly_result_sizes: NULL argument");
    const auto* r = static_cast<const AssemblyResult*>(result);
    *n_groups = (int64_t)r->n_contigs.size();
    *values_len = (int64_t)r->values.size();
    return ROGTK_OK;
}

int rogtk_assembly_result_copy(const void* result, int64_t* offsets, char* values, int64_t* n_contigs) {
    ROGTK_REQUIRE(result, ROGTK_E_INVALID, "assembly_result_copy: NULL result");
    const auto* r = static_cast<const AssemblyResult*>(result);
    if (offsets) std::memcpy(offsets, r->offsets.data(), r->offsets.size() * 8);
    if (values && !r->values.empty()) std::memcpy(values, r->values.data(), r->values.size());
    if (n_contigs && !r->n_contigs.empty()) std::memcpy(n_contigs, r->n_contigs.data(), r->n_contigs.size() * 8);
    return ROGTK_OK;
}

int rogtk_assembly_result_free(void* result) {
    delete static_cast<AssemblyResult*>(result);
    return ROGTK_OK;
}

}  // extern "C"
