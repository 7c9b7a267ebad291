// rogtk_internal.h — shared declarations of librogtk_hip.so (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <vector>

#include "../../include/rogtk_hip.h"

namespace rogtk {

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

#define ROGTK_HIP_CHECK(expr)                                                                    \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) {                                                                  \
            ::rogtk::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                               __LINE__);                                                        \
            return ROGTK_E_HIP;                                                                  \
        }                                                                                        \
    } while (0)

#define ROGTK_REQUIRE(cond, code, ...)        \
    do {                                      \
        if (!(cond)) {                        \
            ::rogtk::set_error(__VA_ARGS__);  \
            return (code);                    \
        }                                     \
    } while (0)

// ------------------------------------------------------------- profiling
enum KernelId {
    K_STAGE = 0,
    K_SCORE_PACKED,
    K_SCORE_ROWS,
    K_MARK,
    K_BITMAP,
    K_SCAN,
    K_COMPACT,
    K_UNION,
    K_FLATTEN,
    K_LABEL,
    K_ASSIGN,
    K_IRREGULAR,
    K_BAM_FIELDS,
    K_BAM_SCAN,
    K_BAM_FILL,
    K_PACK_READS,
    K_ROW_GATHER,
    K_KMER_LDS,
    K_RESOLVE,  // the whole resolve chain of one batch (first launch to last, its stream)
    K_KMER_MZ,  // the minimizer filter of the k-mer spectra (round 4)
    // round 5: single kernels of the C2 step, each timed on its own dispatch packet
    K_K_SLICE_BUCKET,
    K_K_SLICE_MARK,
    K_K_OR_PARTIALS,
    K_K_SCAN_RT,
    K_K_LOCAL_CC,
    K_K_HOOK,
    K_K_JUMP,
    K_K_ROOTS,
    K_K_WORD_LABEL,
    // round 6: the fused pack + grouped staging of C3 (was timed as K_ROW_GATHER) and the
    // wave-per-group k-mer kernel
    K_PACK_GATHER,
    K_KMER_WAVE,
    K_COUNT_
};
extern const char* const kKernelNames[K_COUNT_];

bool profiling_on();
// Brackets one launch with HIP events on `stream` when profiling is enabled.
// exact = true: the events are not recorded on the stream; the launcher attaches them to
// the kernel's dispatch packet (hipExtLaunchKernelGGL(..., start(), stop(), ...)), so the
// elapsed time is the kernel's own execution, as in rocprofv3's kernel trace.
class ProfScope;
// One launch with its own exact events (kernel execution time, as rocprofv3's kernel trace)
// when profiling is on and ID is selected; a plain launch otherwise.
// A stream-ordering event armed by rogtk_event_attach_next rides on the next such launch's
// dispatch packet instead of a marker packet of its own (when that launch is not being
// timed; a timed launch records it right behind).
#define ROGTK_TIMED_LAUNCH(ID, KERNEL, GRID, BLOCK, LDS, S, ...)                                     \
    do {                                                                                           \
        ::rogtk::ProfScope pk_(ID, S, true);                                                       \
        hipEvent_t att_ = ::rogtk::take_attached_event();                                          \
        hipExtLaunchKernelGGL(KERNEL, GRID, BLOCK, LDS, S, pk_.start(), pk_.stop() ? pk_.stop() : att_, 0, \
                              __VA_ARGS__);                                                        \
        if (att_ && pk_.stop()) (void)hipEventRecord(att_, S);                                     \
    } while (0)
// the event armed on this thread (cleared), or nullptr; arm_attached_event re-arms one for
// the next launch, attached_event_taken: whether the last armed one rode on a launch
hipEvent_t take_attached_event();
void arm_attached_event(hipEvent_t e);
bool attached_event_taken();
void set_attached_taken();
class ProfScope {
   public:
    ProfScope(KernelId id, hipStream_t stream, bool exact = false);
    ~ProfScope();
    hipEvent_t start() const { return start_; }
    hipEvent_t stop() const { return stop_; }

   private:
    KernelId id_;
    hipStream_t stream_;
    bool exact_ = false;
    hipEvent_t start_ = nullptr;
    hipEvent_t stop_ = nullptr;
};

// In-kernel span timing (profiling only): a kernel given a non-NULL tspan writes, from
// thread 0 of every workgroup, the device wall clock (wall_clock64, constant rate) at
// entry and, after a final barrier, at exit; span_end() reduces max(exit) - min(entry),
// the kernel's execution span as rocprofv3's kernel trace sees it, without the stream
// events' own fences. span_begin returns NULL when the kernel is not being profiled.
uint64_t* span_begin(KernelId id, int64_t n_blocks, hipStream_t s);
void span_end(KernelId id, uint64_t* tspan, int64_t n_blocks, hipStream_t s);
#ifdef __HIP__
__device__ __forceinline__ void span_enter(uint64_t* tspan) {
    if (tspan && threadIdx.x == 0) tspan[2 * blockIdx.x] = wall_clock64();
}
__device__ __forceinline__ void span_exit(uint64_t* tspan) {
    if (tspan) {
        __syncthreads();
        if (threadIdx.x == 0) tspan[2 * blockIdx.x + 1] = wall_clock64();
    }
}
#endif

// ------------------------------------------------- entropy / ratio tables
// Triangular table T[t][c] = fl(fl(c/t) * log2(fl(c/t))) computed on the host
// with glibc log2 (the function Rust's f64::log2 resolves to), T[t][0] = 0.
__host__ __device__ inline int64_t lut_index(int64_t t, int64_t c) { return t * (t + 1) / 2 + c; }
double plogp_host(uint32_t c, uint32_t t);
// Device copy covering totals 0..max_total on the current device.
int lut_ensure(int64_t max_total, const double** dev, int64_t* covered);

constexpr int kMaxPackedLen = 16;

// Streaming (non-temporal) vector accesses for data touched once per kernel (the code
// stream, the per-row outputs), so that the randomly accessed tables of the same
// kernel keep their L2 lines. ROGTK_NT=0 builds plain accesses (A/B).
#ifndef ROGTK_NT
#define ROGTK_NT 1
#endif
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef double f64x2_t __attribute__((ext_vector_type(2)));
template <class V>
__device__ __forceinline__ V stream_load(const V* p) {
#if ROGTK_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
template <class V>
__device__ __forceinline__ void stream_store(V v, V* p) {
#if ROGTK_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
// Word label (H3 assign): one u32 per 64-code word, written by k_word_label and read by
// k_assign, k_lookup and the fused score + assign:
//   0xFFFFFFFF          no word label: every code of the word is labelled per code;
//   bit 31 clear        the label of every code of the word;
//   bits 31 and 30 set  the label (bits 0..23) of every code but one exception code,
//                       whose bit in the word is bits 24..29 (no mask load);
//   bits 31, 29 set, 30 clear: the label (bits 0..16) of every code but two exception
//                       codes, whose bits are bits 17..22 and 23..28 (no mask load);
//   bit 31 set, 30, 29 clear: the label (bits 0..28) of the codes outside the word's
//                       exception mask wexc[word].
// Returns the code's label, or 0xFFFFFFFF when the code is labelled per code (the
// exceptions). (Round 4 measured keeping the inline forms' exception labels in wexc
// instead of the per-code table: k_assign 100 -> 125-130 us; removed in round 5.)
__device__ __forceinline__ uint32_t decode_word_label(uint32_t wl, const uint64_t* __restrict__ wexc, uint64_t c) {
    if (wl == 0xFFFFFFFFu || !(wl >> 31)) return wl;
    const uint32_t b = (uint32_t)(c & 63);
    if ((wl >> 30) & 1u) return b != ((wl >> 24) & 63u) ? (wl & 0xFFFFFFu) : 0xFFFFFFFFu;
    if ((wl >> 29) & 1u)
        return b != ((wl >> 17) & 63u) && b != ((wl >> 23) & 63u) ? (wl & 0x1FFFFu) : 0xFFFFFFFFu;
    return ((wexc[c >> 6] >> b) & 1ull) ? 0xFFFFFFFFu : (wl & 0x1FFFFFFFu);
}

// the score kernel's 52 B/row of outputs (ROGTK_NT_SCORE_STORE=0: plain stores)
#ifndef ROGTK_NT_SCORE_STORE
#define ROGTK_NT_SCORE_STORE 1
#endif
template <class V>
__device__ __forceinline__ void score_store(V v, V* p) {
#if ROGTK_NT_SCORE_STORE
    stream_store(v, p);
#else
    *p = v;
#endif
}

// Per-call constants of the packed kernel (passed by value as a kernel argument).
struct PackedParams {
    double sh[kMaxPackedLen + 1];    // plogp(c, L)
    double di[kMaxPackedLen + 1];    // plogp(c, L-1)
    double ling[kMaxPackedLen + 1];  // u / min(L-2, 64)
    double frac[kMaxPackedLen + 1];  // k / L
    int L;
    int ham_mode;  // 0 none, 1 compare, 2 byte-length mismatch (u32::MAX / false)
    uint32_t tcode, cmplo, always_mismatch, max_distance;
};

struct ScoreOut {
    double* sh;
    double* ling;
    double* homo;
    double* di;
    uint32_t* longest;
    double* dust;
    double* comb;
};

inline ScoreOut to_score_out(const rogtk_umi_scores* s) {
    if (!s) return ScoreOut{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    return ScoreOut{s->shannon_entropy,      s->linguistic_complexity, s->homopolymer_fraction,
                    s->dinucleotide_entropy, s->longest_homopolymer_run, s->dust_score,
                    s->combined_score};
}
inline bool any_score(const ScoreOut& o) {
    return o.sh || o.ling || o.homo || o.di || o.longest || o.dust || o.comb;
}

// Host-side encoding of a Hamming target against packed UMIs of length L
// (expressions.rs:1057-1063 byte-length check + chars().zip()).
void encode_target(const uint8_t* target, int64_t target_len, int L, uint32_t max_distance,
                   PackedParams* p);
int build_packed_params(int L, PackedParams* p);

// Tables of a fused score + assign (k_score_packed<..., ASG>): a resolved cluster
// workspace's word labels, exception masks and per-code labels, and the id output.
struct AssignIn {
    const uint32_t* wlab;
    const uint64_t* wexc;
    const uint32_t* labelcode;
    uint32_t* out;  // nullptr: no assign in the score pass
};

// ------------------------------------------------------ kernel launchers
int launch_stage(const void* offsets, int offset_width, const uint8_t* values,
                 const uint8_t* validity, int64_t validity_offset, int64_t n, int L,
                 uint32_t* codes, uint64_t* regular_bits, int64_t* irregular_rows,
                 unsigned long long* n_irregular, hipStream_t s);
int launch_score_packed(const uint32_t* codes, const uint64_t* regular_bits, int64_t n,
                        const PackedParams& p, const ScoreOut& o, uint32_t* hd, uint64_t* hw, hipStream_t s,
                        const AssignIn* asg = nullptr);
int launch_score_rows(const void* offsets, int offset_width, const uint8_t* values,
                      const int64_t* rows, const int64_t* n_rows_dev, int64_t max_rows,
                      const double* lut, int64_t lut_max, const ScoreOut& o,
                      const uint8_t* target_dev, int64_t target_len, int ham, uint32_t max_distance,
                      uint32_t* hd, uint64_t* hw, hipStream_t s);

// Cluster workspace layout: a pure function of (L, max_distinct).
struct ClusterLayout {
    int L;
    int64_t max_distinct;
    uint64_t nbits;      // 4^L codes
    int64_t words;       // bitmap words over code space
    int64_t blocks;      // scan blocks over code-space words (1024 words each)
    int64_t rwords;      // root-bitmap words over index space
    int64_t rblocks;     // root-scan workgroups over index-space words (kRootWords each)
    bool label_by_code;  // dense label table indexed by code (L <= 13)
    // byte offsets into the workspace
    int64_t off_stats, off_presence, off_bitmap, off_rt, off_wpref, off_blksum, off_blkoff, off_D, off_f, off_ur,
        off_rbits, off_lroot, off_rpref, off_rblksum, off_rblkoff, off_labelcode, off_ilab, off_active,
        active_words, off_lb, total;
};
int cluster_layout(int L, int64_t max_distinct, ClusterLayout* out);

// Grow-only device buffer owned by a host-side context.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    std::vector<void*> retired;  // outgrown allocations, freed with the buffer
    ~DevBuf() {
        if (p) hipFree(p);
        for (void* q : retired) hipFree(q);
    }
    // A buffer that grows may still be read by kernels enqueued earlier on any stream (the
    // BAM device path never waits for the GPU inside a file), so the outgrown allocation is
    // retired, not freed: no device-wide drain on the host path. A regrown buffer takes
    // 1.5x, so the retired ones together stay below twice the live one.
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return ROGTK_OK;
        size_t grow = 0;
        if (p) {
            retired.push_back(p);
            p = nullptr;
            grow = cap + cap / 2;
            cap = 0;
        }
        size_t want = std::max<size_t>(std::max(bytes, grow), 256);
        want = (want + 255) / 256 * 256;
        ROGTK_HIP_CHECK(hipMalloc(&p, want));
        cap = want;
        return ROGTK_OK;
    }
    // Frees the outgrown allocations (a long-lived context otherwise keeps up to
    // ~2x its live buffers in HBM). Only where the caller has synchronised every stream that
    // used them (hipFree does not wait for kernels still reading them).
    void reclaim() {
        for (void* q : retired) hipFree(q);
        retired.clear();
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};


// XCD-partitioned presence mark (presence bytes; launch_cluster_local_bitmap turns them into bits).
int launch_cluster_mark(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int L,
                        uint8_t* presence, hipStream_t s);
int launch_cluster_local_bitmap(const ClusterLayout& cl, uint8_t* ws, uint64_t* bitmap_out,
                                hipStream_t s);
// presence bitmap straight from the codes by an 8-bit partition sort (7 <= L <= 13)
int cluster_mark_bitmap_temp(int64_t n, int L, int64_t* bytes);
int launch_cluster_mark_bitmap(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int L,
                               uint64_t* bitmap, void* temp, int64_t temp_bytes, hipStream_t s);
// the same in two phases (1: slice-bucket pass; 2: the rest; 0: both)
int launch_cluster_mark_phase(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int L,
                              uint64_t* bitmap, void* temp, int64_t temp_bytes, int phase, hipStream_t s);
// The assign half of a fused score + assign: completes (deferred = false) or registers
// (deferred = true, as launch_cluster_assign) the assign of codes into cluster_id, and
// fills *a with the tables when the fused kernel can label these rows (word labels,
// labels by code); a->out == nullptr otherwise (the caller then uses launch_cluster_assign).
int cluster_assign_prepare(const ClusterLayout& cl, const uint8_t* ws, const uint32_t* codes,
                           const uint64_t* regular_bits, int64_t n, uint32_t* cluster_id, hipStream_t s,
                           bool deferred, AssignIn* a);
int launch_cluster_resolve(const ClusterLayout& cl, uint8_t* ws, const uint64_t* bitmaps,
                           int n_bitmaps, int max_distance, hipStream_t s);
// Waits for an asynchronous resolve's round flags and completes it if needed.
// *redone (nullable): 1 when more rounds (+ labels, + a deferred assign) were enqueued.
int cluster_finish(const void* ws, hipStream_t s, int* redone = nullptr);
void cluster_release(const void* ws);
int cluster_rounds(const void* ws, hipStream_t s, int* rounds);
int cluster_set_spec_rounds(int n);
int cluster_set_lookback_polls(int n);
int cluster_set_mark_method(int m);
// deferred: enqueue without waiting for the resolve's flags (cluster_finish re-runs it
// if the speculative rounds were not enough)
int launch_cluster_assign(const ClusterLayout& cl, const uint8_t* ws, const uint32_t* codes,
                          const uint64_t* regular_bits, int64_t n, uint32_t* cluster_id,
                          hipStream_t s, bool deferred = false);

// Irregular rows grouped by exact bytes (any length <= max_len); ids continue after
// stats_dev[1] (the regular cluster count) or from 0 when stats_dev is NULL.
int irregular_cluster(const void* offsets, int offset_width, const uint8_t* values,
                      const int64_t* rows, int64_t n_rows, int64_t max_len, const int64_t* stats_dev,
                      uint32_t* cluster_id, int64_t* n_irregular_clusters, hipStream_t s);

// Labels of packed regular codes: lab[i] = the regular cluster id of code q[i], or
// 0xFFFFFFFF when q[i] is ~0 or not a present code. Enqueued on s.
using CodeLookup = std::function<int(const uint64_t* q, int64_t nq, uint32_t* lab, hipStream_t s)>;
// max_distance 1 over the irregular rows (irregular.hip): Hamming-1 edges among the
// distinct irregular strings and to the regular clusters (lookup; NULL: no regular
// codes), connected components with the n_reg regular clusters, ids into cluster_id
// (irregular rows) and, when regular clusters merged, relabel[0..relabel_n) remapped in
// place (entries < n_reg). *n_clusters = all clusters. Synchronises s.
int irregular_merge(const void* offsets, int offset_width, const uint8_t* values, const int64_t* rows,
                    int64_t n_rows, int64_t max_len, int L, int64_t n_reg, const CodeLookup* lookup,
                    uint32_t* relabel, int64_t relabel_n, uint32_t* cluster_id, int64_t* n_clusters, hipStream_t s);
// lookup over a sorted code array G[ng] with one label per entry
int sorted_code_lookup(const uint64_t* G, int64_t ng, const uint32_t* labels, const uint64_t* q, int64_t nq,
                       uint32_t* lab, hipStream_t s);
// lookup through a resolved (and assigned) bitmap-engine workspace
int launch_cluster_lookup(const ClusterLayout& cl, const uint8_t* ws, const uint64_t* q, int64_t nq, uint32_t* lab,
                          hipStream_t s);

// records (code with digit p zeroed, p, code) of positions p0 .. p0+np-1 of every code of
// D[nd] (dist_cluster.hip; world 1)
int masked_records_range(const uint64_t* D, int64_t nd, int p0, int np, uint64_t* mk, uint32_t* pos, uint64_t* code,
                         hipStream_t s);

// H3 for 17 <= L <= 32 (sort-based, long_cluster.hip): regular + irregular rows of a
// device column; ids into cid (device), *n_clusters on the host. Synchronises s.
int long_cluster(const void* offsets, int ow, const uint8_t* values, const uint8_t* validity, int64_t voff,
                 int64_t n, int L, int max_distance, int64_t max_len, uint32_t* cid, int64_t* n_clusters,
                 hipStream_t s);

}  // namespace rogtk
