// capi.hip — extern "C" surface of librogtk_hip.so (declared in include/rogtk_hip.h).
//
// Host-side responsibilities: argument validation, thread-local last-error,
// the glibc-log2 entropy tables (bit-exact with the reference's f64::log2),
// Hamming target encoding, the per-thread device context of the level-2
// (host Arrow buffer) entry points, and launch-bracketing profiling events.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "rogtk_internal.h"

namespace rogtk {

// ------------------------------------------------------------------ errors
static thread_local char t_err[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t_err, sizeof(t_err), fmt, ap);
    va_end(ap);
}

// --------------------------------------------------------------- profiling
const char* const kKernelNames[K_COUNT_] = {
    "stage",          "score_packed",   "score_rows",    "cluster_mark",
    "cluster_bitmap", "cluster_scan",   "cluster_compact", "cluster_union",
    "cluster_flatten", "cluster_label", "cluster_assign", "cluster_irregular",
    "bam_fields",     "bam_scan",       "bam_fill",      "pack_reads",
    "row_gather",     "kmer_lds",      "cluster_resolve", "kmer_minimizer",
    "k_slice_bucket", "k_slice_mark",  "k_or_partials",  "k_scan_rt",
    "k_local_cc",     "k_hook_g",      "k_jump",         "k_roots_check", "k_word_label",
    "pack_gather",    "kmer_wave"};

namespace {
std::atomic<bool> g_prof{false};
std::atomic<uint32_t> g_prof_mask{~0u};  // kernels bracketed while g_prof is on (bit per KernelId)
std::mutex g_prof_mu;
struct ProfRec {
    KernelId id;
    hipEvent_t a, b;
};
std::vector<ProfRec> g_prof_pending;
double g_prof_ms[K_COUNT_] = {0};
int64_t g_prof_n[K_COUNT_] = {0};
// in-kernel spans: each profiled launch writes (entry, exit) ticks per workgroup into a
// slice of one preallocated device arena; the min/max reductions run only at drain time
// (profile_read_span / reset / a full arena), so a profiled launch adds no allocation,
// no kernel and no stream dependency to the pipeline it measures
constexpr int kSpanSlots = 1 << 14;
constexpr size_t kSpanArenaBytes = size_t(256) << 20;  // ~400 launches of 10M rows
uint64_t* g_span_dev = nullptr;    // kSpanSlots results
uint64_t* g_span_arena = nullptr;  // per-workgroup ticks of the pending launches
size_t g_span_used = 0;            // bytes of the arena handed out
struct SpanRec {
    KernelId id;
    size_t off;  // u64 offset of the launch's ticks in the arena
    int64_t nb;  // workgroups
};
std::vector<SpanRec> g_span_pending;
double g_span_ms[K_COUNT_] = {0};
int64_t g_span_n[K_COUNT_] = {0};
double g_span_tick_ms = 0;  // wall_clock64 period in ms

// one workgroup per pending launch: max(exit) - min(entry) over its workgroups
__global__ void k_span_reduce(const uint64_t* __restrict__ arena, const int64_t* __restrict__ desc,
                              uint64_t* __restrict__ out) {
    __shared__ uint64_t s_lo[256], s_hi[256];
    const uint64_t* t = arena + desc[2 * blockIdx.x];
    const int64_t nb = desc[2 * blockIdx.x + 1];
    uint64_t lo = ~0ull, hi = 0;
    for (int64_t b = threadIdx.x; b < nb; b += blockDim.x) {
        lo = min(lo, t[2 * b]);
        hi = max(hi, t[2 * b + 1]);
    }
    s_lo[threadIdx.x] = lo;
    s_hi[threadIdx.x] = hi;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            s_lo[threadIdx.x] = min(s_lo[threadIdx.x], s_lo[threadIdx.x + o]);
            s_hi[threadIdx.x] = max(s_hi[threadIdx.x], s_hi[threadIdx.x + o]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = s_hi[0] > s_lo[0] ? s_hi[0] - s_lo[0] : 0;
}

void span_drain_locked() {
    if (g_span_pending.empty() || !g_span_dev) return;
    const size_t n = g_span_pending.size();
    std::vector<int64_t> desc(2 * n);
    for (size_t i = 0; i < n; ++i) {
        desc[2 * i] = (int64_t)g_span_pending[i].off;
        desc[2 * i + 1] = g_span_pending[i].nb;
    }
    std::vector<uint64_t> h(n);
    int64_t* d_desc = nullptr;
    bool ok = hipDeviceSynchronize() == hipSuccess && hipMalloc((void**)&d_desc, desc.size() * 8) == hipSuccess;
    if (ok) {
        ok = hipMemcpy(d_desc, desc.data(), desc.size() * 8, hipMemcpyHostToDevice) == hipSuccess;
        if (ok) {
            hipLaunchKernelGGL(k_span_reduce, dim3((unsigned)n), dim3(256), 0, 0, g_span_arena, d_desc, g_span_dev);
            ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
                 hipMemcpy(h.data(), g_span_dev, n * 8, hipMemcpyDeviceToHost) == hipSuccess;
        }
        (void)hipFree(d_desc);
    }
    if (ok)
        for (size_t i = 0; i < n; ++i) {
            g_span_ms[g_span_pending[i].id] += (double)h[i] * g_span_tick_ms;
            g_span_n[g_span_pending[i].id] += 1;
        }
    g_span_pending.clear();
    g_span_used = 0;
}

// timing events are reused (no create / destroy per profiled launch) and released at
// device scope: a system-scope release would write the L2 back at every bracketed launch
std::vector<hipEvent_t> g_prof_free;

hipEvent_t prof_event_locked() {
    if (!g_prof_free.empty()) {
        hipEvent_t e = g_prof_free.back();
        g_prof_free.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    return hipEventCreateWithFlags(&e, hipEventDisableSystemFence) == hipSuccess ? e : nullptr;
}

void prof_drain_locked() {
    for (auto& r : g_prof_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            g_prof_ms[r.id] += ms;
            g_prof_n[r.id] += 1;
        }
        g_prof_free.push_back(r.a);
        g_prof_free.push_back(r.b);
    }
    g_prof_pending.clear();
}
}  // namespace

bool profiling_on() { return g_prof.load(std::memory_order_relaxed); }

uint64_t* span_begin(KernelId id, int64_t n_blocks, hipStream_t s) {
    (void)s;
    if (!g_prof.load(std::memory_order_relaxed) || !((g_prof_mask.load(std::memory_order_relaxed) >> id) & 1u))
        return nullptr;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (!g_span_dev) {
        int dev = 0, khz = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0 ||
            hipMalloc((void**)&g_span_dev, kSpanSlots * 8) != hipSuccess) {
            g_span_dev = nullptr;
            return nullptr;
        }
        if (hipMalloc((void**)&g_span_arena, kSpanArenaBytes) != hipSuccess) {
            (void)hipFree(g_span_dev);
            g_span_dev = g_span_arena = nullptr;
            return nullptr;
        }
        g_span_tick_ms = 1.0 / (double)khz;
    }
    const size_t need = (size_t)std::max<int64_t>(n_blocks, 1) * 16;
    if (need > kSpanArenaBytes) return nullptr;  // not timed
    if ((int)g_span_pending.size() >= kSpanSlots || g_span_used + need > kSpanArenaBytes) span_drain_locked();
    uint64_t* t = g_span_arena + g_span_used / 8;
    g_span_used += (need + 255) & ~size_t(255);
    return t;
}

void span_end(KernelId id, uint64_t* tspan, int64_t n_blocks, hipStream_t s) {
    (void)s;
    if (!tspan) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_span_pending.push_back({id, (size_t)(tspan - g_span_arena), std::max<int64_t>(n_blocks, 1)});
}

ProfScope::ProfScope(KernelId id, hipStream_t stream, bool exact) : id_(id), stream_(stream), exact_(exact) {
    if (!g_prof.load(std::memory_order_relaxed) || !((g_prof_mask.load(std::memory_order_relaxed) >> id) & 1u)) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    start_ = prof_event_locked();
    if (!start_) return;
    if (exact_) {  // both events ride on the dispatch packet (hipExtLaunchKernelGGL)
        stop_ = prof_event_locked();
        if (!stop_) {
            g_prof_free.push_back(start_);
            start_ = nullptr;
        }
        return;
    }
    hipEventRecord(start_, stream_);
}

ProfScope::~ProfScope() {
    if (!start_) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    hipEvent_t stop = stop_;
    if (!exact_) {
        stop = prof_event_locked();
        if (!stop) {
            g_prof_free.push_back(start_);
            return;
        }
        hipEventRecord(stop, stream_);
    }
    g_prof_pending.push_back({id_, start_, stop});
}

// ------------------------------------------------------------ entropy LUT
double plogp_host(uint32_t c, uint32_t t) {
    // umi_score.rs:67-68 / :140-141: p = count as f64 / total as f64; p * p.log2()
    const double p = (double)c / (double)t;
    return p * std::log2(p);
}

namespace {
struct DevLut {
    double* dev = nullptr;
    int64_t covered = -1;
};
std::mutex g_lut_mu;
std::map<int, DevLut> g_luts;
}  // namespace

int lut_ensure(int64_t max_total, const double** dev, int64_t* covered) {
    int device = 0;
    ROGTK_HIP_CHECK(hipGetDevice(&device));
    std::lock_guard<std::mutex> lk(g_lut_mu);
    DevLut& L = g_luts[device];
    if (L.covered < max_total) {
        int64_t want = std::max<int64_t>(std::max<int64_t>(max_total, 256), L.covered * 2);
        // 4096 covers every UMI/read-length string; the table is 8.4M doubles (67 MB).
        ROGTK_REQUIRE(max_total <= 4096, ROGTK_E_UNSUPPORTED,
                      "byte path: strings longer than 4096 bytes are not supported");
        want = std::min<int64_t>(want, 4096);
        const int64_t entries = lut_index(want + 1, 0);
        std::vector<double> h((size_t)entries, 0.0);
        for (int64_t t = 1; t <= want; ++t)
            for (int64_t c = 1; c <= t; ++c) h[(size_t)lut_index(t, c)] = plogp_host((uint32_t)c, (uint32_t)t);
        double* d = nullptr;
        ROGTK_HIP_CHECK(hipMalloc(&d, (size_t)entries * sizeof(double)));
        ROGTK_HIP_CHECK(hipMemcpy(d, h.data(), (size_t)entries * sizeof(double), hipMemcpyHostToDevice));
        if (L.dev) {
            ROGTK_HIP_CHECK(hipDeviceSynchronize());
            hipFree(L.dev);
        }
        L.dev = d;
        L.covered = want;
    }
    *dev = L.dev;
    *covered = L.covered;
    return ROGTK_OK;
}

int build_packed_params(int L, PackedParams* p) {
    std::memset(p, 0, sizeof(*p));
    p->L = L;
    for (int c = 1; c <= L; ++c) p->sh[c] = plogp_host((uint32_t)c, (uint32_t)L);
    if (L >= 2)
        for (int c = 1; c <= L - 1; ++c) p->di[c] = plogp_host((uint32_t)c, (uint32_t)(L - 1));
    if (L >= 3) {
        const double denom = (double)std::min(L - 2, 64);  // umi_score.rs:90
        for (int u = 0; u <= kMaxPackedLen; ++u) p->ling[u] = (double)u / denom;
    }
    for (int k = 0; k <= L; ++k) p->frac[k] = (double)k / (double)L;  // :120, :31
    return ROGTK_OK;
}

static size_t utf8_next_host(const uint8_t* s, size_t n, size_t i, uint32_t* cp) {
    const uint8_t c = s[i];
    size_t w = c < 0x80 ? 1 : (c >> 5) == 0x6 ? 2 : (c >> 4) == 0xE ? 3 : 4;
    if (i + w > n) w = n - i;
    uint32_t v = w == 1 ? c : w == 2 ? (c & 0x1Fu) : w == 3 ? (c & 0x0Fu) : (c & 0x07u);
    for (size_t k = 1; k < w; ++k) v = (v << 6) | (s[i + k] & 0x3Fu);
    *cp = v;
    return i + w;
}

void encode_target(const uint8_t* target, int64_t tlen, int L, uint32_t maxd, PackedParams* p) {
    p->max_distance = maxd;
    p->tcode = p->cmplo = p->always_mismatch = 0;
    if (!target) {
        p->ham_mode = 0;
        return;
    }
    if (tlen != L) {  // expressions.rs:1057: seq.len() != target.len() -> u32::MAX / false
        p->ham_mode = 2;
        return;
    }
    p->ham_mode = 1;
    // chars().zip(): a packed row is L ASCII chars; the target may hold fewer chars
    // (multi-byte UTF-8) — only the first min(k, L) positions are compared.
    size_t i = 0;
    int j = 0;
    while (i < (size_t)tlen && j < L) {
        uint32_t cp;
        i = utf8_next_host(target, (size_t)tlen, i, &cp);
        const int sh = 2 * (L - 1 - j);
        const int b = cp == 'A' ? 0 : cp == 'C' ? 1 : cp == 'G' ? 2 : cp == 'T' ? 3 : -1;
        if (b < 0) {
            p->always_mismatch += 1;  // a non-ACGT target char never equals a packed base
        } else {
            p->tcode |= (uint32_t)b << sh;
            p->cmplo |= 1u << sh;
        }
        ++j;
    }
}

}  // namespace rogtk

using namespace rogtk;

namespace {

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

int check_offset_width(int ow) {
    ROGTK_REQUIRE(ow == 4 || ow == 8, ROGTK_E_INVALID, "offset_width must be 4 or 8, got %d", ow);
    return ROGTK_OK;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int check_packed_alignment(const uint32_t* codes, const ScoreOut& o, const uint32_t* hd) {
    const void* ps[] = {codes, o.sh, o.ling, o.homo, o.di, o.dust, o.comb, o.longest, hd};
    for (const void* p : ps)
        ROGTK_REQUIRE(!p || aligned16(p), ROGTK_E_INVALID,
                      "packed SoA buffers must be 16-byte aligned (device allocations are)");
    return ROGTK_OK;
}

// --------------------------------------------- per-thread level-2 context
// Host <-> device transfers of the level-2 entry points. Pinned host memory
// (hipHostMalloc / rogtk_host_alloc / hipHostRegister) moves by direct DMA. Pageable
// memory moves through two pinned staging buffers of the context, chunk by chunk, so
// the DMA of one chunk overlaps the host copy of the other; the host copies of a chunk
// are split over a few threads (a single thread's memcpy, and the first-touch page
// faults of a fresh destination, cap a pageable copy well below the PCIe link).
constexpr size_t kStageChunk = (size_t)32 << 20;

int host_copy_threads() {
    static const int t = [] {
        const char* e = getenv("OMP_NUM_THREADS");
        int v = e ? atoi(e) : 0;
        const int hw = (int)std::thread::hardware_concurrency();
        if (v <= 0) v = hw > 0 ? hw : 4;
        return std::max(1, std::min(v, 8));
    }();
    return t;
}

void par_memcpy(void* dst, const void* src, size_t bytes) {
    const int t = bytes >= ((size_t)4 << 20) ? host_copy_threads() : 1;
    if (t <= 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> pool;
    const size_t per = (bytes / t + 4095) / 4096 * 4096;
    for (int k = 0; k < t; ++k) {
        const size_t a = std::min(bytes, per * k), b = std::min(bytes, per * (k + 1));
        if (a < b) pool.emplace_back([=] { std::memcpy((uint8_t*)dst + a, (const uint8_t*)src + a, b - a); });
    }
    for (auto& th : pool) th.join();
}

bool is_pinned(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

struct HostCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    DevBuf offsets, values, validity, codes, regbits, irr, nirr, target, out[8], ws, bitmap;
    int64_t ws_L = -1, ws_maxd = -1;
    void* pin[2] = {nullptr, nullptr};  // staging for pageable host memory
    hipEvent_t ev[2] = {nullptr, nullptr};
    ~HostCtx() {
        for (int k = 0; k < 2; ++k) {
            if (pin[k]) hipHostFree(pin[k]);
            if (ev[k]) hipEventDestroy(ev[k]);
        }
        if (stream) hipStreamDestroy(stream);
    }
    int staging() {
        for (int k = 0; k < 2; ++k) {
            if (!pin[k]) ROGTK_HIP_CHECK(hipHostMalloc(&pin[k], kStageChunk, hipHostMallocDefault));
            if (!ev[k]) ROGTK_HIP_CHECK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
        }
        return ROGTK_OK;
    }
    // device -> host; complete on return
    int d2h(void* dst, const void* src, size_t bytes) {
        if (bytes == 0) return ROGTK_OK;
        if (is_pinned(dst)) {
            ROGTK_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream));
            ROGTK_HIP_CHECK(hipStreamSynchronize(stream));
            return ROGTK_OK;
        }
        if (int rc = staging()) return rc;
        size_t prev_off = 0, prev_len = 0;
        int k = 0;
        for (size_t off = 0; off < bytes; off += kStageChunk, k ^= 1) {
            const size_t len = std::min(kStageChunk, bytes - off);
            ROGTK_HIP_CHECK(hipMemcpyAsync(pin[k], (const uint8_t*)src + off, len, hipMemcpyDeviceToHost, stream));
            ROGTK_HIP_CHECK(hipEventRecord(ev[k], stream));
            if (off > 0) {  // the previous chunk: out of its staging buffer while this one moves
                ROGTK_HIP_CHECK(hipEventSynchronize(ev[k ^ 1]));
                par_memcpy((uint8_t*)dst + prev_off, pin[k ^ 1], prev_len);
            }
            prev_off = off;
            prev_len = len;
        }
        ROGTK_HIP_CHECK(hipEventSynchronize(ev[k ^ 1]));
        par_memcpy((uint8_t*)dst + prev_off, pin[k ^ 1], prev_len);
        return ROGTK_OK;
    }
    // host -> device; enqueued on the stream (the host buffer may be reused on return)
    int h2d(void* dst, const void* src, size_t bytes) {
        if (bytes == 0) return ROGTK_OK;
        if (is_pinned(src)) {
            ROGTK_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream));
            return ROGTK_OK;
        }
        if (int rc = staging()) return rc;
        int k = 0;
        int64_t i = 0;
        for (size_t off = 0; off < bytes; off += kStageChunk, k ^= 1, ++i) {
            const size_t len = std::min(kStageChunk, bytes - off);
            if (i >= 2) ROGTK_HIP_CHECK(hipEventSynchronize(ev[k]));  // its DMA of two chunks ago is done
            par_memcpy(pin[k], (const uint8_t*)src + off, len);
            ROGTK_HIP_CHECK(hipMemcpyAsync((uint8_t*)dst + off, pin[k], len, hipMemcpyHostToDevice, stream));
            ROGTK_HIP_CHECK(hipEventRecord(ev[k], stream));
        }
        // the staging buffers are reused by the next transfer only after these DMAs: every
        // later use first waits on the events above (or the stream is synchronised)
        ROGTK_HIP_CHECK(hipStreamSynchronize(stream));
        return ROGTK_OK;
    }
};

thread_local std::unique_ptr<HostCtx> t_ctx;

int host_ctx(HostCtx** out) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_error("no HIP device available (librogtk_hip needs an MI355X / gfx950 GPU)");
        return ROGTK_E_NODEVICE;
    }
    int dev = 0;
    ROGTK_HIP_CHECK(hipGetDevice(&dev));
    if (!t_ctx || t_ctx->device != dev) {
        t_ctx.reset(new HostCtx());
        t_ctx->device = dev;
        ROGTK_HIP_CHECK(hipStreamCreateWithFlags(&t_ctx->stream, hipStreamNonBlocking));
    }
    *out = t_ctx.get();
    return ROGTK_OK;
}

struct HostCol {
    const void* offsets;
    int ow;
    const uint8_t* values;
    int64_t values_len;
    const uint8_t* validity;
    int64_t voff;
    int64_t n;
    int64_t off0() const { return ow == 4 ? ((const int32_t*)offsets)[0] : ((const int64_t*)offsets)[0]; }
    int64_t off(int64_t i) const {
        return ow == 4 ? ((const int32_t*)offsets)[i] : ((const int64_t*)offsets)[i];
    }
    bool valid(int64_t i) const {
        if (!validity) return true;
        const int64_t b = voff + i;
        return (validity[b >> 3] >> (b & 7)) & 1;
    }
    int first_len() const {
        for (int64_t i = 0; i < n; ++i)
            if (valid(i)) return (int)std::min<int64_t>(off(i + 1) - off(i), 1 << 30);
        return 0;
    }
    int64_t max_len() const {
        int64_t m = 0;
        for (int64_t i = 0; i < n; ++i) m = std::max<int64_t>(m, off(i + 1) - off(i));
        return m;
    }
};

// Longest row of a device column (irregular rows' radix-sort / byte-path width).
template <class O>
__global__ void k_max_len(const O* __restrict__ off, int64_t n, unsigned long long* out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long m = 0;
    if (r < n) m = (unsigned long long)((int64_t)off[r + 1] - (int64_t)off[r]);
    for (int d = 32; d; d >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, d));
    if ((threadIdx.x & 63) == 0 && m) atomicMax(out, m);
}

// max_len of the column already uploaded to c->offsets (device reduction; one sync)
int device_max_len(HostCtx* c, int ow, int64_t n, int64_t* out) {
    if (int rc = c->nirr.ensure(16)) return rc;
    unsigned long long* slot = c->nirr.as<unsigned long long>() + 1;
    ROGTK_HIP_CHECK(hipMemsetAsync(slot, 0, 8, c->stream));
    const dim3 g((unsigned)((n + 255) / 256));
    if (ow == 4)
        hipLaunchKernelGGL(k_max_len<int32_t>, g, dim3(256), 0, c->stream, c->offsets.as<int32_t>(), n, slot);
    else
        hipLaunchKernelGGL(k_max_len<int64_t>, g, dim3(256), 0, c->stream, c->offsets.as<int64_t>(), n, slot);
    ROGTK_HIP_CHECK(hipGetLastError());
    unsigned long long h = 0;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&h, slot, 8, hipMemcpyDeviceToHost, c->stream));
    ROGTK_HIP_CHECK(hipStreamSynchronize(c->stream));
    *out = (int64_t)h;
    return ROGTK_OK;
}

// Upload a host column and stage it; returns the resolved packed length in *L.
int upload_and_stage(HostCtx* c, const HostCol& h, int L_req, int* L_out, int64_t* n_irr_host) {
    const int64_t n = h.n;
    const int ow = h.ow;
    ROGTK_REQUIRE(c->offsets.ensure((size_t)(n + 1) * ow) == ROGTK_OK, ROGTK_E_HIP, "%s", rogtk_last_error());
    if (int rc = c->h2d(c->offsets.p, h.offsets, (size_t)(n + 1) * ow)) return rc;
    // values: upload [0, off(n)) so the device offsets stay valid as given
    const int64_t vbytes = std::max<int64_t>(h.off(n), 1);
    ROGTK_REQUIRE(h.off(n) <= h.values_len || h.values_len < 0, ROGTK_E_INVALID,
                  "offsets reference %lld bytes but values_len is %lld", (long long)h.off(n),
                  (long long)h.values_len);
    if (c->values.ensure((size_t)vbytes) != ROGTK_OK) return ROGTK_E_HIP;
    if (h.off(n) > 0)
        if (int rc = c->h2d(c->values.p, h.values, (size_t)h.off(n))) return rc;
    const uint8_t* dvalid = nullptr;
    if (h.validity) {
        const size_t vb = (size_t)((h.voff + n + 7) / 8);
        if (c->validity.ensure(vb) != ROGTK_OK) return ROGTK_E_HIP;
        if (int rc = c->h2d(c->validity.p, h.validity, vb)) return rc;
        dvalid = c->validity.as<uint8_t>();
    }
    int L = L_req > 0 ? L_req : h.first_len();
    *L_out = L;
    const int64_t words = (n + 63) / 64;
    if (c->codes.ensure((size_t)std::max<int64_t>(n, 4) * 4) != ROGTK_OK ||
        c->regbits.ensure((size_t)std::max<int64_t>(words, 1) * 8) != ROGTK_OK ||
        c->irr.ensure((size_t)std::max<int64_t>(n, 1) * 8) != ROGTK_OK ||
        c->nirr.ensure(16) != ROGTK_OK)
        return ROGTK_E_HIP;
    ROGTK_HIP_CHECK(hipMemsetAsync(c->nirr.p, 0, 8, c->stream));
    int rc = launch_stage(c->offsets.p, ow, c->values.as<uint8_t>(), dvalid, h.voff, n, L,
                          c->codes.as<uint32_t>(), c->regbits.as<uint64_t>(), c->irr.as<int64_t>(),
                          c->nirr.as<unsigned long long>(), c->stream);
    if (rc) return rc;
    if (n_irr_host) {
        ROGTK_HIP_CHECK(hipMemcpyAsync(n_irr_host, c->nirr.p, 8, hipMemcpyDeviceToHost, c->stream));
        ROGTK_HIP_CHECK(hipStreamSynchronize(c->stream));
    }
    return ROGTK_OK;
}

int check_host_col(const HostCol& h) {
    if (int rc = check_offset_width(h.ow)) return rc;
    ROGTK_REQUIRE(h.n >= 0, ROGTK_E_INVALID, "n must be >= 0");
    ROGTK_REQUIRE(h.offsets != nullptr, ROGTK_E_INVALID, "offsets must not be NULL");
    ROGTK_REQUIRE(h.values != nullptr || h.off(h.n) == h.off0(), ROGTK_E_INVALID, "values must not be NULL");
    ROGTK_REQUIRE(h.off0() == 0, ROGTK_E_INVALID,
                  "offsets[0] must be 0 (slice the values buffer instead of the offsets)");
    return ROGTK_OK;
}

}  // namespace

namespace rogtk {
namespace detail_attach {
thread_local hipEvent_t t_attached = nullptr;  // rogtk_event_attach_next
thread_local bool t_attach_taken = false;
}  // namespace
void arm_attached_event(hipEvent_t e) {
    detail_attach::t_attached = e;
    detail_attach::t_attach_taken = false;
}
bool attached_event_taken() { return detail_attach::t_attach_taken; }
void set_attached_taken() {
    detail_attach::t_attached = nullptr;
    detail_attach::t_attach_taken = true;
}
hipEvent_t take_attached_event() {
    using namespace detail_attach;
    hipEvent_t e = t_attached;
    if (e) {
        t_attached = nullptr;
        t_attach_taken = true;
    }
    return e;
}
}  // namespace rogtk

extern "C" {

const char* rogtk_version(void) { return "rogtk-amd 0.1.0 (gfx950)"; }

const char* rogtk_last_error(void) { return t_err; }

// Pinned host memory for callers' output (and input) buffers: transfers from / to it
// are direct DMA. Freed blocks are cached by size class (2 MiB multiples, up to 16 GiB
// in all) because pinning fresh pages costs more than the copy it saves.
namespace {
std::mutex g_pin_mu;
std::multimap<size_t, void*> g_pin_free;
std::map<void*, size_t> g_pin_size;
size_t g_pin_cached = 0;
constexpr size_t kPinCacheMax = (size_t)16 << 30;
}  // namespace

int rogtk_host_alloc(size_t bytes, void** out) {
    ROGTK_REQUIRE(out, ROGTK_E_INVALID, "host_alloc: NULL out");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        set_error("no HIP device available (librogtk_hip needs an MI355X / gfx950 GPU)");
        return ROGTK_E_NODEVICE;
    }
    const size_t cls = (std::max<size_t>(bytes, 1) + ((size_t)2 << 20) - 1) / ((size_t)2 << 20) * ((size_t)2 << 20);
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        auto it = g_pin_free.find(cls);
        if (it != g_pin_free.end()) {
            *out = it->second;
            g_pin_cached -= cls;
            g_pin_free.erase(it);
            return ROGTK_OK;
        }
    }
    void* p = nullptr;
    ROGTK_HIP_CHECK(hipHostMalloc(&p, cls, hipHostMallocDefault));
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pin_size[p] = cls;
    *out = p;
    return ROGTK_OK;
}

int rogtk_host_free(void* p) {
    if (!p) return ROGTK_OK;
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pin_size.find(p);
    ROGTK_REQUIRE(it != g_pin_size.end(), ROGTK_E_INVALID, "host_free: not a rogtk_host_alloc block");
    const size_t cls = it->second;
    if (g_pin_cached + cls <= kPinCacheMax) {
        g_pin_free.emplace(cls, p);
        g_pin_cached += cls;
    } else {
        g_pin_size.erase(it);
        ROGTK_HIP_CHECK(hipHostFree(p));
    }
    return ROGTK_OK;
}

int rogtk_device_count(int* out) {
    ROGTK_REQUIRE(out, ROGTK_E_INVALID, "out_count is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return ROGTK_OK;
}

int rogtk_stage_strings(const void* offsets, int offset_width, const uint8_t* values,
                        const uint8_t* validity, int64_t validity_offset, int64_t n, int umi_len,
                        uint32_t* codes, uint64_t* regular_bits, int64_t* irregular_rows,
                        int64_t* n_irregular, void* stream) {
    if (int rc = check_offset_width(offset_width)) return rc;
    ROGTK_REQUIRE(n >= 0, ROGTK_E_INVALID, "n must be >= 0");
    ROGTK_REQUIRE(n == 0 || (offsets && codes && regular_bits && irregular_rows && n_irregular),
                  ROGTK_E_INVALID, "stage: NULL buffer");
    hipStream_t s = as_stream(stream);
    if (n_irregular) ROGTK_HIP_CHECK(hipMemsetAsync(n_irregular, 0, 8, s));
    return launch_stage(offsets, offset_width, values, validity, validity_offset, n, umi_len, codes,
                        regular_bits, irregular_rows, (unsigned long long*)n_irregular, s);
}

int rogtk_umi_score_packed(const uint32_t* codes, const uint64_t* regular_bits, int64_t n,
                           int umi_len, const rogtk_umi_scores* scores, const uint8_t* target,
                           int64_t target_len, uint32_t max_distance, uint32_t* hamming_distance,
                           uint64_t* hamming_within_bits, void* stream) {
    ROGTK_REQUIRE(umi_len >= 1 && umi_len <= kMaxPackedLen, ROGTK_E_UNSUPPORTED,
                  "packed path: umi_len %d outside 1..%d", umi_len, kMaxPackedLen);
    ROGTK_REQUIRE(n >= 0, ROGTK_E_INVALID, "n must be >= 0");
    ROGTK_REQUIRE(n == 0 || codes, ROGTK_E_INVALID, "codes is NULL");
    ROGTK_REQUIRE(target_len >= 0, ROGTK_E_INVALID, "target_len must be >= 0");
    const ScoreOut o = to_score_out(scores);
    if (int rc = check_packed_alignment(codes, o, hamming_distance)) return rc;
    PackedParams p;
    build_packed_params(umi_len, &p);
    encode_target(target, target_len, umi_len, max_distance, &p);
    return launch_score_packed(codes, regular_bits, n, p, o, hamming_distance, hamming_within_bits,
                               as_stream(stream));
}

int rogtk_umi_score_assign_packed(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int umi_len,
                                  const rogtk_umi_scores* scores, const uint8_t* target, int64_t target_len,
                                  uint32_t max_distance, uint32_t* hamming_distance,
                                  uint64_t* hamming_within_bits, const void* cluster_ws,
                                  int64_t cluster_max_distinct, uint32_t* cluster_id, int deferred,
                                  void* stream) {
    ROGTK_REQUIRE(umi_len >= 1 && umi_len <= kMaxPackedLen, ROGTK_E_UNSUPPORTED,
                  "packed path: umi_len %d outside 1..%d", umi_len, kMaxPackedLen);
    ROGTK_REQUIRE(n >= 0, ROGTK_E_INVALID, "n must be >= 0");
    ROGTK_REQUIRE(n == 0 || (codes && cluster_id), ROGTK_E_INVALID, "codes / cluster_id is NULL");
    ROGTK_REQUIRE(cluster_ws, ROGTK_E_INVALID, "score_assign: cluster_ws is NULL");
    ROGTK_REQUIRE(target_len >= 0, ROGTK_E_INVALID, "target_len must be >= 0");
    ROGTK_REQUIRE(aligned16(codes) && aligned16(cluster_id), ROGTK_E_INVALID,
                  "score_assign: codes/cluster_id must be 16-byte aligned");
    const ScoreOut o = to_score_out(scores);
    if (int rc = check_packed_alignment(codes, o, hamming_distance)) return rc;
    ClusterLayout cl;
    if (int rc = cluster_layout(umi_len, cluster_max_distinct, &cl)) return rc;
    PackedParams p;
    build_packed_params(umi_len, &p);
    encode_target(target, target_len, umi_len, max_distance, &p);
    hipStream_t s = as_stream(stream);
    AssignIn a;
    if (int rc = cluster_assign_prepare(cl, (const uint8_t*)cluster_ws, codes, regular_bits, n, cluster_id, s,
                                        deferred != 0, &a))
        return rc;
    const bool any = any_score(o) || (p.ham_mode && (hamming_distance || hamming_within_bits));
    if (a.out && any)  // one pass: scores, Hamming and ids
        return launch_score_packed(codes, regular_bits, n, p, o, hamming_distance, hamming_within_bits, s, &a);
    if (int rc = launch_score_packed(codes, regular_bits, n, p, o, hamming_distance, hamming_within_bits, s))
        return rc;
    return launch_cluster_assign(cl, (const uint8_t*)cluster_ws, codes, regular_bits, n, cluster_id, s,
                                 deferred != 0);
}

int rogtk_umi_score_rows(const void* offsets, int offset_width, const uint8_t* values,
                         const int64_t* rows, const int64_t* n_rows_dev, int64_t max_rows,
                         int64_t max_len, const rogtk_umi_scores* scores, const uint8_t* target,
                         int64_t target_len, uint32_t max_distance, uint32_t* hamming_distance,
                         uint64_t* hamming_within_bits, void* stream) {
    if (int rc = check_offset_width(offset_width)) return rc;
    ROGTK_REQUIRE(max_rows >= 0 && max_len >= 0 && target_len >= 0, ROGTK_E_INVALID,
                  "score_rows: negative size");
    if (max_rows == 0) return ROGTK_OK;
    ROGTK_REQUIRE(offsets && rows, ROGTK_E_INVALID, "score_rows: NULL offsets/rows");
    const double* lut = nullptr;
    int64_t covered = 0;
    if (int rc = lut_ensure(std::max<int64_t>(max_len, 1), &lut, &covered)) return rc;
    hipStream_t s = as_stream(stream);
    const uint8_t* tdev = nullptr;
    thread_local DevBuf t_target;
    if (target) {
        if (int rc = t_target.ensure((size_t)std::max<int64_t>(target_len, 1))) return rc;
        if (target_len)
            ROGTK_HIP_CHECK(hipMemcpyAsync(t_target.p, target, (size_t)target_len, hipMemcpyHostToDevice, s));
        tdev = t_target.as<uint8_t>();
    }
    return launch_score_rows(offsets, offset_width, values, rows, n_rows_dev, max_rows, lut, covered,
                             to_score_out(scores), tdev, target_len, target ? 1 : 0, max_distance,
                             hamming_distance, hamming_within_bits, s);
}

int rogtk_cluster_workspace_size(int umi_len, int64_t max_distinct, int64_t* bytes) {
    ROGTK_REQUIRE(bytes, ROGTK_E_INVALID, "bytes is NULL");
    ClusterLayout cl;
    if (int rc = cluster_layout(umi_len, max_distinct, &cl)) return rc;
    *bytes = cl.total;
    return ROGTK_OK;
}

int rogtk_cluster_bitmap_words(int umi_len, int64_t* words) {
    ROGTK_REQUIRE(words, ROGTK_E_INVALID, "words is NULL");
    ClusterLayout cl;
    if (int rc = cluster_layout(umi_len, 1, &cl)) return rc;
    *words = cl.words;
    return ROGTK_OK;
}

int rogtk_cluster_init(void* ws, int umi_len, int64_t max_distinct, void* stream) {
    ClusterLayout cl;
    if (int rc = cluster_layout(umi_len, max_distinct, &cl)) return rc;
    ROGTK_REQUIRE(ws, ROGTK_E_INVALID, "ws is NULL");
    cluster_release(ws);  // a reused address must not inherit a stale pending resolve
    ROGTK_HIP_CHECK(hipMemsetAsync(ws, 0, (size_t)cl.total, as_stream(stream)));
    return ROGTK_OK;
}

int rogtk_cluster_mark(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int umi_len,
                       void* ws, int64_t max_distinct, void* stream) {
    ROGTK_REQUIRE(ws, ROGTK_E_INVALID, "ws is NULL");
    ClusterLayout cl;
    if (int rc = cluster_layout(umi_len, max_distinct, &cl)) return rc;
    ROGTK_REQUIRE(n >= 0 && (n == 0 || codes), ROGTK_E_INVALID, "mark: bad codes/n");
    ROGTK_REQUIRE(aligned16(codes), ROGTK_E_INVALID, "mark: codes must be 16-byte aligned");
    return launch_cluster_mark(codes, regular_bits, n, umi_len, (uint8_t*)ws + cl.off_presence,
                               as_stream(stream));
}

int rogtk_cluster_local_bitmap(void* ws, int umi_len, int64_t max_distinct, uint64_t* bitmap_out,
                               void* stream) {
    ClusterLayout cl;
    if (int rc = cluster_layout(umi_len, max_distinct, &cl)) return rc;
    ROGTK_REQUIRE(ws && bitmap_out, ROGTK_E_INVALID, "ws/bitmap_out is NULL");
    return launch_cluster_local_bitmap(cl, (uint8_t*)ws, bitmap_out, as_stream(stream));
}

int rogtk_cluster_resolve(void* ws, int umi_len, int64_t max_distinct, const uint64_t* bitmaps,
                          int n_bitmaps, int max_distance, void* stream) {
    ClusterLayout cl;
    if (int rc = cluster_layout(umi_len, max_distinct, &cl)) return rc;
    ROGTK_REQUIRE(ws && bitmaps, ROGTK_E_INVALID, "ws/bitmaps is NULL");
    ROGTK_REQUIRE(n_bitmaps >= 1, ROGTK_E_INVALID, "n_bitmaps must be >= 1");
    ROGTK_REQUIRE(max_distance == 0 || max_distance == 1, ROGTK_E_UNSUPPORTED,
                  "max_distance %d: only 0 (exact) and 1 (Hamming<=1 components) are supported",
                  max_distance);
    return launch_cluster_resolve(cl, (uint8_t*)ws, bitmaps, n_bitmaps, max_distance, as_stream(stream));
}

int rogtk_cluster_assign(const void* ws, int umi_len, int64_t max_distinct, const uint32_t* codes,
                         const uint64_t* regular_bits, int64_t n, uint32_t* cluster_id,
                         void* stream) {
    ClusterLayout cl;
    if (int rc = cluster_layout(umi_len, max_distinct, &cl)) return rc;
    ROGTK_REQUIRE(ws && (n == 0 || (codes && cluster_id)), ROGTK_E_INVALID, "assign: NULL buffer");
    ROGTK_REQUIRE(aligned16(codes) && aligned16(cluster_id), ROGTK_E_INVALID,
                  "assign: codes/cluster_id must be 16-byte aligned");
    return launch_cluster_assign(cl, (const uint8_t*)ws, codes, regular_bits, n, cluster_id,
                                 as_stream(stream));
}

int rogtk_cluster_assign_deferred(const void* ws, int umi_len, int64_t max_distinct, const uint32_t* codes,
                                  const uint64_t* regular_bits, int64_t n, uint32_t* cluster_id, void* stream) {
    ClusterLayout cl;
    if (int rc = cluster_layout(umi_len, max_distinct, &cl)) return rc;
    ROGTK_REQUIRE(ws && (n == 0 || (codes && cluster_id)), ROGTK_E_INVALID, "assign: NULL buffer");
    ROGTK_REQUIRE(aligned16(codes) && aligned16(cluster_id), ROGTK_E_INVALID,
                  "assign: codes/cluster_id must be 16-byte aligned");
    return launch_cluster_assign(cl, (const uint8_t*)ws, codes, regular_bits, n, cluster_id, as_stream(stream),
                                 true);
}

int rogtk_cluster_sync(const void* ws, void* stream, int* redone) {
    ROGTK_REQUIRE(ws, ROGTK_E_INVALID, "ws is NULL");
    return cluster_finish(ws, as_stream(stream), redone);
}

int rogtk_cluster_stats(const void* ws, int umi_len, int64_t max_distinct, int64_t* out4,
                        void* stream) {
    ClusterLayout cl;
    if (int rc = cluster_layout(umi_len, max_distinct, &cl)) return rc;
    ROGTK_REQUIRE(ws && out4, ROGTK_E_INVALID, "stats: NULL buffer");
    hipStream_t s = as_stream(stream);
    if (int rc = cluster_finish(ws, s)) return rc;
    ROGTK_HIP_CHECK(hipMemcpyAsync(out4, (const uint8_t*)ws + cl.off_stats, 32, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    return ROGTK_OK;
}

int rogtk_cluster_rounds(const void* ws, void* stream, int* rounds) {
    ROGTK_REQUIRE(ws && rounds, ROGTK_E_INVALID, "rounds: NULL buffer");
    return cluster_rounds(ws, as_stream(stream), rounds);
}

int rogtk_cluster_set_spec_rounds(int n) { return cluster_set_spec_rounds(n); }
int rogtk_cluster_set_lookback_polls(int n) { return cluster_set_lookback_polls(n); }
int rogtk_cluster_set_mark_method(int method) { return cluster_set_mark_method(method); }
int rogtk_cluster_mark_bitmap_temp_bytes(int64_t n, int umi_len, int64_t* bytes) {
    ROGTK_REQUIRE(bytes, ROGTK_E_INVALID, "null bytes");
    return cluster_mark_bitmap_temp(n, umi_len, bytes);
}
int rogtk_cluster_mark_bitmap(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int umi_len,
                              uint64_t* bitmap_out, void* temp, int64_t temp_bytes, void* stream) {
    ROGTK_REQUIRE((codes || n == 0) && bitmap_out, ROGTK_E_INVALID, "null codes / bitmap_out");
    return launch_cluster_mark_bitmap(codes, regular_bits, n, umi_len, bitmap_out, temp, temp_bytes,
                                      as_stream(stream));
}
int rogtk_cluster_mark_bitmap_phase(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int umi_len,
                                    uint64_t* bitmap_out, void* temp, int64_t temp_bytes, int phase, void* stream) {
    ROGTK_REQUIRE((codes || n == 0) && bitmap_out, ROGTK_E_INVALID, "null codes / bitmap_out");
    return launch_cluster_mark_phase(codes, regular_bits, n, umi_len, bitmap_out, temp, temp_bytes, phase,
                                     as_stream(stream));
}
int rogtk_cluster_release(const void* ws) {
    if (ws) cluster_release(ws);
    return ROGTK_OK;
}

// ----------------------------------------------------------------- level 2
int rogtk_umi_complexity_host(const void* offsets, int offset_width, const uint8_t* values,
                              int64_t values_len, const uint8_t* validity, int64_t validity_offset,
                              int64_t n, const rogtk_umi_scores* out) {
    HostCol h{offsets, offset_width, values, values_len, validity, validity_offset, n};
    if (int rc = check_host_col(h)) return rc;
    ROGTK_REQUIRE(out, ROGTK_E_INVALID, "out is NULL");
    if (n == 0) return ROGTK_OK;
    HostCtx* c;
    if (int rc = host_ctx(&c)) return rc;
    int L = 0;
    int64_t n_irr = 0;
    if (int rc = upload_and_stage(c, h, 0, &L, &n_irr)) return rc;
    int64_t max_len = 0;  // only the byte path (irregular rows) needs it
    if (n_irr > 0)
        if (int rc = device_max_len(c, offset_width, n, &max_len)) return rc;
    const ScoreOut ho = to_score_out(out);
    // device outputs
    double* dptr[6] = {nullptr};
    const double* hptr[6] = {ho.sh, ho.ling, ho.homo, ho.di, ho.dust, ho.comb};
    for (int k = 0; k < 6; ++k)
        if (hptr[k]) {
            if (int rc = c->out[k].ensure((size_t)n * 8)) return rc;
            dptr[k] = c->out[k].as<double>();
        }
    uint32_t* dlong = nullptr;
    if (ho.longest) {
        if (int rc = c->out[6].ensure((size_t)n * 4)) return rc;
        dlong = c->out[6].as<uint32_t>();
    }
    rogtk_umi_scores ds{dptr[0], dptr[1], dptr[2], dptr[3], dlong, dptr[4], dptr[5]};
    const bool packable = L >= 1 && L <= kMaxPackedLen;
    if (packable) {
        int rc = rogtk_umi_score_packed(c->codes.as<uint32_t>(), c->regbits.as<uint64_t>(), n, L, &ds,
                                        nullptr, 0, 0, nullptr, nullptr, c->stream);
        if (rc) return rc;
    }
    if (n_irr > 0) {
        int rc = rogtk_umi_score_rows(c->offsets.p, offset_width, c->values.as<uint8_t>(),
                                      c->irr.as<int64_t>(), nullptr, n_irr, max_len, &ds, nullptr, 0,
                                      0, nullptr, nullptr, c->stream);
        if (rc) return rc;
    }
    for (int k = 0; k < 6; ++k)
        if (hptr[k])
            if (int rc = c->d2h((void*)hptr[k], dptr[k], (size_t)n * 8)) return rc;
    if (ho.longest)
        if (int rc = c->d2h(ho.longest, dlong, (size_t)n * 4)) return rc;
    return ROGTK_OK;
}

int rogtk_hamming_host(const void* offsets, int offset_width, const uint8_t* values,
                       int64_t values_len, const uint8_t* validity, int64_t validity_offset,
                       int64_t n, const uint8_t* target, int64_t target_len, uint32_t max_distance,
                       uint32_t* distance, uint8_t* within_bits) {
    HostCol h{offsets, offset_width, values, values_len, validity, validity_offset, n};
    if (int rc = check_host_col(h)) return rc;
    ROGTK_REQUIRE(target || target_len == 0, ROGTK_E_INVALID, "target is NULL");
    ROGTK_REQUIRE(target_len >= 0, ROGTK_E_INVALID, "target_len must be >= 0");
    if (n == 0) return ROGTK_OK;
    static const uint8_t kEmpty = 0;
    const uint8_t* tg = target ? target : &kEmpty;
    HostCtx* c;
    if (int rc = host_ctx(&c)) return rc;
    int L = 0;
    int64_t n_irr = 0;
    if (int rc = upload_and_stage(c, h, 0, &L, &n_irr)) return rc;
    int64_t max_len = 0;  // only the byte path (irregular rows) needs it
    if (n_irr > 0)
        if (int rc = device_max_len(c, offset_width, n, &max_len)) return rc;
    uint32_t* dd = nullptr;
    uint64_t* dw = nullptr;
    if (distance) {
        if (int rc = c->out[0].ensure((size_t)n * 4)) return rc;
        dd = c->out[0].as<uint32_t>();
    }
    const int64_t words = (n + 63) / 64;
    if (within_bits) {
        if (int rc = c->out[1].ensure((size_t)words * 8)) return rc;
        dw = c->out[1].as<uint64_t>();
    }
    if (L >= 1 && L <= kMaxPackedLen) {
        int rc = rogtk_umi_score_packed(c->codes.as<uint32_t>(), c->regbits.as<uint64_t>(), n, L,
                                        nullptr, tg, target_len, max_distance, dd, dw, c->stream);
        if (rc) return rc;
    } else if (dw) {
        ROGTK_HIP_CHECK(hipMemsetAsync(dw, 0, (size_t)words * 8, c->stream));
    }
    if (n_irr > 0) {
        int rc = rogtk_umi_score_rows(c->offsets.p, offset_width, c->values.as<uint8_t>(),
                                      c->irr.as<int64_t>(), nullptr, n_irr, max_len, nullptr, tg,
                                      target_len, max_distance, dd, dw, c->stream);
        if (rc) return rc;
    }
    if (distance)
        if (int rc = c->d2h(distance, dd, (size_t)n * 4)) return rc;
    if (within_bits)
        if (int rc = c->d2h(within_bits, dw, (size_t)(n + 7) / 8)) return rc;
    return ROGTK_OK;
}

namespace {


// H3 over a column already staged into c->codes / regbits / irr (n_irr irregular rows):
// regular rows through the cluster engine, then the irregular rows (exact bytes, or for
// max_distance 1 their Hamming-1 edges merged with the regular clusters, irregular.hip);
// ids into did (device), on stream s.
int cluster_staged(HostCtx* c, const void* d_offsets, int ow, const uint8_t* d_values, const uint8_t* d_validity,
                   int64_t voff, int64_t n, int L, int64_t n_irr, int64_t max_len, int max_distance, uint32_t* did,
                   int64_t* n_clusters, hipStream_t s) {
    if (L > kMaxPackedLen && L <= 32)  // long UMIs: sort-based engine (regular + irregular rows)
        return long_cluster(d_offsets, ow, d_values, d_validity, voff, n, L, max_distance, max_len, did, n_clusters, s);
    int64_t n_reg_clusters = 0;
    const int64_t* stats_dev = nullptr;
    if (L >= 1 && L <= kMaxPackedLen) {
        const int64_t space = (int64_t)1 << std::min(2 * L, 40);
        const int64_t maxd = std::max<int64_t>(1, std::min<int64_t>(space, n));
        ClusterLayout cl;
        if (int rc = cluster_layout(L, maxd, &cl)) return rc;
        if (c->ws_L != L || c->ws_maxd < cl.max_distinct) {
            if (int rc = c->ws.ensure((size_t)cl.total)) return rc;
            if (int rc = rogtk_cluster_init(c->ws.p, L, cl.max_distinct, s)) return rc;
            c->ws_L = L;
            c->ws_maxd = cl.max_distinct;
        }
        ClusterLayout use;
        cluster_layout(L, c->ws_maxd, &use);
        if (int rc = c->bitmap.ensure((size_t)use.words * 8)) return rc;
        int rc = rogtk_cluster_mark(c->codes.as<uint32_t>(), c->regbits.as<uint64_t>(), n, L, c->ws.p,
                                    use.max_distinct, s);
        if (!rc) rc = rogtk_cluster_local_bitmap(c->ws.p, L, use.max_distinct, c->bitmap.as<uint64_t>(), s);
        if (!rc) rc = rogtk_cluster_resolve(c->ws.p, L, use.max_distinct, c->bitmap.as<uint64_t>(), 1,
                                            max_distance, s);
        if (!rc) rc = rogtk_cluster_assign(c->ws.p, L, use.max_distinct, c->codes.as<uint32_t>(),
                                           c->regbits.as<uint64_t>(), n, did, s);
        if (rc) {
            c->ws_L = -1;  // presence may be dirty: re-initialise on the next call
            return rc;
        }
        int64_t st[4];
        if (int rc2 = rogtk_cluster_stats(c->ws.p, L, use.max_distinct, st, s)) return rc2;
        ROGTK_REQUIRE(st[2] == 0, ROGTK_E_OVERFLOW, "cluster: distinct UMIs exceeded max_distinct");
        n_reg_clusters = st[1];
        stats_dev = (const int64_t*)((uint8_t*)c->ws.p + use.off_stats);
    } else {
        ROGTK_HIP_CHECK(hipMemsetAsync(did, 0xFF, (size_t)n * 4, s));
    }
    int64_t total = n_reg_clusters;
    if (n_irr > 0 && max_distance == 1) {
        // Hamming-1 edges of the irregular rows (to each other and to regular codes)
        const bool packable = L >= 1 && L <= kMaxPackedLen;
        ClusterLayout use{};
        if (packable) cluster_layout(L, c->ws_maxd, &use);
        const uint8_t* ws = (const uint8_t*)c->ws.p;
        CodeLookup lk = [&](const uint64_t* q, int64_t nq, uint32_t* lab, hipStream_t st) {
            return launch_cluster_lookup(use, ws, q, nq, lab, st);
        };
        int rc = irregular_merge(d_offsets, ow, d_values, c->irr.as<int64_t>(), n_irr, max_len, L, n_reg_clusters,
                                 packable ? &lk : nullptr, did, n, did, &total, s);
        if (rc) return rc;
    } else if (n_irr > 0) {
        int64_t n_irr_clusters = 0;
        int rc = irregular_cluster(d_offsets, ow, d_values, c->irr.as<int64_t>(), n_irr, max_len, stats_dev, did,
                                   &n_irr_clusters, s);
        if (rc) return rc;
        total += n_irr_clusters;
    }
    if (n_clusters) *n_clusters = total;
    return ROGTK_OK;
}

}  // namespace

int rogtk_umi_cluster_host(const void* offsets, int offset_width, const uint8_t* values,
                           int64_t values_len, const uint8_t* validity, int64_t validity_offset,
                           int64_t n, int umi_len, int max_distance, uint32_t* cluster_id,
                           int64_t* n_clusters, int* resolved_umi_len) {
    HostCol h{offsets, offset_width, values, values_len, validity, validity_offset, n};
    if (int rc = check_host_col(h)) return rc;
    ROGTK_REQUIRE(cluster_id || n == 0, ROGTK_E_INVALID, "cluster_id is NULL");
    ROGTK_REQUIRE(max_distance == 0 || max_distance == 1, ROGTK_E_UNSUPPORTED,
                  "max_distance %d: only 0 and 1 are supported", max_distance);
    int L = umi_len > 0 ? umi_len : h.first_len();
    if (resolved_umi_len) *resolved_umi_len = L;
    if (n_clusters) *n_clusters = 0;
    if (n == 0) return ROGTK_OK;
    HostCtx* c;
    if (int rc = host_ctx(&c)) return rc;
    int64_t n_irr = 0;
    if (int rc = upload_and_stage(c, h, L, &L, &n_irr)) return rc;
    if (int rc = c->out[0].ensure((size_t)std::max<int64_t>(n, 4) * 4)) return rc;
    uint32_t* did = c->out[0].as<uint32_t>();
    int64_t max_len = 0;  // irregular rows and the long engine need it
    if (n_irr || (L > kMaxPackedLen && L <= 32))
        if (int rc = device_max_len(c, offset_width, n, &max_len)) return rc;
    if (int rc = cluster_staged(c, c->offsets.p, offset_width, c->values.as<uint8_t>(),
                                h.validity ? c->validity.as<uint8_t>() : nullptr, h.voff, n, L, n_irr, max_len,
                                max_distance, did, n_clusters, c->stream))
        return rc;
    return c->d2h(cluster_id, did, (size_t)n * 4);
}

int rogtk_umi_cluster_dev(const int64_t* offsets, const uint8_t* values, const uint8_t* validity, int64_t n,
                          int umi_len, int max_distance, uint32_t* cluster_id, int64_t* n_clusters, void* stream) {
    ROGTK_REQUIRE(n >= 0 && (n == 0 || (offsets && values && cluster_id)), ROGTK_E_INVALID,
                  "umi_cluster_dev: NULL argument");
    ROGTK_REQUIRE(umi_len >= 1, ROGTK_E_INVALID, "umi_cluster_dev: umi_len must be >= 1");
    ROGTK_REQUIRE(max_distance == 0 || max_distance == 1, ROGTK_E_UNSUPPORTED,
                  "max_distance %d: only 0 and 1 are supported", max_distance);
    if (n_clusters) *n_clusters = 0;
    if (n == 0) return ROGTK_OK;
    hipStream_t s = as_stream(stream);
    HostCtx* c;
    if (int rc = host_ctx(&c)) return rc;
    const int64_t words = (n + 63) / 64;
    if (c->codes.ensure((size_t)std::max<int64_t>(n, 4) * 4) != ROGTK_OK ||
        c->regbits.ensure((size_t)std::max<int64_t>(words, 1) * 8) != ROGTK_OK ||
        c->irr.ensure((size_t)std::max<int64_t>(n, 1) * 8) != ROGTK_OK || c->nirr.ensure(16) != ROGTK_OK)
        return ROGTK_E_HIP;
    ROGTK_HIP_CHECK(hipMemsetAsync(c->nirr.p, 0, 16, s));
    if (int rc = launch_stage(offsets, 8, values, validity, 0, n, umi_len, c->codes.as<uint32_t>(),
                              c->regbits.as<uint64_t>(), c->irr.as<int64_t>(), c->nirr.as<unsigned long long>(), s))
        return rc;
    hipLaunchKernelGGL(k_max_len<int64_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, offsets, n,
                       c->nirr.as<unsigned long long>() + 1);
    ROGTK_HIP_CHECK(hipGetLastError());
    int64_t hv[2];
    ROGTK_HIP_CHECK(hipMemcpyAsync(hv, c->nirr.p, 16, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    return cluster_staged(c, offsets, 8, values, validity, 0, n, umi_len, hv[0], hv[1], max_distance, cluster_id,
                          n_clusters, s);
}

// --------------------------------------------------------------- stream events
int rogtk_event_create(int flags, void** out) {
    ROGTK_REQUIRE(out, ROGTK_E_INVALID, "event_create: NULL out");
    *out = nullptr;
    ROGTK_REQUIRE((flags & ~1) == 0, ROGTK_E_INVALID, "event_create: unknown flags %d", flags);
    hipEvent_t e = nullptr;
    const unsigned f = hipEventDisableTiming | ((flags & 1) ? hipEventDisableSystemFence : 0u);
    ROGTK_HIP_CHECK(hipEventCreateWithFlags(&e, f));
    *out = e;
    return ROGTK_OK;
}

int rogtk_event_destroy(void* ev) {
    if (!ev) return ROGTK_OK;
    ROGTK_HIP_CHECK(hipEventDestroy((hipEvent_t)ev));
    return ROGTK_OK;
}

int rogtk_event_attach_next(void* ev) {
    rogtk::detail_attach::t_attached = (hipEvent_t)ev;
    rogtk::detail_attach::t_attach_taken = false;
    return ROGTK_OK;
}

int rogtk_event_attach_done(int* taken) {
    ROGTK_REQUIRE(taken, ROGTK_E_INVALID, "event_attach_done: NULL argument");
    *taken = rogtk::detail_attach::t_attach_taken ? 1 : 0;
    rogtk::detail_attach::t_attached = nullptr;
    rogtk::detail_attach::t_attach_taken = false;
    return ROGTK_OK;
}

int rogtk_event_record(void* ev, void* stream) {
    ROGTK_REQUIRE(ev, ROGTK_E_INVALID, "event_record: NULL event");
    ROGTK_HIP_CHECK(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream));
    return ROGTK_OK;
}

int rogtk_stream_wait_event(void* stream, void* ev) {
    ROGTK_REQUIRE(ev, ROGTK_E_INVALID, "stream_wait_event: NULL event");
    ROGTK_HIP_CHECK(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0));
    return ROGTK_OK;
}

int rogtk_event_query(void* ev, int* done) {
    ROGTK_REQUIRE(ev && done, ROGTK_E_INVALID, "event_query: NULL argument");
    const hipError_t e = hipEventQuery((hipEvent_t)ev);
    if (e == hipErrorNotReady) {
        (void)hipGetLastError();
        *done = 0;
        return ROGTK_OK;
    }
    ROGTK_HIP_CHECK(e);
    *done = 1;
    return ROGTK_OK;
}

int rogtk_event_synchronize(void* ev) {
    ROGTK_REQUIRE(ev, ROGTK_E_INVALID, "event_synchronize: NULL event");
    ROGTK_HIP_CHECK(hipEventSynchronize((hipEvent_t)ev));
    return ROGTK_OK;
}

// --------------------------------------------------------------- profiling
int rogtk_profile_enable(int on) {
    g_prof.store(on != 0);
    return ROGTK_OK;
}

int rogtk_profile_select(const char* kernel) {
    if (!kernel || !kernel[0]) {
        g_prof_mask.store(~0u);
        return ROGTK_OK;
    }
    // one name or a comma-separated list
    uint32_t mask = 0;
    for (const char* p = kernel; *p;) {
        const char* e = std::strchr(p, ',');
        const size_t len = e ? (size_t)(e - p) : std::strlen(p);
        int found = -1;
        for (int k = 0; k < K_COUNT_; ++k)
            if (std::strlen(kKernelNames[k]) == len && std::strncmp(p, kKernelNames[k], len) == 0) found = k;
        if (found < 0) {
            set_error("profile_select: unknown kernel '%.*s'", (int)len, p);
            return ROGTK_E_INVALID;
        }
        mask |= 1u << found;
        p += len + (e ? 1 : 0);
    }
    g_prof_mask.store(mask);
    return ROGTK_OK;
}

int rogtk_profile_reset(void) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    prof_drain_locked();
    span_drain_locked();
    for (int k = 0; k < K_COUNT_; ++k) {
        g_prof_ms[k] = 0;
        g_prof_n[k] = 0;
        g_span_ms[k] = 0;
        g_span_n[k] = 0;
    }
    return ROGTK_OK;
}

int rogtk_profile_read_span(const char* kernel, double* total_ms, int64_t* launches) {
    ROGTK_REQUIRE(kernel && total_ms && launches, ROGTK_E_INVALID, "profile_read_span: NULL argument");
    std::lock_guard<std::mutex> lk(g_prof_mu);
    span_drain_locked();
    for (int k = 0; k < K_COUNT_; ++k)
        if (std::strcmp(kernel, kKernelNames[k]) == 0) {
            *total_ms = g_span_ms[k];
            *launches = g_span_n[k];
            return ROGTK_OK;
        }
    set_error("profile_read_span: unknown kernel '%s'", kernel);
    return ROGTK_E_INVALID;
}

int rogtk_profile_read(const char* kernel, double* total_ms, int64_t* launches) {
    ROGTK_REQUIRE(kernel && total_ms && launches, ROGTK_E_INVALID, "profile_read: NULL argument");
    std::lock_guard<std::mutex> lk(g_prof_mu);
    prof_drain_locked();
    for (int k = 0; k < K_COUNT_; ++k)
        if (std::strcmp(kernel, kKernelNames[k]) == 0) {
            *total_ms = g_prof_ms[k];
            *launches = g_prof_n[k];
            return ROGTK_OK;
        }
    set_error("profile_read: unknown kernel '%s'", kernel);
    return ROGTK_E_INVALID;
}

}  // extern "C"
