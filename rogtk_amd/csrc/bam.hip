// bam.hip — BAM records -> Arrow columns, decoded on the GPU.
//
// Replaces the record loops of the reference's BAM converters:
//   mode ROGTK_BAM_NOODLES       extract_record_data_enhanced   src/bam.rs:170-262 (noodles 0.82;
//                                bam_to_parquet / bam_to_arrow_ipc / bams_* / *_parallel / *_gzp_parallel)
//   mode ROGTK_BAM_HTSLIB        process_htslib_records_to_batch src/bam.rs:3028-3148 (rust-htslib 0.47;
//                                bam_to_arrow_ipc_htslib_{parallel,optimized,mmap_parallel,multi_reader_parallel},
//                                bams_to_arrow_ipc_htslib_optimized)
//   mode ROGTK_BAM_HTSLIB_BLOCKS process_htslib_records_to_batch src/bam_htslib.rs:154-241
//                                (bam_to_arrow_ipc_htslib_bgzf_blocks: 0-based start, bam_endpos end)
// Schema (create_bam_schema, bam.rs:3203-3221): name, chrom, start, end, flags, [sequence], [quality_scores].
//
// Work split (MI355X-first):
//   host  : BGZF inflate (zlib, one block per task, all blocks of a chunk in parallel on
//           the reader's threads) into a pinned stream buffer; record framing (one u32 per
//           record); the header (binary reference list, names lossy-UTF-8 as
//           String::from_utf8_lossy, bam.rs:2611-2618).
//   device: every per-record field: k_bam_fields (thread per record: fixed fields, CIGAR
//           reference length, output lengths, validity via wave ballots), an exclusive scan
//           of the lengths, k_bam_fill (one wave per record: read name with UTF-8 lossy
//           repair, chromosome name, 4-bit -> ASCII bases, PHRED+33 qualities).
// The raw record bytes cross PCIe once; columns are produced in HBM and copied back
// (host API) or left there for the UMI engine (rogtk_bam_next_dev).
#include <hipcub/hipcub.hpp>
#include <zlib.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

// ------------------------------------------------------------------ device
// Rust String::from_utf8_lossy: every maximal invalid subsequence -> U+FFFD (EF BF BD).
// Returns the output length; writes when out != nullptr.
__device__ __host__ inline int utf8_lossy(const uint8_t* p, int n, uint8_t* out) {
    int i = 0, o = 0;
    while (i < n) {
        const uint8_t b = p[i];
        int need = 0;
        uint8_t lo = 0x80, hi = 0xBF;
        if (b < 0x80) {
            if (out) out[o] = b;
            ++o;
            ++i;
            continue;
        } else if (b >= 0xC2 && b <= 0xDF) {
            need = 1;
        } else if (b == 0xE0) {
            need = 2, lo = 0xA0;
        } else if ((b >= 0xE1 && b <= 0xEC) || b == 0xEE || b == 0xEF) {
            need = 2;
        } else if (b == 0xED) {
            need = 2, hi = 0x9F;
        } else if (b == 0xF0) {
            need = 3, lo = 0x90;
        } else if (b >= 0xF1 && b <= 0xF3) {
            need = 3;
        } else if (b == 0xF4) {
            need = 3, hi = 0x8F;
        }
        int j = i + 1, got = 0;
        if (need) {
            for (; got < need && j < n; ++got, ++j) {
                const uint8_t c = p[j];
                const uint8_t l = got == 0 ? lo : 0x80, h = got == 0 ? hi : 0xBF;
                if (c < l || c > h) break;
            }
        }
        if (need && got == need) {
            for (int k = i; k < j; ++k)
                if (out) out[o + (k - i)] = p[k];
            o += j - i;
        } else {
            if (out) out[o] = 0xEF, out[o + 1] = 0xBF, out[o + 2] = 0xBD;
            o += 3;
        }
        i = j;
    }
    return o;
}

__device__ inline uint32_t ld_u32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ inline uint16_t ld_u16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

// Per-record layout (SAMv1 §4.2): after block_size: refID@0 pos@4 l_read_name@8 mapq@9
// bin@10 n_cigar_op@12 flag@14 l_seq@16 next_refID@20 next_pos@24 tlen@28 read_name@32,
// cigar, seq ((l_seq+1)/2), qual (l_seq), tags.
struct RecView {
    const uint8_t* b;  // first byte after block_size
    uint32_t bsize;
    int32_t ref_id, pos;
    uint32_t l_name, n_cigar, flag, l_seq;
    __device__ void load(const uint8_t* raw, int64_t off) {
        bsize = ld_u32(raw + off);
        b = raw + off + 4;
        ref_id = (int32_t)ld_u32(b);
        pos = (int32_t)ld_u32(b + 4);
        l_name = b[8];
        n_cigar = ld_u16(b + 12);
        flag = ld_u16(b + 14);
        l_seq = ld_u32(b + 16);
    }
    __device__ const uint8_t* name() const { return b + 32; }
    __device__ const uint8_t* cigar() const { return b + 32 + l_name; }
    __device__ const uint8_t* seq() const { return cigar() + 4u * n_cigar; }
    __device__ const uint8_t* qual() const { return seq() + (l_seq + 1) / 2; }
    // bytes the fixed fields + variable fields need (sanity against block_size)
    __device__ bool fits() const {
        return bsize >= 32 && (uint64_t)32 + l_name + 4ull * n_cigar + (l_seq + 1ull) / 2 + l_seq <= bsize;
    }
};

// name length without the NUL terminator
__device__ inline uint32_t qname_len(const RecView& r) { return r.l_name ? r.l_name - 1 : 0; }

// noodles: a read name of "*" is a missing name (-> "unknown", bam.rs:178-180)
__device__ inline bool noodles_missing_name(const RecView& r) {
    return r.l_name == 0 || (r.l_name == 2 && r.name()[0] == '*');
}

struct FieldsOut {
    int64_t* len[4];      // name, chrom, sequence, quality_scores (output bytes per row)
    uint64_t* valid[7];   // chrom, start, end, sequence, quality_scores (bitmap words); [0..4]
    uint32_t* start;
    uint32_t* end;
    uint32_t* flags;
    int32_t* chrom_id;    // resolved reference index or -1
    unsigned long long* bad;  // records whose fields overrun block_size
};

template <int MODE>
__global__ __launch_bounds__(256) void k_bam_fields(const uint8_t* __restrict__ raw, const int64_t* __restrict__ roff,
                                                    int64_t n, const int64_t* __restrict__ ref_off, int32_t n_ref,
                                                    FieldsOut o) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool v_chrom = false, v_start = false, v_end = false, v_seq = false, v_qual = false;
    if (r < n) {
        RecView rv;
        rv.load(raw, roff[r]);
        if (!rv.fits()) {
            atomicAdd(o.bad, 1ull);
            rv.l_name = 0, rv.n_cigar = 0, rv.l_seq = 0;
        }
        // --- name
        int64_t name_len;
        const uint32_t ql = qname_len(rv);
        if (MODE == ROGTK_BAM_NOODLES && noodles_missing_name(rv)) {
            name_len = 7;  // "unknown"
        } else {
            bool ascii = true;
            for (uint32_t i = 0; i < ql; ++i) ascii &= rv.name()[i] < 0x80;
            name_len = ascii ? ql : utf8_lossy(rv.name(), (int)ql, nullptr);
        }
        // --- chrom: tid in [0, n_ref) (bam.rs:186-197, 3052-3062; bam_htslib.rs:178-183)
        int32_t cid = (rv.ref_id >= 0 && rv.ref_id < n_ref) ? rv.ref_id : -1;
        v_chrom = cid >= 0;
        // --- positions
        uint32_t start = 0, end = 0;
        if (MODE == ROGTK_BAM_HTSLIB) {  // bam.rs:3064-3073: 1-based start, end = start + seq_len - 1
            v_start = v_end = rv.pos >= 0;
            start = (uint32_t)rv.pos + 1u;
            end = start + rv.l_seq - 1u;
        } else {
            // reference length of the CIGAR: M D N = X (noodles calculate_bam_alignment_length
            // bam.rs:3238-3256; htslib bam_cigar2rlen)
            uint32_t rlen = 0;
            const uint8_t* cg = rv.cigar();
            for (uint32_t k = 0; k < rv.n_cigar; ++k) {
                const uint32_t op = ld_u32(cg + 4 * k);
                const uint32_t kind = op & 15u;
                if (kind == 0 || kind == 2 || kind == 3 || kind == 7 || kind == 8) rlen += op >> 4;
            }
            if (MODE == ROGTK_BAM_NOODLES) {  // bam.rs:199-211: 1-based, end = start + ref_len - 1
                v_start = v_end = rv.pos >= 0;
                start = (uint32_t)rv.pos + 1u;
                end = start + rlen - 1u;
            } else {  // bam_htslib.rs:186-193: 0-based start, end = bam_endpos if > pos else start
                v_start = rv.pos >= 0;
                start = (uint32_t)rv.pos;
                const int64_t ref_end = ((rv.flag & 4u) == 0 && rv.n_cigar > 0) ? (int64_t)rv.pos + rlen
                                                                                : (int64_t)rv.pos + 1;
                if (ref_end > (int64_t)rv.pos) {
                    v_end = true;
                    end = (uint32_t)ref_end;
                } else {
                    v_end = v_start;
                    end = start;
                }
            }
        }
        // --- sequence / qualities
        v_seq = rv.l_seq > 0;
        if (MODE == ROGTK_BAM_HTSLIB)  // bam.rs:3095-3101: missing qualities (0xFF) -> null
            v_qual = rv.l_seq > 0 && rv.qual()[0] != 0xFF;
        else
            v_qual = rv.l_seq > 0;
        o.len[0][r] = name_len;
        o.len[1][r] = v_chrom ? ref_off[cid + 1] - ref_off[cid] : 0;
        o.len[2][r] = v_seq ? rv.l_seq : 0;
        o.len[3][r] = v_qual ? rv.l_seq : 0;
        o.start[r] = v_start ? start : 0;
        o.end[r] = v_end ? end : 0;
        o.flags[r] = rv.flag;
        o.chrom_id[r] = cid;
    }
    // validity bitmaps: one 64-bit word per wave (lane order = Arrow LSB order)
    const bool vs[5] = {v_chrom, v_start, v_end, v_seq, v_qual};
    const int64_t w = r >> 6;
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        const uint64_t bits = __ballot(vs[c]);
        if ((threadIdx.x & 63) == 0 && w * 64 < n) o.valid[c][w] = bits;
    }
}

struct FillIn {
    const int64_t* off[4];  // output offsets (exclusive scan of len, n + 1)
    uint8_t* val[4];
    const int64_t* len[4];
    const int32_t* chrom_id;
    const int64_t* ref_off;
    const uint8_t* ref_val;
    int include_seq, include_qual;
};

__device__ inline uint8_t base_ascii(uint32_t nib, int mode) {
    // decode_base (bam.rs:3227-3236, 3083-3091): 1 A, 2 C, 4 G, 8 T, else N;
    // htslib seq_nt16_str for ROGTK_BAM_HTSLIB_BLOCKS (`seq().as_bytes()`, bam_htslib.rs:199)
    if (mode == ROGTK_BAM_HTSLIB_BLOCKS) {
        const char* t = "=ACMGRSVTWYHKDBN";
        return (uint8_t)t[nib & 15];
    }
    switch (nib) {
        case 1: return 'A';
        case 2: return 'C';
        case 4: return 'G';
        case 8: return 'T';
        default: return 'N';
    }
}

// One wave per record.
template <int MODE>
__global__ __launch_bounds__(256) void k_bam_fill(const uint8_t* __restrict__ raw, const int64_t* __restrict__ roff,
                                                  int64_t n, FillIn f) {
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (r >= n) return;
    RecView rv;
    rv.load(raw, roff[r]);
    if (!rv.fits()) rv.l_name = 0, rv.n_cigar = 0, rv.l_seq = 0;
    // name
    {
        uint8_t* out = f.val[0] + f.off[0][r];
        const uint32_t ql = qname_len(rv);
        if (MODE == ROGTK_BAM_NOODLES && noodles_missing_name(rv)) {
            if (lane < 7) out[lane] = (uint8_t)"unknown"[lane];
        } else if (f.len[0][r] == (int64_t)ql) {
            for (uint32_t i = lane; i < ql; i += 64) out[i] = rv.name()[i];
        } else if (lane == 0) {
            utf8_lossy(rv.name(), (int)ql, out);
        }
    }
    // chrom
    if (f.chrom_id[r] >= 0) {
        const int32_t c = f.chrom_id[r];
        const int64_t a = f.ref_off[c], len = f.ref_off[c + 1] - a;
        uint8_t* out = f.val[1] + f.off[1][r];
        for (int64_t i = lane; i < len; i += 64) out[i] = f.ref_val[a + i];
    }
    // sequence: 4-bit codes, high nibble first
    if (f.include_seq && f.len[2][r] > 0) {
        const uint8_t* s = rv.seq();
        uint8_t* out = f.val[2] + f.off[2][r];
        for (uint32_t i = lane; i < rv.l_seq; i += 64) {
            const uint8_t byte = s[i >> 1];
            out[i] = base_ascii((i & 1) ? (byte & 15u) : (byte >> 4), MODE);
        }
    }
    // qualities: PHRED + 33, wrapping u8 add (quality_to_string_zero_copy, bam.rs:2622-2636)
    if (f.include_qual && f.len[3][r] > 0) {
        const uint8_t* q = rv.qual();
        uint8_t* out = f.val[3] + f.off[3][r];
        for (uint32_t i = lane; i < rv.l_seq; i += 64) out[i] = (uint8_t)(q[i] + 33u);
    }
}

// UMI of each record for the H1-H3 engine: source 0 = the first umi_len bases of the
// decoded sequence, 1 = the read name after its last `sep` byte (UMI-tools
// READNAME_<UMI> convention). Null when the sequence is null / the name has no sep.
__global__ __launch_bounds__(256) void k_umi_len(const int64_t* __restrict__ seq_off, const uint64_t* __restrict__ seq_valid,
                                                 const int64_t* __restrict__ name_off, const uint8_t* __restrict__ name_val,
                                                 int64_t n, int source, int umi_len, int sep, int64_t* len,
                                                 int64_t* start, uint64_t* valid, int64_t row_base = -1) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool v = false;
    if (r < n) {
        int64_t a = 0, l = 0;
        if (source == 0) {
            v = !seq_valid || ((seq_valid[r >> 6] >> (r & 63)) & 1);
            a = seq_off[r];
            l = v ? min<int64_t>(umi_len, seq_off[r + 1] - a) : 0;
        } else {
            const int64_t b = name_off[r], e = name_off[r + 1];
            int64_t k = e - 1;
            while (k >= b && name_val[k] != (uint8_t)sep) --k;
            v = k >= b;
            a = k + 1;
            l = v ? e - a : 0;
        }
        len[r] = l;
        start[r] = a;
    }
    const uint64_t bits = __ballot(v);
    if ((threadIdx.x & 63) == 0 && (r >> 6) * 64 < n) {
        if (row_base < 0) {
            valid[r >> 6] = bits;
        } else {  // append: the wave's 64 rows start at bit row_base + r of a zeroed bitmap
            const int64_t g = row_base + r;
            const int sh = (int)(g & 63);
            if (bits) {
                atomicOr((unsigned long long*)valid + (g >> 6), (unsigned long long)(bits << sh));
                if (sh && (bits >> (64 - sh))) atomicOr((unsigned long long*)valid + (g >> 6) + 1,
                                                        (unsigned long long)(bits >> (64 - sh)));
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_umi_fill(const uint8_t* __restrict__ src, const int64_t* __restrict__ start,
                                                  const int64_t* __restrict__ off, int64_t n, uint8_t* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t a = start[r], o = off[r], l = off[r + 1] - o;
    for (int64_t i = 0; i < l; ++i) out[o + i] = src[a + i];
}

// Append mode (rogtk_bam_umi_append / rogtk_bam_append_strings): a batch's offsets, scanned
// from 0, are moved to the column's running byte count *base (device), which then moves
// to the new total; no host round trip. The copy kernels skip rows past cap and count them
// in *ovf (checked once per column by the caller).
__global__ __launch_bounds__(256) void k_add_base(int64_t* __restrict__ off, int64_t n1, const int64_t* __restrict__ base) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n1) off[i] += *base;
}
__global__ void k_set_base(const int64_t* __restrict__ off_end, int64_t* __restrict__ base) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *base = *off_end;
}
// one wave per row: out[off[r] ..] = src[start[r] ..] (len = off[r+1] - off[r])
__global__ __launch_bounds__(256) void k_copy_rows(const uint8_t* __restrict__ src, const int64_t* __restrict__ start,
                                                   const int64_t* __restrict__ off, int64_t n, int64_t cap,
                                                   uint8_t* __restrict__ out, unsigned long long* __restrict__ ovf) {
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (r >= n) return;
    const int64_t a = start[r], o = off[r], l = off[r + 1] - o;
    if (o + l > cap) {
        if (lane == 0) atomicAdd(ovf, 1ull);
        return;
    }
    for (int64_t i = lane; i < l; i += 64) out[o + i] = src[a + i];
}

// ------------------------------------------------------------------ host
struct PinnedBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    int ensure(size_t bytes, size_t keep = 0) {
        if (bytes <= cap && p) return ROGTK_OK;
        size_t want = std::max<size_t>(bytes + bytes / 2, 1 << 20);
        uint8_t* q = nullptr;
        ROGTK_HIP_CHECK(hipHostMalloc((void**)&q, want, hipHostMallocDefault));
        if (p && keep) memcpy(q, p, keep);
        if (p) (void)hipHostFree(p);
        p = q;
        cap = want;
        return ROGTK_OK;
    }
};

inline double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One cached pinned stream buffer, handed from a closed reader to the next one opened
// (page-locking hundreds of MB costs more than decoding them).
// Stream buffers of closed readers, reused by the next ones (a pinned allocation of the
// size a file's stream needs costs ~0.2 s): a pool, so the concurrent range readers of one
// file (rogtk_amd/bam.py bams_umi_cluster) each find one after the first call (round 5;
// one cached buffer left three of four range readers growing their own)
constexpr size_t kPinPool = 8;
std::mutex g_pin_mu;
std::vector<PinnedBuf*> g_pin_pool;

// Round 6: the pool is warmed when the first reader of a process opens: kPinWarm buffers
// (concurrent range readers: one per range of a rank, bams_umi_cluster) of the size stream
// buffers reach (g_pin_hint: the largest pinned so far, at least kPinWarmBytes), pinned by one
// thread each, joined before the open returns (concurrent opens wait in call_once), so the
// range readers of a rank's first call take pooled buffers instead of page-locking and
// growing their own inside the call.
constexpr size_t kPinWarm = 4;
constexpr size_t kPinWarmBytes = (size_t)256 << 20;
size_t g_pin_hint = 0;  // the largest stream buffer pinned so far (guarded by g_pin_mu)
std::once_flag g_pin_warm_once;

void pin_note(size_t cap) {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pin_hint = std::max(g_pin_hint, cap);
}

void pin_warm(size_t n, size_t bytes) {
    std::vector<PinnedBuf*> got(n, nullptr);
    std::vector<std::thread> th;
    for (size_t i = 0; i < n; ++i)
        th.emplace_back([&got, i, bytes] {
            auto* b = new PinnedBuf();
            if (b->ensure(bytes) == ROGTK_OK) got[i] = b;  // (ensure pins 1.5x bytes)
            else delete b;
        });
    for (auto& t : th) t.join();
    std::lock_guard<std::mutex> lk(g_pin_mu);
    for (PinnedBuf* b : got) {
        if (b && g_pin_pool.size() < kPinPool) g_pin_pool.push_back(b);
        else delete b;
    }
}

void pin_take(PinnedBuf& b) {  // the largest pooled buffer, if any
    std::lock_guard<std::mutex> lk(g_pin_mu);
    if (g_pin_pool.empty()) return;
    auto best = std::max_element(g_pin_pool.begin(), g_pin_pool.end(),
                                 [](const PinnedBuf* x, const PinnedBuf* y) { return x->cap < y->cap; });
    std::swap(b.p, (*best)->p);
    std::swap(b.cap, (*best)->cap);
    delete *best;
    g_pin_pool.erase(best);
}

void pin_give(PinnedBuf& b) {  // back to the pool (the smallest pooled one freed when full)
    if (!b.p) return;
    std::lock_guard<std::mutex> lk(g_pin_mu);
    if (g_pin_pool.size() >= kPinPool) {
        auto small = std::min_element(g_pin_pool.begin(), g_pin_pool.end(),
                                      [](const PinnedBuf* x, const PinnedBuf* y) { return x->cap < y->cap; });
        if ((*small)->cap >= b.cap) return;  // b is freed by its owner
        delete *small;
        g_pin_pool.erase(small);
    }
    auto* keep = new PinnedBuf();
    std::swap(keep->p, b.p);
    std::swap(keep->cap, b.cap);
    g_pin_pool.push_back(keep);
}

struct Bgzf {
    // diagnostics (rogtk_bam_timers), seconds on the caller's thread: t_read file reads,
    // t_move framing of blocks + buffer moves (includes t_read), t_inflate inflating or
    // waiting for the read-ahead thread; t_read_bg: reads overlapped with an inflate;
    // t_ahead: busy seconds of the read-ahead thread
    double t_read = 0, t_inflate = 0, t_move = 0, t_ahead = 0, t_read_bg = 0;
    FILE* f = nullptr;
    int threads = 1;
    bool file_eof = false;
    std::vector<uint8_t> comp;  // compressed bytes not yet inflated: [0, comp_len)
    size_t comp_len = 0;
    PinnedBuf buf;              // uncompressed stream: [pos, end)
    size_t pos = 0, end = 0;
    std::string err;
    // compressed bytes read per step (ROGTK_BAM_CHUNK overrides, read at open: tests use
    // small chunks to cover many read-ahead steps and buffer moves with small files)
    size_t chunk = [] {
        const char* e = getenv("ROGTK_BAM_CHUNK");
        const long long v = e ? atoll(e) : 0;
        return v >= 4096 ? (size_t)v : (size_t)(32u << 20);
    }();

    // Read-ahead (ROGTK_BAM_READAHEAD=0: off). While the caller frames, decodes and uses
    // a batch, one thread keeps reading and inflating whole chunks into buf behind `end`
    // ([end, ahead_end)) until the buffer is full or the file ends; the caller takes what
    // has arrived and joins the thread only to compact the buffer. While it runs, only
    // the thread touches comp / comp_len / file_eof / f and the bytes past `end`; the
    // caller reads [pos, end) and moves pos.
    bool readahead = [] {
        const char* e = getenv("ROGTK_BAM_READAHEAD");
        return !(e && e[0] == '0');
    }();
    std::thread ahead;
    bool ahead_on = false;
    std::mutex ahead_mu;
    std::condition_variable ahead_cv;
    size_t ahead_end = 0;     // guarded by ahead_mu
    bool ahead_done = false;  // guarded by ahead_mu
    std::string ahead_err;    // set by the thread, read after join

    struct Blk {
        size_t h0, c0, clen, out;  // header and data offsets in comp, data bytes, offset in dst
        uint32_t isize;
    };

    // Range reading (rogtk_bam_open_range): only records that START before the block at
    // compressed offset c_end are this reader's. file_off = the file offset of comp[0];
    // u_base = the stream position of buf[0] (stream positions count from the reader's
    // first inflated byte); once the block at c_end is framed, u_limit = its stream
    // position (limit_set). Past that block the reader inflates one block at a time, only
    // as far as its last record needs.
    int64_t file_off = 0;
    int64_t c_end = -1;
    uint64_t u_base = 0;
    std::atomic<bool> limit_set{false};
    std::atomic<uint64_t> u_limit{0};

    // the blocks of comp the next inflate may take: those before c_end, or one block once
    // the range end is reached (a record straddling it needs the next block's bytes)
    size_t frame_cap() const {
        if (c_end < 0) return SIZE_MAX;
        return c_end > file_off ? (size_t)(c_end - file_off) : 0;
    }

    // Before inflating blks into dst: note the stream position of the block at c_end.
    void note_limit(const std::vector<Blk>& blks, const uint8_t* dst) {
        if (c_end < 0 || limit_set.load()) return;
        for (const Blk& k : blks)
            if (file_off + (int64_t)k.h0 >= c_end) {
                u_limit.store(u_base + (uint64_t)(dst - buf.p) + k.out);
                limit_set.store(true);
                return;
            }
    }

    ~Bgzf() { stop_ahead(); }

    void read_comp() {
        if (file_eof) return;
        if (comp.size() < comp_len + chunk) comp.resize(comp_len + chunk);
        const size_t got = fread(comp.data() + comp_len, 1, chunk, f);
        comp_len += got;
        if (got < chunk) file_eof = true;
    }

    // Frame the whole BGZF blocks at the start of comp. false + e set on a malformed block.
    // max_off: no block starting at or past it is framed, unless it is the first one (then
    // exactly that block).
    static bool frame(const std::vector<uint8_t>& comp, size_t comp_len, std::vector<Blk>& blks, size_t& o,
                      size_t& total, std::string& e, size_t max_off = SIZE_MAX) {
        blks.clear();
        o = total = 0;
        while (o + 18 <= comp_len) {
            if (o >= max_off && !blks.empty()) break;
            const uint8_t* h = comp.data() + o;
            if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) {
                e = "not a BGZF file (bad gzip block header)";
                return false;
            }
            const size_t xlen = h[10] | (h[11] << 8);
            if (o + 12 + xlen > comp_len) break;
            size_t bsize = 0;
            for (size_t x = 0; x + 4 <= xlen;) {
                const uint8_t* sf = h + 12 + x;
                const size_t slen = sf[2] | (sf[3] << 8);
                if (sf[0] == 'B' && sf[1] == 'C' && slen == 2) bsize = (size_t)(sf[4] | (sf[5] << 8)) + 1;
                x += 4 + slen;
            }
            if (bsize == 0) {
                e = "BGZF block without a BC (BSIZE) subfield";
                return false;
            }
            if (o + bsize > comp_len) break;
            const uint8_t* t = h + bsize - 4;
            const uint32_t isize = t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24);
            const size_t c0 = o + 12 + xlen;
            if (bsize < 12 + xlen + 8) {
                e = "corrupt BGZF block (BSIZE too small)";
                return false;
            }
            blks.push_back({o, c0, bsize - 12 - xlen - 8, total, isize});
            total += isize;
            o += bsize;
            if (o > max_off) break;  // the one block at or past max_off
        }
        return true;
    }

    // Inflate blks (framed from comp) into dst on `threads` threads. The calling thread
    // reads the next compressed chunk meanwhile (past comp_len: room is made first, so
    // no worker's input moves), then drops the consumed [0, o) from comp.
    bool inflate_blocks(const std::vector<Blk>& blks, size_t o, uint8_t* dst, std::string& e, double* t_rd) {
        std::atomic<size_t> next{0};
        std::atomic<bool> bad{false};
        auto work = [&] {
            z_stream zs;
            memset(&zs, 0, sizeof zs);
            if (inflateInit2(&zs, -15) != Z_OK) {
                bad = true;
                return;
            }
            for (size_t b; (b = next.fetch_add(1)) < blks.size();) {
                const Blk& k = blks[b];
                inflateReset(&zs);
                zs.next_in = comp.data() + k.c0;
                zs.avail_in = (uInt)k.clen;
                zs.next_out = dst + k.out;
                zs.avail_out = k.isize;
                const int rc = ::inflate(&zs, Z_FINISH);
                if (rc != Z_STREAM_END || zs.avail_out != 0) bad = true;
            }
            inflateEnd(&zs);
        };
        const bool read_next = !file_eof && comp_len - o < chunk;
        if (read_next && comp.size() < comp_len + chunk) comp.resize(comp_len + chunk);
        const int nt = (int)std::min<size_t>((size_t)std::max(threads, 1), blks.size());
        std::vector<std::thread> th;
        for (int t = (read_next ? 0 : 1); t < nt; ++t) th.emplace_back(work);
        if (read_next) {
            const double t0 = now_s();
            read_comp();
            *t_rd += now_s() - t0;
        }
        work();
        for (auto& t : th) t.join();
        if (bad) {
            e = "BGZF inflate failed (corrupt deflate stream)";
            return false;
        }
        memmove(comp.data(), comp.data() + o, comp_len - o);
        comp_len -= o;
        file_off += (int64_t)o;
        return true;
    }

    void start_ahead() {
        if (!readahead || ahead_on || !err.empty() || (file_eof && comp_len == 0) || limit_set.load()) return;
        ahead_end = end;
        ahead_done = false;
        ahead_on = true;
        ahead = std::thread([this, e0 = end] {
            const double t0 = now_s();
            double t_rd = 0;
            std::vector<Blk> blks;
            size_t e = e0;
            std::string er;
            for (;;) {
                if (comp_len < chunk && !file_eof) read_comp();
                if (limit_set.load()) break;  // past the range end: the caller reads on demand
                size_t o = 0, total = 0;
                if (!frame(comp, comp_len, blks, o, total, er, frame_cap())) break;
                if (blks.empty()) {  // end of input, or a block longer than what is buffered
                    if (file_eof) break;
                    read_comp();
                    continue;
                }
                if (e + total > buf.cap) break;
                note_limit(blks, buf.p + e);
                if (!inflate_blocks(blks, o, buf.p + e, er, &t_rd)) break;
                e += total;
                std::lock_guard<std::mutex> lk(ahead_mu);
                ahead_end = e;
                ahead_cv.notify_all();
            }
            std::lock_guard<std::mutex> lk(ahead_mu);
            ahead_err = er;
            ahead_done = true;
            t_ahead += now_s() - t0;
            ahead_cv.notify_all();
        });
    }

    void stop_ahead() {
        if (!ahead_on) return;
        ahead.join();
        ahead_on = false;
        end = std::max(end, ahead_end);
        if (err.empty() && !ahead_err.empty()) err = ahead_err;
        ahead_err.clear();
    }

    // Make more bytes available after `end`, keeping the bytes from `keep_from` on (they
    // may move to the front). Returns false at end of input or on error.
    bool more(size_t keep_from) {
        if (!err.empty()) return false;
        if (ahead_on) {
            const double t0 = now_s();
            bool done;
            size_t ae;
            {
                std::unique_lock<std::mutex> lk(ahead_mu);
                ahead_cv.wait(lk, [&] { return ahead_done || ahead_end > end; });
                done = ahead_done;
                ae = ahead_end;
            }
            t_inflate += now_s() - t0;
            if (!done) {  // the thread carries on behind the new end
                end = ae;
                return true;
            }
            const size_t before = end;
            stop_ahead();
            if (!err.empty()) return false;
            if (end > before) {
                start_ahead();
                return true;
            }
            // the thread stopped with nothing new: buffer full (or end of input); go on here
        }
        // read compressed bytes
        double t0 = now_s();
        if (comp_len < chunk) read_comp();
        std::vector<Blk> blks;
        size_t o = 0, total = 0;
        for (;;) {
            if (!frame(comp, comp_len, blks, o, total, err, frame_cap())) return false;
            if (!blks.empty() || file_eof) break;
            read_comp();  // a block longer than what is buffered (small ROGTK_BAM_CHUNK)
        }
        t_read += now_s() - t0;
        if (blks.empty()) {
            if (file_eof && comp_len > 0) err = "truncated BGZF block at end of file";
            return false;
        }
        // make room. Append in place while the buffer has space; otherwise move the
        // bytes still needed ([keep_from, end)) to the front, growing the buffer
        // geometrically if they do not fit (one move per batch in steady state).
        if (end + total > buf.cap) {
            const size_t keep = end - keep_from;
            const size_t need = keep + total;
            if (need > buf.cap) {
                PinnedBuf nb;
                if (nb.ensure(std::max(need, 2 * buf.cap)) != ROGTK_OK) {
                    err = "pinned host allocation failed";
                    return false;
                }
                pin_note(nb.cap);
                if (keep) memcpy(nb.p, buf.p + keep_from, keep);
                std::swap(buf.p, nb.p);
                std::swap(buf.cap, nb.cap);
            } else if (keep && keep_from) {
                memmove(buf.p, buf.p + keep_from, keep);
            }
            pos -= keep_from;
            end = keep;
            u_base += keep_from;
        }
        // inflate blocks in parallel
        const double t1 = now_s();
        t_move += t1 - t0;
        note_limit(blks, buf.p + end);
        if (!inflate_blocks(blks, o, buf.p + end, err, &t_read_bg)) return false;
        t_inflate += now_s() - t1;
        end += total;
        start_ahead();
        return true;
    }
    // at least n bytes available from pos + rel (compacting [pos, end) to the front)
    bool ensure_rel(size_t rel, size_t n) {
        while (end - pos < rel + n)
            if (!more(pos)) return false;
        return true;
    }
};

struct BamReader {
    Bgzf z;
    double t_frame = 0, t_decode = 0, t_d2h = 0;
    std::string text;
    std::vector<int64_t> ref_off{0};
    std::vector<uint8_t> ref_val;
    int device = -1;
    hipStream_t stream = nullptr;
    // range reading: bytes of this range's last record past the range end (the next
    // range's skip), -1 until the range is exhausted / for a whole-file reader
    int64_t tail = -1;
    // batch state
    int64_t n = 0;
    std::vector<int64_t> roff;  // record offsets relative to batch start (n + 1)
    DevBuf d_raw, d_roff, d_len[4], d_off[4], d_val[4], d_valid[5], d_start, d_end, d_flags, d_cid, d_ref_off,
        d_ref_val, d_bad, d_cub;
    // device mode (rogtk_bam_next_dev): the value buffers are sized from host-known bounds
    // (no host sync per batch); d_bad accumulates over the batches and is checked by
    // rogtk_bam_check. copied: fires when the batch's H2D copy of the stream buffer is done
    // (the next framing may move those bytes: it waits for it first).
    bool bad_cleared = false;
    hipEvent_t copied = nullptr;
    bool copy_pending = false;
    int32_t max_ref_len = 0;
    // host outputs (pinned)
    PinnedBuf h_off[4], h_val[4], h_valid[5], h_u32[3];
    ~BamReader() {
        z.stop_ahead();  // the read-ahead thread uses the file and the stream buffer
        if (z.f) fclose(z.f);
        pin_give(z.buf);
        if (copied) (void)hipEventDestroy(copied);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// lossy UTF-8 (String::from_utf8_lossy) on the host, for header reference names
std::string lossy_host(const uint8_t* p, int n) {
    std::string s((size_t)utf8_lossy(p, n, nullptr), '\0');
    utf8_lossy(p, n, (uint8_t*)&s[0]);
    return s;
}

int read_header(BamReader* R) {
    auto need = [&](size_t n) -> int {
        ROGTK_REQUIRE(R->z.ensure_rel(0, n), ROGTK_E_INVALID, "BAM header: %s",
                      R->z.err.empty() ? "unexpected end of file" : R->z.err.c_str());
        return ROGTK_OK;
    };
    auto rd32 = [&]() {
        const uint8_t* p = R->z.buf.p + R->z.pos;
        R->z.pos += 4;
        return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
    };
    int rc;
    if ((rc = need(8)) != ROGTK_OK) return rc;
    ROGTK_REQUIRE(memcmp(R->z.buf.p + R->z.pos, "BAM\1", 4) == 0, ROGTK_E_INVALID, "not a BAM file (bad magic)");
    R->z.pos += 4;
    const int32_t l_text = rd32();
    ROGTK_REQUIRE(l_text >= 0, ROGTK_E_INVALID, "BAM header: negative l_text");
    if ((rc = need((size_t)l_text + 4)) != ROGTK_OK) return rc;
    R->text.assign((const char*)R->z.buf.p + R->z.pos, (size_t)l_text);
    R->z.pos += l_text;
    const int32_t n_ref = rd32();
    ROGTK_REQUIRE(n_ref >= 0, ROGTK_E_INVALID, "BAM header: negative n_ref");
    for (int32_t i = 0; i < n_ref; ++i) {
        if ((rc = need(4)) != ROGTK_OK) return rc;
        const int32_t l_name = rd32();
        ROGTK_REQUIRE(l_name >= 1, ROGTK_E_INVALID, "BAM header: bad reference name length");
        if ((rc = need((size_t)l_name + 4)) != ROGTK_OK) return rc;
        const std::string nm = lossy_host(R->z.buf.p + R->z.pos, l_name - 1);
        R->z.pos += l_name;
        (void)rd32();  // l_ref
        R->ref_val.insert(R->ref_val.end(), nm.begin(), nm.end());
        R->ref_off.push_back((int64_t)R->ref_val.size());
    }
    return ROGTK_OK;
}

constexpr size_t kMaxBatchBytes = size_t(1) << 30;

// Frame up to max_records records from the stream; leaves them at [pos, pos + roff[n]).
int frame_batch(BamReader* R, int64_t max_records) {
    Bgzf& z = R->z;
    R->roff.assign(1, 0);
    size_t rel = 0;  // bytes of the batch framed so far (from z.pos)
    int64_t n = 0;
    while (n < max_records && rel < kMaxBatchBytes) {
        if (!z.ensure_rel(rel, 4)) {
            ROGTK_REQUIRE(z.err.empty(), ROGTK_E_INVALID, "BAM: %s", z.err.c_str());
            ROGTK_REQUIRE(z.end - z.pos == rel, ROGTK_E_INVALID,
                          "BAM: truncated record at end of file (%zu stray bytes)", z.end - z.pos - rel);
            break;  // clean end of file
        }
        if (z.limit_set.load()) {  // a record that starts at or past the range end is the next range's
            const uint64_t at = z.u_base + z.pos + rel, lim = z.u_limit.load();
            if (at >= lim) {
                R->tail = (int64_t)(at - lim);
                break;
            }
        }
        const uint8_t* p = z.buf.p + z.pos + rel;
        const uint32_t bs = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
        ROGTK_REQUIRE(bs >= 32 && bs < (1u << 30), ROGTK_E_INVALID, "BAM: invalid record block_size %u", bs);
        ROGTK_REQUIRE(z.ensure_rel(rel, 4 + (size_t)bs), ROGTK_E_INVALID, "BAM: %s",
                      z.err.empty() ? "truncated record at end of file" : z.err.c_str());
        rel += 4 + bs;
        ++n;
        R->roff.push_back((int64_t)rel);
    }
    R->n = n;
    return ROGTK_OK;
}

// sync_totals: size the value buffers from the scanned totals (one host sync per batch:
// the host path, which copies the columns back anyway) or from bounds known on the host
// (device path: name <= 3 bytes per raw byte + 7 per record (U+FFFD per invalid byte,
// "unknown"), chrom <= the longest reference name per record, sequence / qualities <= the
// raw bytes), so that the host never waits for the GPU inside a file.
int decode_batch(BamReader* R, int mode, int include_seq, int include_qual, bool sync_totals = true) {
    const int64_t n = R->n;
    hipStream_t s = R->stream;
    const int64_t bytes = R->roff[n];
    if (R->d_raw.ensure((size_t)std::max<int64_t>(bytes, 4)) != ROGTK_OK ||
        R->d_roff.ensure((size_t)(n + 1) * 8) != ROGTK_OK)
        return ROGTK_E_HIP;
    if (bytes) ROGTK_HIP_CHECK(hipMemcpyAsync(R->d_raw.p, R->z.buf.p + R->z.pos, bytes, hipMemcpyHostToDevice, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(R->d_roff.p, R->roff.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, s));
    if (!R->copied) ROGTK_HIP_CHECK(hipEventCreateWithFlags(&R->copied, hipEventDisableTiming));
    ROGTK_HIP_CHECK(hipEventRecord(R->copied, s));
    R->copy_pending = true;
    const int64_t words = (n + 63) / 64;
    for (int c = 0; c < 4; ++c) {
        if (R->d_len[c].ensure((size_t)(n + 1) * 8) != ROGTK_OK || R->d_off[c].ensure((size_t)(n + 1) * 8) != ROGTK_OK)
            return ROGTK_E_HIP;
    }
    for (int c = 0; c < 5; ++c)
        if (R->d_valid[c].ensure((size_t)std::max<int64_t>(words, 1) * 8) != ROGTK_OK) return ROGTK_E_HIP;
    if (R->d_start.ensure((size_t)std::max<int64_t>(n, 1) * 4) != ROGTK_OK ||
        R->d_end.ensure((size_t)std::max<int64_t>(n, 1) * 4) != ROGTK_OK ||
        R->d_flags.ensure((size_t)std::max<int64_t>(n, 1) * 4) != ROGTK_OK ||
        R->d_cid.ensure((size_t)std::max<int64_t>(n, 1) * 4) != ROGTK_OK || R->d_bad.ensure(8) != ROGTK_OK)
        return ROGTK_E_HIP;
    if (sync_totals || !R->bad_cleared) {
        ROGTK_HIP_CHECK(hipMemsetAsync(R->d_bad.p, 0, 8, s));
        R->bad_cleared = !sync_totals;
    }
    FieldsOut fo;
    for (int c = 0; c < 4; ++c) fo.len[c] = R->d_len[c].as<int64_t>();
    for (int c = 0; c < 5; ++c) fo.valid[c] = R->d_valid[c].as<uint64_t>();
    fo.start = R->d_start.as<uint32_t>();
    fo.end = R->d_end.as<uint32_t>();
    fo.flags = R->d_flags.as<uint32_t>();
    fo.chrom_id = R->d_cid.as<int32_t>();
    fo.bad = R->d_bad.as<unsigned long long>();
    const int32_t n_ref = (int32_t)R->ref_off.size() - 1;
    if (n > 0) {
        ProfScope prof(K_BAM_FIELDS, s);
        const dim3 g((unsigned)((n + 255) / 256));
        if (mode == ROGTK_BAM_NOODLES)
            hipLaunchKernelGGL(k_bam_fields<ROGTK_BAM_NOODLES>, g, dim3(256), 0, s, R->d_raw.as<uint8_t>(),
                               R->d_roff.as<int64_t>(), n, R->d_ref_off.as<int64_t>(), n_ref, fo);
        else if (mode == ROGTK_BAM_HTSLIB)
            hipLaunchKernelGGL(k_bam_fields<ROGTK_BAM_HTSLIB>, g, dim3(256), 0, s, R->d_raw.as<uint8_t>(),
                               R->d_roff.as<int64_t>(), n, R->d_ref_off.as<int64_t>(), n_ref, fo);
        else
            hipLaunchKernelGGL(k_bam_fields<ROGTK_BAM_HTSLIB_BLOCKS>, g, dim3(256), 0, s, R->d_raw.as<uint8_t>(),
                               R->d_roff.as<int64_t>(), n, R->d_ref_off.as<int64_t>(), n_ref, fo);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    // exclusive scans of the four length columns (n + 1 entries: the last is the total)
    for (int c = 0; c < 4; ++c) {
        ProfScope prof_scan(K_BAM_SCAN, s);
        ROGTK_HIP_CHECK(hipMemsetAsync(R->d_len[c].as<int64_t>() + n, 0, 8, s));
        size_t tb = 0;
        ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, R->d_len[c].as<int64_t>(),
                                                         R->d_off[c].as<int64_t>(), (int)(n + 1), s));
        if (R->d_cub.ensure(tb) != ROGTK_OK) return ROGTK_E_HIP;
        ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(R->d_cub.p, tb, R->d_len[c].as<int64_t>(),
                                                         R->d_off[c].as<int64_t>(), (int)(n + 1), s));
    }
    int64_t tot[4];
    if (sync_totals) {
        unsigned long long bad = 0;
        for (int c = 0; c < 4; ++c)
            ROGTK_HIP_CHECK(hipMemcpyAsync(&tot[c], R->d_off[c].as<int64_t>() + n, 8, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipMemcpyAsync(&bad, R->d_bad.p, 8, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipStreamSynchronize(s));
        R->copy_pending = false;
        ROGTK_REQUIRE(bad == 0, ROGTK_E_INVALID, "BAM: %llu record(s) whose fields overrun their block_size", bad);
    } else {
        tot[0] = 3 * bytes + 7 * n;
        tot[1] = (int64_t)R->max_ref_len * n;
        tot[2] = include_seq ? bytes : 0;
        tot[3] = include_qual ? bytes : 0;
    }
    for (int c = 0; c < 4; ++c)
        if (R->d_val[c].ensure((size_t)std::max<int64_t>(tot[c], 1)) != ROGTK_OK) return ROGTK_E_HIP;
    FillIn fi;
    for (int c = 0; c < 4; ++c) {
        fi.off[c] = R->d_off[c].as<int64_t>();
        fi.val[c] = R->d_val[c].as<uint8_t>();
        fi.len[c] = R->d_len[c].as<int64_t>();
    }
    fi.chrom_id = R->d_cid.as<int32_t>();
    fi.ref_off = R->d_ref_off.as<int64_t>();
    fi.ref_val = R->d_ref_val.as<uint8_t>();
    fi.include_seq = include_seq;
    fi.include_qual = include_qual;
    if (n > 0) {
        ProfScope prof(K_BAM_FILL, s);
        const dim3 g((unsigned)((n * 64 + 255) / 256));
        if (mode == ROGTK_BAM_NOODLES)
            hipLaunchKernelGGL(k_bam_fill<ROGTK_BAM_NOODLES>, g, dim3(256), 0, s, R->d_raw.as<uint8_t>(),
                               R->d_roff.as<int64_t>(), n, fi);
        else if (mode == ROGTK_BAM_HTSLIB)
            hipLaunchKernelGGL(k_bam_fill<ROGTK_BAM_HTSLIB>, g, dim3(256), 0, s, R->d_raw.as<uint8_t>(),
                               R->d_roff.as<int64_t>(), n, fi);
        else
            hipLaunchKernelGGL(k_bam_fill<ROGTK_BAM_HTSLIB_BLOCKS>, g, dim3(256), 0, s, R->d_raw.as<uint8_t>(),
                               R->d_roff.as<int64_t>(), n, fi);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    return ROGTK_OK;
}

// ------------------------------------------------ splitting one file (host only)
// The reference splits a BAM at BGZF block boundaries near file_size * i / n
// (discover_split_points, bam_htslib.rs:247-290; find_nearest_bgzf_boundary :293-320)
// and seeks htslib to block << 16 (:377-393), i.e. it assumes a record starts there, which
// BAM does not promise (records straddle blocks). Here a split point is also a block
// start, but the range reader skips the tail of the record that straddles it: the skip
// is found by chained record validation (rogtk_bam_find_record) and checked against the
// previous range's tail (rogtk_bam_range_tail) by the caller, so results never depend on
// a guess.

// a complete, valid BGZF block header at p (n bytes available): its BSIZE, else 0
size_t bgzf_block_at(const uint8_t* p, size_t n) {
    if (n < 18 || p[0] != 31 || p[1] != 139 || p[2] != 8 || !(p[3] & 4)) return 0;
    const size_t xlen = p[10] | (p[11] << 8);
    if (12 + xlen > n) return 0;
    size_t bsize = 0;
    for (size_t x = 0; x + 4 <= xlen;) {
        const uint8_t* sf = p + 12 + x;
        const size_t slen = sf[2] | (sf[3] << 8);
        if (sf[0] == 'B' && sf[1] == 'C' && slen == 2) bsize = (size_t)(sf[4] | (sf[5] << 8)) + 1;
        x += 4 + slen;
    }
    return bsize >= 12 + xlen + 8 ? bsize : 0;
}

// Inflate whole BGZF blocks from file offset c0 until at least `want` bytes (or EOF).
// block_end (optional): the file offset after each block, by its stream end position.
bool inflate_from(FILE* f, int64_t c0, size_t want, std::vector<uint8_t>& out, std::string& err,
                  std::vector<std::pair<size_t, int64_t>>* block_end = nullptr) {
    out.clear();
    if (fseeko(f, (off_t)c0, SEEK_SET) != 0) {
        err = "seek failed";
        return false;
    }
    std::vector<uint8_t> comp;
    size_t clen = 0;
    bool eof = false;
    int64_t off = c0;
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) {
        err = "zlib init failed";
        return false;
    }
    while (out.size() < want) {
        if (clen < (1u << 17) && !eof) {
            comp.resize(clen + (1u << 20));
            const size_t got = fread(comp.data() + clen, 1, 1u << 20, f);
            clen += got;
            eof = got < (1u << 20);
        }
        const size_t bsize = bgzf_block_at(comp.data(), clen);
        if (!bsize || bsize > clen) {
            if (clen == 0 && eof) break;
            err = "not a BGZF block at the split point";
            inflateEnd(&zs);
            return false;
        }
        const size_t xlen = comp[10] | (comp[11] << 8);
        const uint8_t* t = comp.data() + bsize - 4;
        const uint32_t isize = t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24);
        const size_t at = out.size();
        out.resize(at + isize);
        inflateReset(&zs);
        zs.next_in = comp.data() + 12 + xlen;
        zs.avail_in = (uInt)(bsize - 12 - xlen - 8);
        zs.next_out = out.data() + at;
        zs.avail_out = isize;
        if (isize && (::inflate(&zs, Z_FINISH) != Z_STREAM_END || zs.avail_out != 0)) {
            err = "BGZF inflate failed";
            inflateEnd(&zs);
            return false;
        }
        off += (int64_t)bsize;
        if (block_end) block_end->push_back({out.size(), off});
        memmove(comp.data(), comp.data() + bsize, clen - bsize);
        clen -= bsize;
        if (clen == 0 && eof) break;
    }
    inflateEnd(&zs);
    return true;
}

inline uint32_t rd_u32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// The structural invariants of a record at d[o] (SAMv1 §4.2; loose on purpose: any refID,
// pos and name bytes, as the decoders accept): block_size >= 32 and below 2^28, a
// NUL-terminated read name, the variable fields inside block_size. Returns the record's
// length, 0 when invalid, or SIZE_MAX when d ends inside the fixed fields.
size_t record_ok(const uint8_t* d, size_t n, size_t o) {
    if (o + 4 + 32 > n) return SIZE_MAX;
    const uint32_t bs = rd_u32(d + o);
    if (bs < 32 || bs >= (1u << 28)) return 0;
    const uint8_t* b = d + o + 4;
    const uint32_t l_name = b[8], n_cig = b[12] | (b[13] << 8), l_seq = rd_u32(b + 16);
    if (l_name < 1 || (l_seq >> 31)) return 0;
    if ((uint64_t)32 + l_name + 4ull * n_cig + (l_seq + 1ull) / 2 + l_seq > bs) return 0;
    if (o + 4 + 32 + l_name <= n && b[32 + l_name - 1] != 0) return 0;
    return 4 + (size_t)bs;
}

// The first offset in d from which `chain` consecutive records validate (or all records
// up to the end of d, at least one of them complete); SIZE_MAX when none in [0, max_o).
size_t first_record(const uint8_t* d, size_t n, size_t max_o, int chain, bool eof) {
    if (n == 0) return eof ? 0 : SIZE_MAX;  // only empty blocks (the EOF marker) from here
    for (size_t o = 0; o < max_o && o < n; ++o) {
        size_t q = o;
        int ok = 0;
        bool good = true;
        while (ok < chain) {
            if (q == n && eof) break;  // the records end with the file
            const size_t len = record_ok(d, n, q);
            if (len == 0) {
                good = false;
                break;
            }
            if (len == SIZE_MAX || q + len > n) break;  // d ends inside this record
            q += len;
            ++ok;
        }
        if (good && ok >= 1) return o;
        if (good && ok == 0 && o == n) return o;
    }
    return SIZE_MAX;
}

}  // namespace
}  // namespace rogtk

using namespace rogtk;

extern "C" {

int rogtk_bam_split_points(const char* path, int n, int64_t* points, int* n_ranges) {
    ROGTK_REQUIRE(path && points && n_ranges && n >= 1, ROGTK_E_INVALID, "bam split: bad arguments");
    FILE* f = fopen(path, "rb");
    ROGTK_REQUIRE(f, ROGTK_E_INVALID, "Failed to open BAM file '%s'", path);
    std::unique_ptr<FILE, int (*)(FILE*)> guard(f, fclose);
    fseeko(f, 0, SEEK_END);
    const int64_t size = (int64_t)ftello(f);
    // the block holding the first record byte: no split point at or before it
    std::vector<uint8_t> d;
    std::vector<std::pair<size_t, int64_t>> ends;
    std::string err;
    size_t hlen = 0;
    int64_t c_rec = 0;
    for (size_t want = 1 << 16;; want *= 4) {
        ROGTK_REQUIRE(inflate_from(f, 0, want, d, err, &ends), ROGTK_E_INVALID, "BAM %s: %s", path, err.c_str());
        ROGTK_REQUIRE(d.size() >= 8 && memcmp(d.data(), "BAM\1", 4) == 0, ROGTK_E_INVALID, "not a BAM file (bad magic)");
        size_t o = 8 + (size_t)rd_u32(d.data() + 4);
        bool done = o + 4 <= d.size();
        if (done) {
            const uint32_t nref = rd_u32(d.data() + o);
            o += 4;
            for (uint32_t i = 0; i < nref && done; ++i) {
                if (o + 4 > d.size()) done = false;
                else o += 8 + (size_t)rd_u32(d.data() + o);
            }
            done = done && o <= d.size();
        }
        if (done) {
            hlen = o;
            break;
        }
        ROGTK_REQUIRE(d.size() >= want, ROGTK_E_INVALID, "BAM header: unexpected end of file");
    }
    for (const auto& e : ends)
        if (e.first > hlen) break;
        else c_rec = e.second;  // the first record byte lies in the block from here (or later)
    int k = 0;
    points[k++] = 0;
    std::vector<uint8_t> win(1 << 18);
    for (int i = 1; i < n; ++i) {
        const int64_t target = size * i / n;
        if (target <= std::max(c_rec, points[k - 1])) continue;
        fseeko(f, (off_t)target, SEEK_SET);
        const size_t got = fread(win.data(), 1, win.size(), f);
        int64_t found = -1;
        for (size_t j = 0; j + 18 <= got && found < 0; ++j) {
            const size_t bs = bgzf_block_at(win.data() + j, got - j);
            if (!bs) continue;
            const int64_t at = target + (int64_t)j;
            const bool next_ok = at + (int64_t)bs == size ||
                                 (j + bs + 18 <= got && bgzf_block_at(win.data() + j + bs, got - j - bs) != 0);
            if (next_ok) found = at;
        }
        // no split inside the EOF marker block (28 bytes) or after it
        if (found > points[k - 1] && found > c_rec && found + 28 < size) points[k++] = found;
    }
    points[k] = size;
    *n_ranges = k;
    return ROGTK_OK;
}

int rogtk_bam_find_record(const char* path, int64_t c_begin, int64_t* skip) {
    ROGTK_REQUIRE(path && skip && c_begin >= 0, ROGTK_E_INVALID, "bam find_record: bad arguments");
    FILE* f = fopen(path, "rb");
    ROGTK_REQUIRE(f, ROGTK_E_INVALID, "Failed to open BAM file '%s'", path);
    std::unique_ptr<FILE, int (*)(FILE*)> guard(f, fclose);
    std::vector<uint8_t> d;
    std::string err;
    // a straddling record is < 2^28 bytes; records this long are not expected in practice,
    // so 4 MB of stream covers the skip and a chain of records after it
    ROGTK_REQUIRE(inflate_from(f, c_begin, 4u << 20, d, err), ROGTK_E_INVALID, "BAM %s: %s", path, err.c_str());
    const bool eof = d.size() < (4u << 20);
    const size_t o = first_record(d.data(), d.size(), d.size() + 1, 16, eof);
    ROGTK_REQUIRE(o != SIZE_MAX, ROGTK_E_INVALID, "BAM %s: no record start found after offset %lld", path,
                  (long long)c_begin);
    *skip = (int64_t)o;
    return ROGTK_OK;
}

int rogtk_bam_open(const char* path, int n_threads, void** reader) {
    return rogtk_bam_open_range(path, n_threads, 0, -1, 0, reader);
}

int rogtk_bam_open_range(const char* path, int n_threads, int64_t c_begin, int64_t c_end, int64_t skip,
                         void** reader) {
    ROGTK_REQUIRE(path && reader, ROGTK_E_INVALID, "bam: NULL argument");
    ROGTK_REQUIRE(c_begin >= 0 && skip >= 0 && (c_end < 0 || c_end > c_begin), ROGTK_E_INVALID,
                  "bam range: bad range [%lld, %lld) / skip %lld", (long long)c_begin, (long long)c_end,
                  (long long)skip);
    *reader = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_error("no HIP device available (librogtk_hip needs an MI355X / gfx950 GPU)");
        return ROGTK_E_NODEVICE;
    }
    std::unique_ptr<BamReader> R(new BamReader());
    R->z.f = fopen(path, "rb");
    ROGTK_REQUIRE(R->z.f, ROGTK_E_INVALID, "Failed to open BAM file '%s'", path);
    std::call_once(g_pin_warm_once, [] {
        size_t hint;
        {
            std::lock_guard<std::mutex> lk(g_pin_mu);
            hint = std::max(g_pin_hint, kPinWarmBytes);
        }
        pin_warm(kPinWarm, hint);
    });
    pin_take(R->z.buf);
    R->z.threads = n_threads > 0 ? n_threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    ROGTK_HIP_CHECK(hipGetDevice(&R->device));
    ROGTK_HIP_CHECK(hipStreamCreateWithFlags(&R->stream, hipStreamNonBlocking));
    fseeko(R->z.f, 0, SEEK_END);
    const int64_t fsize = (int64_t)ftello(R->z.f);
    fseeko(R->z.f, 0, SEEK_SET);
    if (c_end >= fsize) c_end = -1;  // the range runs to the end of the file
    const bool ranged = c_begin > 0;
    const bool ra = R->z.readahead;
    const size_t chunk = R->z.chunk;
    if (ranged) {  // the header only: no read-ahead into other ranges' bytes
        R->z.readahead = false;
        R->z.chunk = 1u << 20;
    } else {
        R->z.c_end = c_end;
    }
    int rc = read_header(R.get());
    if (rc != ROGTK_OK) return rc;
    if (ranged) {  // restart the stream at the range's first block
        Bgzf& z = R->z;
        z.stop_ahead();
        z.readahead = ra;
        z.chunk = chunk;
        ROGTK_REQUIRE(fseeko(z.f, (off_t)c_begin, SEEK_SET) == 0, ROGTK_E_INVALID, "bam range: seek failed");
        z.comp_len = 0;
        z.file_eof = false;
        z.file_off = c_begin;
        z.pos = z.end = 0;
        z.u_base = 0;
        z.c_end = c_end;
        ROGTK_REQUIRE(skip == 0 || z.ensure_rel(0, (size_t)skip), ROGTK_E_INVALID, "bam range: %s",
                      z.err.empty() ? "skip past the end of the file" : z.err.c_str());
        z.pos += (size_t)skip;
    }
    for (size_t i = 0; i + 1 < R->ref_off.size(); ++i)
        R->max_ref_len = std::max<int32_t>(R->max_ref_len, (int32_t)(R->ref_off[i + 1] - R->ref_off[i]));
    const size_t rb = R->ref_off.size() * 8, vb = std::max<size_t>(R->ref_val.size(), 1);
    if (R->d_ref_off.ensure(rb) != ROGTK_OK || R->d_ref_val.ensure(vb) != ROGTK_OK) return ROGTK_E_HIP;
    ROGTK_HIP_CHECK(hipMemcpy(R->d_ref_off.p, R->ref_off.data(), rb, hipMemcpyHostToDevice));
    if (!R->ref_val.empty())
        ROGTK_HIP_CHECK(hipMemcpy(R->d_ref_val.p, R->ref_val.data(), R->ref_val.size(), hipMemcpyHostToDevice));
    *reader = R.release();
    return ROGTK_OK;
}

int rogtk_bam_header(void* reader, int64_t* n_ref, const int64_t** name_offsets, const uint8_t** name_values,
                     const char** text, int64_t* text_len) {
    ROGTK_REQUIRE(reader, ROGTK_E_INVALID, "bam: NULL reader");
    auto* R = static_cast<BamReader*>(reader);
    if (n_ref) *n_ref = (int64_t)R->ref_off.size() - 1;
    if (name_offsets) *name_offsets = R->ref_off.data();
    if (name_values) *name_values = R->ref_val.data();
    if (text) *text = R->text.c_str();
    if (text_len) *text_len = (int64_t)R->text.size();
    return ROGTK_OK;
}

static int bam_next_common(BamReader* R, int64_t max_records, int mode, int include_sequence, int include_quality,
                           bool sync_totals = true) {
    ROGTK_REQUIRE(max_records > 0, ROGTK_E_INVALID, "bam: max_records must be > 0");
    ROGTK_REQUIRE(mode == ROGTK_BAM_NOODLES || mode == ROGTK_BAM_HTSLIB || mode == ROGTK_BAM_HTSLIB_BLOCKS,
                  ROGTK_E_INVALID, "bam: unknown mode %d", mode);
    ROGTK_HIP_CHECK(hipSetDevice(R->device));
    if (R->copy_pending) {  // the previous batch's H2D copy still reads the stream buffer
        ROGTK_HIP_CHECK(hipEventSynchronize(R->copied));
        R->copy_pending = false;
    }
    // release the previous batch's bytes
    R->z.pos += R->n ? (size_t)R->roff[R->n] : 0;
    R->n = 0;
    const double t0 = now_s();
    const double in0 = R->z.t_read + R->z.t_inflate + R->z.t_move;
    int rc = frame_batch(R, max_records);
    const double t1 = now_s();
    R->t_frame += (t1 - t0) - (R->z.t_read + R->z.t_inflate + R->z.t_move - in0);
    if (rc != ROGTK_OK) return rc;
    rc = decode_batch(R, mode, include_sequence, include_quality, sync_totals);
    R->t_decode += now_s() - t1;
    return rc;
}

int rogtk_bam_next(void* reader, int64_t max_records, int mode, int include_sequence, int include_quality,
                   int64_t* n_records, rogtk_bam_batch* out) {
    ROGTK_REQUIRE(reader && n_records && out, ROGTK_E_INVALID, "bam: NULL argument");
    auto* R = static_cast<BamReader*>(reader);
    *n_records = 0;
    int rc = bam_next_common(R, max_records, mode, include_sequence, include_quality);
    if (rc != ROGTK_OK) return rc;
    const int64_t n = R->n;
    hipStream_t s = R->stream;
    memset(out, 0, sizeof *out);
    const int64_t words = (n + 63) / 64;
    const double td = now_s();
    for (int c = 0; c < 4; ++c) {
        if ((c == 2 && !include_sequence) || (c == 3 && !include_quality)) continue;
        int64_t tot = 0;
        ROGTK_HIP_CHECK(hipMemcpyAsync(&tot, R->d_off[c].as<int64_t>() + n, 8, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipStreamSynchronize(s));
        if (R->h_off[c].ensure((size_t)(n + 1) * 8) != ROGTK_OK ||
            R->h_val[c].ensure((size_t)std::max<int64_t>(tot, 1)) != ROGTK_OK)
            return ROGTK_E_HIP;
        ROGTK_HIP_CHECK(hipMemcpyAsync(R->h_off[c].p, R->d_off[c].p, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, s));
        if (tot) ROGTK_HIP_CHECK(hipMemcpyAsync(R->h_val[c].p, R->d_val[c].p, (size_t)tot, hipMemcpyDeviceToHost, s));
        out->offsets[c] = (const int64_t*)R->h_off[c].p;
        out->values[c] = R->h_val[c].p;
    }
    // validity: chrom, start, end, sequence, quality_scores
    for (int c = 0; c < 5; ++c) {
        if ((c == 3 && !include_sequence) || (c == 4 && !include_quality)) continue;
        if (R->h_valid[c].ensure((size_t)std::max<int64_t>(words, 1) * 8) != ROGTK_OK) return ROGTK_E_HIP;
        if (words)
            ROGTK_HIP_CHECK(hipMemcpyAsync(R->h_valid[c].p, R->d_valid[c].p, (size_t)words * 8, hipMemcpyDeviceToHost, s));
    }
    out->validity[1] = R->h_valid[0].p;
    out->validity[2] = include_sequence ? R->h_valid[3].p : nullptr;
    out->validity[3] = include_quality ? R->h_valid[4].p : nullptr;
    DevBuf* u[3] = {&R->d_start, &R->d_end, &R->d_flags};
    for (int c = 0; c < 3; ++c) {
        if (R->h_u32[c].ensure((size_t)std::max<int64_t>(n, 1) * 4) != ROGTK_OK) return ROGTK_E_HIP;
        if (n) ROGTK_HIP_CHECK(hipMemcpyAsync(R->h_u32[c].p, u[c]->p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        out->u32[c] = (const uint32_t*)R->h_u32[c].p;
    }
    out->u32_validity[0] = R->h_valid[1].p;
    out->u32_validity[1] = R->h_valid[2].p;
    out->u32_validity[2] = nullptr;
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    R->t_d2h += now_s() - td;
    *n_records = n;
    return ROGTK_OK;
}

int rogtk_bam_next_dev(void* reader, int64_t max_records, int mode, int include_sequence, int include_quality,
                       int64_t* n_records, rogtk_bam_batch* out, void* stream) {
    ROGTK_REQUIRE(reader && n_records && out, ROGTK_E_INVALID, "bam: NULL argument");
    auto* R = static_cast<BamReader*>(reader);
    *n_records = 0;
    // the batch is decoded on the caller's stream (ordered with what the caller does next)
    hipStream_t own = R->stream;
    if (stream) R->stream = reinterpret_cast<hipStream_t>(stream);
    // no host sync inside a file: value buffers sized from host bounds, d_bad checked by
    // rogtk_bam_check (a NULL stream keeps the synchronous behaviour)
    int rc = bam_next_common(R, max_records, mode, include_sequence, include_quality, stream == nullptr);
    // NULL: the batch is complete on return (the reader's own stream is non-blocking, so
    // nothing the caller enqueues afterwards, e.g. on the null stream, is ordered after its
    // fill kernel: a UMI append on the null stream read half-filled sequences)
    if (rc == ROGTK_OK && !stream) rc = hipStreamSynchronize(own) == hipSuccess ? ROGTK_OK : ROGTK_E_HIP;
    R->stream = own;
    if (rc != ROGTK_OK) return rc;
    memset(out, 0, sizeof *out);
    for (int c = 0; c < 4; ++c) {
        out->offsets[c] = R->d_off[c].as<int64_t>();
        out->values[c] = R->d_val[c].as<uint8_t>();
    }
    out->validity[1] = R->d_valid[0].as<uint8_t>();
    out->validity[2] = R->d_valid[3].as<uint8_t>();
    out->validity[3] = R->d_valid[4].as<uint8_t>();
    out->u32[0] = R->d_start.as<uint32_t>();
    out->u32[1] = R->d_end.as<uint32_t>();
    out->u32[2] = R->d_flags.as<uint32_t>();
    out->u32_validity[0] = R->d_valid[1].as<uint8_t>();
    out->u32_validity[1] = R->d_valid[2].as<uint8_t>();
    *n_records = R->n;
    return ROGTK_OK;
}

int rogtk_bam_umi_dev(const rogtk_bam_batch* batch, int64_t n, int source, int umi_len, int sep, int64_t* offsets,
                      uint8_t* values, int64_t values_cap, uint8_t* validity, void* stream) {
    ROGTK_REQUIRE(batch && offsets && values && validity, ROGTK_E_INVALID, "bam umi: NULL argument");
    ROGTK_REQUIRE(source == 0 || source == 1, ROGTK_E_INVALID, "bam umi: source must be 0 (sequence) or 1 (name)");
    ROGTK_REQUIRE(source == 1 || umi_len > 0, ROGTK_E_INVALID, "bam umi: umi_len must be > 0");
    ROGTK_REQUIRE(source == 1 || batch->offsets[2], ROGTK_E_INVALID, "bam umi: the batch has no sequence column");
    ROGTK_REQUIRE(n >= 0, ROGTK_E_INVALID, "bam umi: n must be >= 0");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    thread_local DevBuf len, start, cub;
    if (len.ensure((size_t)(n + 1) * 8) != ROGTK_OK || start.ensure((size_t)(n + 1) * 8) != ROGTK_OK)
        return ROGTK_E_HIP;
    if (n > 0) {
        hipLaunchKernelGGL(k_umi_len, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, batch->offsets[2],
                           (const uint64_t*)batch->validity[2], batch->offsets[0], batch->values[0], n, source,
                           umi_len, sep, len.as<int64_t>(), start.as<int64_t>(), (uint64_t*)validity);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    ROGTK_HIP_CHECK(hipMemsetAsync(len.as<int64_t>() + n, 0, 8, s));
    size_t tb = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, len.as<int64_t>(), offsets, (int)(n + 1), s));
    if (cub.ensure(tb) != ROGTK_OK) return ROGTK_E_HIP;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(cub.p, tb, len.as<int64_t>(), offsets, (int)(n + 1), s));
    int64_t total = 0;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&total, offsets + n, 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));  // (rogtk_bam_umi_append: no sync)
    ROGTK_REQUIRE(total <= values_cap, ROGTK_E_OVERFLOW, "bam umi: %lld bytes exceed values_cap %lld",
                  (long long)total, (long long)values_cap);
    if (n > 0) {
        const uint8_t* src = source == 0 ? batch->values[2] : batch->values[0];
        hipLaunchKernelGGL(k_umi_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, start.as<int64_t>(),
                           offsets, n, values);
        ROGTK_HIP_CHECK(hipGetLastError());
    }
    return ROGTK_OK;
}

int rogtk_bam_umi_append(const rogtk_bam_batch* batch, int64_t n, int source, int umi_len, int sep,
                         int64_t* offsets, uint8_t* values, int64_t values_cap, uint8_t* validity, int64_t row_base,
                         int64_t* base, unsigned long long* overflow, void* stream) {
    ROGTK_REQUIRE(batch && offsets && values && validity && base && overflow, ROGTK_E_INVALID,
                  "bam umi append: NULL argument");
    ROGTK_REQUIRE(source == 0 || source == 1, ROGTK_E_INVALID, "bam umi: source must be 0 (sequence) or 1 (name)");
    ROGTK_REQUIRE(source == 1 || umi_len > 0, ROGTK_E_INVALID, "bam umi: umi_len must be > 0");
    ROGTK_REQUIRE(source == 1 || batch->offsets[2], ROGTK_E_INVALID, "bam umi: the batch has no sequence column");
    ROGTK_REQUIRE(n >= 0 && row_base >= 0, ROGTK_E_INVALID, "bam umi append: n and row_base must be >= 0");
    if (n == 0) return ROGTK_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    thread_local DevBuf len, start, cub;
    if (len.ensure((size_t)(n + 1) * 8) != ROGTK_OK || start.ensure((size_t)(n + 1) * 8) != ROGTK_OK)
        return ROGTK_E_HIP;
    int64_t* off = offsets + row_base;
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_umi_len, dim3(g), dim3(256), 0, s, batch->offsets[2], (const uint64_t*)batch->validity[2],
                       batch->offsets[0], batch->values[0], n, source, umi_len, sep, len.as<int64_t>(),
                       start.as<int64_t>(), (uint64_t*)validity, row_base);
    ROGTK_HIP_CHECK(hipGetLastError());
    ROGTK_HIP_CHECK(hipMemsetAsync(len.as<int64_t>() + n, 0, 8, s));
    size_t tb = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, len.as<int64_t>(), off, (int)(n + 1), s));
    if (cub.ensure(tb) != ROGTK_OK) return ROGTK_E_HIP;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(cub.p, tb, len.as<int64_t>(), off, (int)(n + 1), s));
    hipLaunchKernelGGL(k_add_base, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, s, off, n + 1,
                       (const int64_t*)base);
    hipLaunchKernelGGL(k_set_base, dim3(1), dim3(64), 0, s, (const int64_t*)(off + n), base);
    const uint8_t* src = source == 0 ? batch->values[2] : batch->values[0];
    hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, s, src, start.as<int64_t>(),
                       (const int64_t*)off, n, values_cap, values, overflow);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

int rogtk_bam_append_strings(const int64_t* src_offsets, const uint8_t* src_values, int64_t n, int64_t* offsets,
                             uint8_t* values, int64_t values_cap, int64_t row_base, int64_t* base,
                             unsigned long long* overflow, void* stream) {
    ROGTK_REQUIRE(src_offsets && src_values && offsets && values && base && overflow && n >= 0 && row_base >= 0,
                  ROGTK_E_INVALID, "bam append strings: bad arguments");
    if (n == 0) return ROGTK_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int64_t* off = offsets + row_base;
    ROGTK_HIP_CHECK(hipMemcpyAsync(off, src_offsets, (size_t)(n + 1) * 8, hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_add_base, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, s, off, n + 1,
                       (const int64_t*)base);
    hipLaunchKernelGGL(k_set_base, dim3(1), dim3(64), 0, s, (const int64_t*)(off + n), base);
    hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, s, src_values, src_offsets,
                       (const int64_t*)off, n, values_cap, values, overflow);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

namespace {
// dst bits [row_base, row_base + n) = src bits [0, n) (dst zeroed before; a part's first word
// may hold the previous part's last bits: ORed, the rest stored whole)
__global__ __launch_bounds__(256) void k_bits_append(const uint64_t* __restrict__ src, int64_t n, uint64_t* dst,
                                                     int64_t row_base) {
    const int64_t w0 = row_base >> 6, w1 = (row_base + n - 1) >> 6;
    const int64_t w = w0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n <= 0 || w > w1) return;
    const int64_t lo = max<int64_t>(64 * w, row_base), hi = min<int64_t>(64 * w + 64, row_base + n);
    const int64_t s0 = lo - row_base;  // first source bit
    const int len = (int)(hi - lo);
    const int sh = (int)(s0 & 63);
    uint64_t v = src[s0 >> 6] >> sh;
    if (sh && sh + len > 64) v |= src[(s0 >> 6) + 1] << (64 - sh);
    if (len < 64) v &= (1ull << len) - 1ull;
    v <<= (int)(lo - 64 * w);
    if (w == w0) atomicOr((unsigned long long*)(dst + w), (unsigned long long)v);
    else dst[w] = v;
}
}  // namespace

// Round 6: k device string columns (int64 offsets from 0, values, validity bits) into one,
// in order, with the library's own kernels (rogtk_amd.bam's range concatenation: torch's
// cat / bit kernels cost their first call ~0.5 s of module loading in a fresh process)
int rogtk_concat_strings_dev(int k, const int64_t* const* offsets, const uint8_t* const* values,
                             const uint64_t* const* validity, const int64_t* counts, int64_t* out_offsets,
                             uint8_t* out_values, int64_t values_cap, uint64_t* out_validity, int64_t* base,
                             unsigned long long* overflow, void* stream) {
    ROGTK_REQUIRE(k >= 0 && (k == 0 || (offsets && values && validity && counts)) && out_offsets && out_values &&
                      out_validity && base && overflow,
                  ROGTK_E_INVALID, "concat strings: bad arguments");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int64_t n = 0;
    for (int i = 0; i < k; ++i) n += counts[i];
    ROGTK_HIP_CHECK(hipMemsetAsync(out_validity, 0, (size_t)std::max<int64_t>((n + 63) / 64, 1) * 8, s));
    ROGTK_HIP_CHECK(hipMemsetAsync(base, 0, 8, s));
    ROGTK_HIP_CHECK(hipMemsetAsync(overflow, 0, 8, s));
    ROGTK_HIP_CHECK(hipMemsetAsync(out_offsets, 0, 8, s));
    int64_t row = 0;
    for (int i = 0; i < k; ++i) {
        if (counts[i] == 0) continue;
        if (int rc = rogtk_bam_append_strings(offsets[i], values[i], counts[i], out_offsets, out_values, values_cap,
                                              row, base, overflow, stream))
            return rc;
        const int64_t words = ((row + counts[i] - 1) >> 6) - (row >> 6) + 1;
        hipLaunchKernelGGL(k_bits_append, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, validity[i], counts[i],
                           out_validity, row);
        ROGTK_HIP_CHECK(hipGetLastError());
        row += counts[i];
    }
    return ROGTK_OK;
}

int rogtk_bam_batch_bytes(void* reader, int64_t* bytes) {
    ROGTK_REQUIRE(reader && bytes, ROGTK_E_INVALID, "bam: NULL argument");
    auto* R = static_cast<BamReader*>(reader);
    *bytes = R->n ? R->roff[R->n] : 0;
    return ROGTK_OK;
}

int rogtk_bam_check(void* reader, void* stream) {
    ROGTK_REQUIRE(reader, ROGTK_E_INVALID, "bam: NULL reader");
    auto* R = static_cast<BamReader*>(reader);
    if (!R->bad_cleared) return ROGTK_OK;  // no device-mode batch, or every batch checked
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : R->stream;
    unsigned long long bad = 0;
    ROGTK_HIP_CHECK(hipMemcpyAsync(&bad, R->d_bad.p, 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    ROGTK_REQUIRE(bad == 0, ROGTK_E_INVALID, "BAM: %llu record(s) whose fields overrun their block_size", bad);
    return ROGTK_OK;
}

int rogtk_copy(void* dst, const void* src, int64_t bytes, void* stream) {
    ROGTK_REQUIRE(bytes >= 0 && (bytes == 0 || (dst && src)), ROGTK_E_INVALID, "copy: bad arguments");
    if (bytes == 0) return ROGTK_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    ROGTK_HIP_CHECK(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    return ROGTK_OK;
}

int rogtk_bam_range_tail(void* reader, int64_t* tail) {
    ROGTK_REQUIRE(reader && tail, ROGTK_E_INVALID, "bam: NULL argument");
    *tail = static_cast<BamReader*>(reader)->tail;
    return ROGTK_OK;
}

int rogtk_bam_timers(void* reader, double* out6) {
    ROGTK_REQUIRE(reader && out6, ROGTK_E_INVALID, "bam: NULL argument");
    auto* R = static_cast<BamReader*>(reader);
    const double t[6] = {R->z.t_read, R->z.t_move - R->z.t_read, R->z.t_inflate, R->t_frame, R->t_decode, R->t_d2h};
    memcpy(out6, t, sizeof t);
    return ROGTK_OK;
}

int rogtk_bam_close(void* reader) {
    if (!reader) return ROGTK_OK;
    auto* R = static_cast<BamReader*>(reader);
    if (R->stream) (void)hipStreamSynchronize(R->stream);
    delete R;
    return ROGTK_OK;
}

}  // extern "C"
