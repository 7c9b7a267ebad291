// strings.hip — element-wise DNA / CIGAR / PHRED string transforms on gfx950
// (the remaining per-row string expressions of rogtk).
//
//   op                         reference (src/expressions.rs)
//   ROGTK_STR_REVCOMP          reverse_complement_series / _to_output   :957-977
//   ROGTK_STR_PARSE_CIGAR      parse_cigar_series / parse_cigar_str     :450-505
//   ROGTK_STR_ALIGNED_REF      cigar_aligned_ref_expr + expand_cigar_   :257-394
//   ROGTK_STR_ALIGNED_QUERY    cigar_aligned_query_expr   alignment     :257-336,396-444
//   ROGTK_STR_CIGAR_INSERTIONS extract_cigar_insertions_expr            :29-80,207-251
//   ROGTK_STR_ENRICH_ALLELE    enrich_allele_insertions_expr            :84-205
//   ROGTK_STR_PHRED_STR        phred_to_numeric_series_str / split_string :632-665
//   ROGTK_STR_PHRED_LIST       phred_to_numeric_series (List[u8] values) :598-630
//
// Every op is ONE device function run twice over the rows (thread per row): a
// measuring pass that only counts output bytes, then, after an exclusive scan of
// the counts, a filling pass that writes them at the row's offset. The emitter is
// the only difference between the passes, so the two can never disagree.
// Arithmetic follows the reference's release build (Cargo.toml [profile.release]:
// no overflow checks): usize sums wrap, `u8 - base` wraps.
#include <hipcub/hipcub.hpp>

#include <cstdlib>
#include <memory>
#include <vector>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

constexpr int kBlock = 256;

struct Col {
    const void* off;
    int ow;
    const uint8_t* val;
    const uint8_t* valid;
    int64_t voff;
    int bcast;  // row 0 for every row (a length-1 column broadcast)
};

struct Cols {
    Col c[3];
};

__device__ __forceinline__ int64_t col_off(const Col& c, int64_t i) {
    return c.ow == 4 ? (int64_t)((const int32_t*)c.off)[i] : ((const int64_t*)c.off)[i];
}
__device__ __forceinline__ bool col_valid(const Col& c, int64_t i) {
    if (c.bcast) i = 0;
    if (!c.valid) return true;
    const int64_t b = c.voff + i;
    return (c.valid[b >> 3] >> (b & 7)) & 1;
}

struct Str {
    const uint8_t* p;
    uint64_t n;
};
__device__ __forceinline__ Str col_str(const Col& c, int64_t i) {
    if (c.bcast) i = 0;
    const int64_t a = col_off(c, i), b = col_off(c, i + 1);
    return Str{c.val + a, (uint64_t)(b - a)};
}

// Counting (FILL = false) or writing (FILL = true) output bytes.
template <bool FILL>
struct Emit {
    uint8_t* p;
    uint64_t n = 0;
    __device__ __forceinline__ void put(uint8_t b) {
        if (FILL) p[n] = b;
        ++n;
    }
    __device__ __forceinline__ void fill(uint8_t b, uint64_t k) {
        if (FILL)
            for (uint64_t j = 0; j < k; ++j) p[n + j] = b;
        n += k;
    }
    __device__ __forceinline__ void bytes(const uint8_t* s, uint64_t k) {
        if (FILL)
            for (uint64_t j = 0; j < k; ++j) p[n + j] = s[j];
        n += k;
    }
    // `format!("{}", v)` of a usize / u8
    __device__ __forceinline__ void dec(uint64_t v) {
        uint8_t t[20];
        int k = 0;
        do {
            t[k++] = (uint8_t)('0' + v % 10);
            v /= 10;
        } while (v);
        while (k) put(t[--k]);
    }
    // `String::push((b as char).to_ascii_{upper,lower}case())`: a byte >= 0x80 is the
    // Latin-1 char U+00XX, two bytes of UTF-8 in the output
    __device__ __forceinline__ void latin1(uint8_t b, bool upper) {
        if (b < 0x80) {
            if (upper && b >= 'a' && b <= 'z') b -= 32;
            if (!upper && b >= 'A' && b <= 'Z') b += 32;
            put(b);
        } else {
            put((uint8_t)(0xC0 | (b >> 6)));
            put((uint8_t)(0x80 | (b & 0x3F)));
        }
    }
    // String::from_utf8_lossy of s[a, a + k) where s is valid UTF-8: continuation bytes
    // cut off from their lead are one U+FFFD each; a sequence cut at the end is one
    __device__ void lossy(const uint8_t* s, uint64_t k) {
        uint64_t j = 0;
        while (j < k && (s[j] & 0xC0) == 0x80) {
            put(0xEF), put(0xBF), put(0xBD);
            ++j;
        }
        while (j < k) {
            const uint8_t b = s[j];
            const uint64_t w = b < 0x80 ? 1 : b < 0xE0 ? 2 : b < 0xF0 ? 3 : 4;
            if (j + w > k) {
                put(0xEF), put(0xBF), put(0xBD);
                return;
            }
            bytes(s + j, w);
            j += w;
        }
    }
};

// CIGAR tokenizer of the reference loops: digits accumulate (`is_ascii_digit`), any
// other char ends a token; `num_buf.parse::<usize>()` fails on an empty buffer or
// on overflow, and a failed parse skips the op. Multi-byte chars: their lead byte
// ends the token (an unknown op), their continuation bytes see an empty buffer.
struct CigarTok {
    const uint8_t* s;
    uint64_t n, j = 0;
    __device__ bool next(uint8_t* op, uint64_t* len) {
        uint64_t v = 0;
        bool digits = false, over = false;
        while (j < n) {
            const uint8_t c = s[j++];
            if (c >= '0' && c <= '9') {
                const uint64_t d = c - '0';
                if (v > (~0ull - d) / 10) over = true;
                v = v * 10 + d;
                digits = true;
                continue;
            }
            if (digits && !over) {
                *op = c;
                *len = v;
                return true;
            }
            v = 0;
            digits = over = false;
        }
        return false;
    }
};

// ---------------------------------------------------------------- the ops
template <bool F>
__device__ void op_revcomp(Emit<F>& o, Str s) {
    // dna.chars().rev(): whole UTF-8 chars in reverse order, ASCII A/T/C/G/N mapped
    uint64_t e = s.n;
    while (e > 0) {
        uint64_t b = e - 1;
        while (b > 0 && (s.p[b] & 0xC0) == 0x80) --b;
        if (e - b == 1) {
            uint8_t c = s.p[b];
            c = c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'C' ? 'G' : c == 'G' ? 'C' : c;
            o.put(c);
        } else {
            o.bytes(s.p + b, e - b);
        }
        e = b;
    }
}

template <bool F>
__device__ void op_parse_cigar(Emit<F>& o, Str cig, bool block_dels) {
    CigarTok t{cig.p, cig.n};
    uint8_t op;
    uint64_t len, ref = 0;
    bool first = true;
    auto sep = [&] {
        if (!first) o.put('|');
        first = false;
    };
    while (t.next(&op, &len)) {
        if (op == 'D') {
            if (block_dels) {
                sep();
                o.put('D'), o.put(','), o.dec(ref), o.put(','), o.dec(len);
            } else {
                const uint64_t end = ref + len;  // wrapping, as the release build
                for (uint64_t p = ref; p < end; ++p) {
                    sep();
                    o.put('D'), o.put(','), o.dec(p), o.put(','), o.put('1');
                }
            }
            ref += len;
        } else if (op == 'I') {
            sep();
            o.put('I'), o.put(','), o.dec(ref), o.put(','), o.dec(len);
        } else {
            ref += len;
        }
    }
}

// expand_cigar_alignment: side 0 = aligned reference, 1 = aligned query
template <bool F>
__device__ void op_aligned(Emit<F>& o, Str ref, Str qry, Str cig, int side) {
    CigarTok t{cig.p, cig.n};
    uint8_t op;
    uint64_t len, rp = 0, qp = 0;
    while (t.next(&op, &len)) {
        const uint64_t rk = min(len, ref.n - rp), qk = min(len, qry.n - qp);
        switch (op) {
            case 'M':
            case '=':
            case 'X':
                if (side == 0)
                    for (uint64_t j = 0; j < rk; ++j) o.latin1(ref.p[rp + j], true);
                else
                    for (uint64_t j = 0; j < qk; ++j) o.latin1(qry.p[qp + j], true);
                rp += rk;
                qp += qk;
                break;
            case 'I':
                if (side == 0)
                    o.fill('-', len);
                else
                    for (uint64_t j = 0; j < qk; ++j) o.latin1(qry.p[qp + j], true);
                qp += qk;
                break;
            case 'D':
            case 'N':
                if (side == 0)
                    for (uint64_t j = 0; j < rk; ++j) o.latin1(ref.p[rp + j], true);
                else
                    o.fill('-', len);
                rp += rk;
                break;
            case 'S':
                if (side == 0)
                    o.fill('-', len);
                else
                    for (uint64_t j = 0; j < qk; ++j) o.latin1(qry.p[qp + j], false);
                qp += qk;
                break;
            default:  // 'H', 'P', unknown
                break;
        }
    }
}

// extract_insertions_from_cigar: calls fn(ref_pos, seq_pos, len) for every insertion
// the reference inserts into its HashMap (in walk order; later ones overwrite)
template <class Fn>
__device__ void walk_insertions(Str seq, Str cig, Fn&& fn) {
    CigarTok t{cig.p, cig.n};
    uint8_t op;
    uint64_t len, sp = 0, rp = 0;
    while (t.next(&op, &len)) {
        switch (op) {
            case 'M':
            case '=':
            case 'X':
                sp += len;
                rp += len;
                break;
            case 'I':
                if (sp + len <= seq.n) fn(rp, sp, len);
                sp += len;
                break;
            case 'D':
            case 'N':
                rp += len;
                break;
            case 'S':
                sp += len;
                break;
            default:
                break;
        }
    }
}

template <bool F>
__device__ void op_insertions(Emit<F>& o, Str seq, Str cig) {
    // map keys ascend in walk order (ref_pos never decreases), so sorting the map is
    // the walk order with each run of equal keys reduced to its last insertion
    bool have = false, first = true;
    uint64_t pr = 0, ps = 0, pl = 0;
    auto flush = [&] {
        if (!first) o.put('|');
        first = false;
        o.dec(pr);
        o.put(':');
        o.lossy(seq.p + ps, pl);
    };
    walk_insertions(seq, cig, [&](uint64_t r, uint64_t s, uint64_t l) {
        if (have && r != pr) flush();
        have = true;
        pr = r, ps = s, pl = l;
    });
    if (have) flush();
}

// `str::parse::<usize>()`: optional '+', then >= 1 ASCII digits, no overflow
__device__ bool parse_usize(const uint8_t* s, uint64_t n, uint64_t* v) {
    uint64_t j = 0;
    if (n > 0 && s[0] == '+') j = 1;
    if (j == n) return false;
    uint64_t x = 0;
    for (; j < n; ++j) {
        const uint8_t c = s[j];
        if (c < '0' || c > '9') return false;
        const uint64_t d = c - '0';
        if (x > (~0ull - d) / 10) return false;
        x = x * 10 + d;
    }
    *v = x;
    return true;
}

// the last insertion at ref_pos key (HashMap::get after all inserts)
__device__ bool find_insertion(Str seq, Str cig, uint64_t key, uint64_t* s_out, uint64_t* l_out) {
    bool hit = false;
    walk_insertions(seq, cig, [&](uint64_t r, uint64_t s, uint64_t l) {
        if (r == key) {
            hit = true;
            *s_out = s;
            *l_out = l;
        }
    });
    return hit;
}

template <bool F>
__device__ void op_enrich(Emit<F>& o, Str al, Str seq, Str cig, bool have_ins) {
    if (!have_ins) {  // seq or CIGAR null: the allele as is
        o.bytes(al.p, al.n);
        return;
    }
    uint64_t j = 0;
    while (j < al.n) {
        const uint8_t c = al.p[j];
        if (c != '[') {
            o.put(c);
            ++j;
            continue;
        }
        uint64_t k = j + 1;
        while (k < al.n && al.p[k] != ']') ++k;
        const uint8_t* ct = al.p + j + 1;
        const uint64_t cn = k - j - 1;
        o.put('[');
        o.bytes(ct, cn);
        if (k == al.n) return;  // no closing bracket: '[' + the rest
        // "pos:...I" -> the insertion at pos - 1 (or pos): append ":SEQ"
        uint64_t colon = 0;
        while (colon < cn && ct[colon] != ':') ++colon;
        // split_once(':') -> (pos_str, rest); rest.ends_with('I') needs a non-empty rest
        uint64_t pos;
        if (colon + 1 < cn && ct[cn - 1] == 'I' && parse_usize(ct, colon, &pos)) {
            uint64_t s = 0, l = 0;
            const bool hit =
                (pos > 0 && find_insertion(seq, cig, pos - 1, &s, &l)) || find_insertion(seq, cig, pos, &s, &l);
            if (hit) {
                o.put(':');
                o.lossy(seq.p + s, l);
            }
        }
        o.put(']');
        j = k + 1;
    }
}

// `phred_char as u8 - base` per char (low 8 bits of the code point, wrapping)
template <bool F>
__device__ void op_phred(Emit<F>& o, Str s, uint8_t base, bool as_text) {
    uint64_t j = 0;
    bool first = true;
    while (j < s.n) {
        const uint8_t b = s.p[j];
        uint32_t cp;
        uint64_t w;
        if (b < 0x80) cp = b, w = 1;
        else if (b < 0xE0) cp = b & 0x1F, w = 2;
        else if (b < 0xF0) cp = b & 0x0F, w = 3;
        else cp = b & 0x07, w = 4;
        for (uint64_t q = 1; q < w && j + q < s.n; ++q) cp = (cp << 6) | (s.p[j + q] & 0x3F);
        j += w;
        const uint8_t v = (uint8_t)((uint8_t)cp - base);
        if (as_text) {
            if (!first) o.put('|');
            o.dec(v);
        } else {
            o.put(v);
        }
        first = false;
    }
}

struct OpArgs {
    int op;
    int64_t n;
    int64_t param;
    Cols cols;
};

// Row i of op: false = null output row.
template <bool F>
__device__ bool run_row(const OpArgs& a, int64_t i, Emit<F>& o) {
    const Col* c = a.cols.c;
    switch (a.op) {
        case ROGTK_STR_REVCOMP:
            if (!col_valid(c[0], i)) return false;
            op_revcomp(o, col_str(c[0], i));
            return true;
        case ROGTK_STR_PARSE_CIGAR:
            if (!col_valid(c[0], i)) return false;
            op_parse_cigar(o, col_str(c[0], i), a.param != 0);
            return true;
        case ROGTK_STR_ALIGNED_REF:
        case ROGTK_STR_ALIGNED_QUERY:
            if (!col_valid(c[0], i) || !col_valid(c[1], i) || !col_valid(c[2], i)) return false;
            op_aligned(o, col_str(c[0], i), col_str(c[1], i), col_str(c[2], i),
                       a.op == ROGTK_STR_ALIGNED_REF ? 0 : 1);
            return true;
        case ROGTK_STR_CIGAR_INSERTIONS:
            if (!col_valid(c[0], i) || !col_valid(c[1], i)) return false;
            op_insertions(o, col_str(c[0], i), col_str(c[1], i));
            return true;
        case ROGTK_STR_ENRICH_ALLELE: {
            if (!col_valid(c[0], i)) return false;
            const bool both = col_valid(c[1], i) && col_valid(c[2], i);
            const Str none{nullptr, 0};
            op_enrich(o, col_str(c[0], i), both ? col_str(c[1], i) : none, both ? col_str(c[2], i) : none, both);
            return true;
        }
        case ROGTK_STR_PHRED_STR:
        case ROGTK_STR_PHRED_LIST:
            if (!col_valid(c[0], i)) return false;
            op_phred(o, col_str(c[0], i), (uint8_t)a.param, a.op == ROGTK_STR_PHRED_STR);
            return true;
        default:
            return false;
    }
}

// lengths[i] = output bytes of row i (0 for null rows); validity bit per row (ballot)
__global__ __launch_bounds__(kBlock) void k_str_measure(OpArgs a, int64_t* __restrict__ lengths,
                                                        uint64_t* __restrict__ valid_bits) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    bool ok = false;
    if (i < a.n) {
        Emit<false> o{nullptr};
        ok = run_row(a, i, o);
        lengths[i] = ok ? (int64_t)o.n : 0;
    }
    const uint64_t m = __ballot(ok);
    if ((threadIdx.x & 63) == 0 && i < a.n) valid_bits[i >> 6] = m;
}

__global__ __launch_bounds__(kBlock) void k_str_fill(OpArgs a, const int64_t* __restrict__ offsets,
                                                     uint8_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n) return;
    Emit<true> o{out + offsets[i]};
    run_row(a, i, o);
}

int n_inputs(int op) {
    switch (op) {
        case ROGTK_STR_REVCOMP:
        case ROGTK_STR_PARSE_CIGAR:
        case ROGTK_STR_PHRED_STR:
        case ROGTK_STR_PHRED_LIST:
            return 1;
        case ROGTK_STR_CIGAR_INSERTIONS:
            return 2;
        case ROGTK_STR_ALIGNED_REF:
        case ROGTK_STR_ALIGNED_QUERY:
        case ROGTK_STR_ENRICH_ALLELE:
            return 3;
        default:
            return -1;
    }
}

int make_args(int op, const rogtk_str_col* cols, int n_cols, int64_t n_rows, int64_t param, OpArgs* a) {
    const int need = n_inputs(op);
    ROGTK_REQUIRE(need > 0, ROGTK_E_INVALID, "unknown string op %d", op);
    ROGTK_REQUIRE(n_cols == need, ROGTK_E_INVALID, "string op %d takes %d input columns, got %d", op, need, n_cols);
    ROGTK_REQUIRE(n_rows >= 0, ROGTK_E_INVALID, "n_rows must be >= 0");
    if (op == ROGTK_STR_PARSE_CIGAR) param = param != 0;
    if (op == ROGTK_STR_PHRED_STR || op == ROGTK_STR_PHRED_LIST)
        ROGTK_REQUIRE(param >= 0 && param <= 255, ROGTK_E_INVALID, "base %lld does not fit in u8", (long long)param);
    *a = OpArgs{op, n_rows, param, {}};
    for (int k = 0; k < need; ++k) {
        const rogtk_str_col& c = cols[k];
        ROGTK_REQUIRE(c.offset_width == 4 || c.offset_width == 8, ROGTK_E_INVALID, "offset_width must be 4 or 8");
        ROGTK_REQUIRE(c.n == n_rows || c.n == 1, ROGTK_E_INVALID,
                      "input %d has %lld rows (expected %lld or a broadcast of 1)", k, (long long)c.n,
                      (long long)n_rows);
        a->cols.c[k] = Col{c.offsets, c.offset_width, c.values, c.validity, c.validity_offset,
                           c.n == 1 && n_rows != 1 ? 1 : 0};
    }
    return ROGTK_OK;
}

inline unsigned grid_rows(int64_t n) { return (unsigned)std::max<int64_t>((n + kBlock - 1) / kBlock, 1); }

// per-thread scan scratch of the host entry point
struct StrCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    DevBuf off[3], val[3], valid[3], lengths, offsets, bits, cub, out;
    ~StrCtx() {
        if (stream) hipStreamDestroy(stream);
    }
};
thread_local std::unique_ptr<StrCtx> t_str;

}  // namespace
}  // namespace rogtk

using namespace rogtk;

extern "C" {

int rogtk_str_temp_bytes(int64_t n_rows, int64_t* bytes) {
    ROGTK_REQUIRE(bytes && n_rows >= 0, ROGTK_E_INVALID, "bad arguments");
    size_t tb = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (const int64_t*)nullptr, (int64_t*)nullptr,
                                                     (int)(n_rows + 1)));
    // lengths (n + 1 int64) + the scan's own storage
    *bytes = (int64_t)((n_rows + 1) * 8 + 256 + tb);
    return ROGTK_OK;
}

int rogtk_str_measure(int op, const rogtk_str_col* cols, int n_cols, int64_t n_rows, int64_t param,
                      int64_t* out_offsets, uint64_t* out_valid_bits, void* temp, int64_t temp_bytes,
                      void* stream) {
    OpArgs a;
    if (int rc = make_args(op, cols, n_cols, n_rows, param, &a)) return rc;
    ROGTK_REQUIRE(n_rows < (int64_t)1 << 31, ROGTK_E_UNSUPPORTED, "at most 2^31 - 1 rows per call");
    ROGTK_REQUIRE(out_offsets && out_valid_bits && temp, ROGTK_E_INVALID, "null output / temp pointer");
    hipStream_t s = (hipStream_t)stream;
    int64_t* lengths = (int64_t*)temp;
    const size_t head = ((size_t)(n_rows + 1) * 8 + 255) / 256 * 256;
    size_t tb = 0;
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, lengths, out_offsets, (int)(n_rows + 1), s));
    ROGTK_REQUIRE((int64_t)(head + tb) <= temp_bytes, ROGTK_E_INVALID, "temp_bytes %lld too small (need %lld)",
                  (long long)temp_bytes, (long long)(head + tb));
    ROGTK_HIP_CHECK(hipMemsetAsync(lengths + n_rows, 0, 8, s));
    if (n_rows > 0)
        hipLaunchKernelGGL(k_str_measure, dim3(grid_rows(n_rows)), dim3(kBlock), 0, s, a, lengths, out_valid_bits);
    ROGTK_HIP_CHECK(hipGetLastError());
    ROGTK_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum((uint8_t*)temp + head, tb, lengths, out_offsets,
                                                     (int)(n_rows + 1), s));
    return ROGTK_OK;
}

int rogtk_str_fill(int op, const rogtk_str_col* cols, int n_cols, int64_t n_rows, int64_t param,
                   const int64_t* offsets, uint8_t* out_values, void* stream) {
    OpArgs a;
    if (int rc = make_args(op, cols, n_cols, n_rows, param, &a)) return rc;
    if (n_rows > 0)
        hipLaunchKernelGGL(k_str_fill, dim3(grid_rows(n_rows)), dim3(kBlock), 0, (hipStream_t)stream, a, offsets,
                           out_values);
    ROGTK_HIP_CHECK(hipGetLastError());
    return ROGTK_OK;
}

int rogtk_str_transform_host(int op, const rogtk_str_col* cols, int n_cols, int64_t n_rows, int64_t param,
                             rogtk_str_result* out) {
    ROGTK_REQUIRE(out && cols, ROGTK_E_INVALID, "null argument");
    *out = rogtk_str_result{};
    {
        OpArgs chk;
        if (int rc = make_args(op, cols, n_cols, n_rows, param, &chk)) return rc;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_error("no HIP device available (librogtk_hip needs an MI355X / gfx950 GPU)");
        return ROGTK_E_NODEVICE;
    }
    int dev = 0;
    ROGTK_HIP_CHECK(hipGetDevice(&dev));
    if (!t_str || t_str->device != dev) {
        t_str.reset(new StrCtx());
        t_str->device = dev;
        ROGTK_HIP_CHECK(hipStreamCreateWithFlags(&t_str->stream, hipStreamNonBlocking));
    }
    StrCtx* c = t_str.get();
    hipStream_t s = c->stream;
    // upload the input columns (values [off(0), off(n)); offsets rebased to 0)
    rogtk_str_col dcols[3];
    std::vector<int64_t> off64;
    for (int k = 0; k < n_cols; ++k) {
        const rogtk_str_col& h = cols[k];
        const int64_t n = h.n;
        off64.resize(n + 1);
        for (int64_t r = 0; r <= n; ++r)
            off64[r] = h.offset_width == 4 ? ((const int32_t*)h.offsets)[r] : ((const int64_t*)h.offsets)[r];
        const int64_t base = off64[0], vb = off64[n] - base;
        ROGTK_REQUIRE(vb >= 0 && (h.values_len < 0 || off64[n] <= h.values_len), ROGTK_E_INVALID,
                      "input %d: offsets reference bytes outside values", k);
        for (int64_t r = 0; r <= n; ++r) off64[r] -= base;
        if (c->off[k].ensure((size_t)(n + 1) * 8) || c->val[k].ensure((size_t)std::max<int64_t>(vb, 1)))
            return ROGTK_E_HIP;
        ROGTK_HIP_CHECK(hipMemcpyAsync(c->off[k].p, off64.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, s));
        if (vb > 0)
            ROGTK_HIP_CHECK(hipMemcpyAsync(c->val[k].p, h.values + base, (size_t)vb, hipMemcpyHostToDevice, s));
        const uint8_t* dvalid = nullptr;
        if (h.validity) {
            const size_t nb = (size_t)((h.validity_offset + n + 7) / 8);
            if (c->valid[k].ensure(std::max<size_t>(nb, 1))) return ROGTK_E_HIP;
            ROGTK_HIP_CHECK(hipMemcpyAsync(c->valid[k].p, h.validity, nb, hipMemcpyHostToDevice, s));
            dvalid = c->valid[k].as<uint8_t>();
        }
        // the host staging buffer is reused by the next column: wait for the copy
        ROGTK_HIP_CHECK(hipStreamSynchronize(s));
        dcols[k] = rogtk_str_col{c->off[k].p, 8, c->val[k].as<uint8_t>(), vb, dvalid, h.validity_offset, n};
    }
    int64_t tb = 0;
    if (int rc = rogtk_str_temp_bytes(n_rows, &tb)) return rc;
    const int64_t words = std::max<int64_t>((n_rows + 63) / 64, 1);
    if (c->cub.ensure((size_t)tb) || c->offsets.ensure((size_t)(n_rows + 1) * 8) ||
        c->bits.ensure((size_t)words * 8))
        return ROGTK_E_HIP;
    if (int rc = rogtk_str_measure(op, dcols, n_cols, n_rows, param, c->offsets.as<int64_t>(), c->bits.as<uint64_t>(),
                                   c->cub.p, tb, s))
        return rc;
    int64_t* offs = (int64_t*)malloc((size_t)(n_rows + 1) * 8);
    uint8_t* bits = (uint8_t*)malloc((size_t)words * 8);
    if (!offs || !bits) {
        free(offs);
        free(bits);
        set_error("out of host memory");
        return ROGTK_E_INVALID;
    }
    *out = rogtk_str_result{n_rows, offs, nullptr, 0, bits, 0};
    ROGTK_HIP_CHECK(hipMemcpyAsync(offs, c->offsets.p, (size_t)(n_rows + 1) * 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipMemcpyAsync(bits, c->bits.p, (size_t)words * 8, hipMemcpyDeviceToHost, s));
    ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    const int64_t total = offs[n_rows];
    out->values = (uint8_t*)malloc((size_t)std::max<int64_t>(total, 1));
    ROGTK_REQUIRE(out->values, ROGTK_E_INVALID, "out of host memory for %lld output bytes", (long long)total);
    out->values_len = total;
    if (total > 0) {
        if (c->out.ensure((size_t)total)) return ROGTK_E_HIP;
        if (int rc = rogtk_str_fill(op, dcols, n_cols, n_rows, param, c->offsets.as<int64_t>(), c->out.as<uint8_t>(),
                                    s))
            return rc;
        ROGTK_HIP_CHECK(hipMemcpyAsync(out->values, c->out.p, (size_t)total, hipMemcpyDeviceToHost, s));
        ROGTK_HIP_CHECK(hipStreamSynchronize(s));
    }
    int64_t nulls = 0;
    for (int64_t r = 0; r < n_rows; ++r) nulls += !((bits[r >> 3] >> (r & 7)) & 1);
    out->null_count = nulls;
    return ROGTK_OK;
}

void rogtk_str_result_free(rogtk_str_result* r) {
    if (!r) return;
    free(r->offsets);
    free(r->values);
    free(r->validity);
    *r = rogtk_str_result{};
}

}  // extern "C"
