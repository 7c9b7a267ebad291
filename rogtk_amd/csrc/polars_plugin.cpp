// polars expression-plugin ABI of librogtk_hip.so: the drop-in boundary itself.
//
// The reference registers its expressions with
//   register_plugin_function(plugin_path=Path(__file__).parent, function_name=<name>, ...)
// (rogtk/__init__.py:138-156, 216-234, 266-287, 305-323, 333-349, 419-526); polars then
// dlopens the shared library in the package directory and calls the symbols that
// pyo3-polars 0.17's #[polars_expr] generates (Cargo.toml:39; src/expressions.rs:1048,
// 1075, 1234, 1286-1410, 695, 770, 880; src/fracture_opt.rs:283):
//
//   void _polars_plugin_<name>(SeriesExport* inputs, size_t n_inputs,
//                              const uint8_t* kwargs, size_t kwargs_len,
//                              SeriesExport* out, CallerContext* ctx);
//   void _polars_plugin_field_<name>(ArrowSchema* fields, size_t n_fields,
//                                    ArrowSchema* out, const uint8_t* kwargs, size_t kwargs_len);
//   uint32_t _polars_plugin_get_version(void);
//   const char* _polars_plugin_get_last_error_message(void);
//
// Protocol as implemented by polars-ffi version_0 (crate sources are not in this image:
// restated, marked unverified in SURVEY.md §8b):
//   * inputs are moved into the plugin: it releases every input ArrowArray and then
//     calls each input SeriesExport's release;
//   * the output SeriesExport owns one schema and `len` ArrowArray pointers; the caller
//     moves the arrays out (and releases them itself), then calls out->release, which
//     frees the containers and the schema but not the arrays;
//   * on error nothing is written to *out (private_data stays NULL) and the message is
//     kept per thread for _polars_plugin_get_last_error_message;
//   * kwargs arrive as a Python pickle of a flat dict (polars `pickle.dumps(kwargs,
//     protocol=5)`, serde-pickle on the Rust side): unknown keys are ignored, missing
//     Option fields are None, a missing required field is an error.
//
// Compute goes through the Level-2 host entry points of include/rogtk_hip.h (GPU
// kernels), never through a CPU implementation. Strings may arrive as Utf8 ("u"),
// LargeUtf8 ("U") or Utf8View ("vu", polars' own String layout); views are flattened
// on the host into int64 offsets + values before the H2D copy. String results are
// exported as Utf8View like polars' own.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rogtk_hip.h"

namespace {

// ----------------------------------------------------- Arrow C Data Interface
struct ArrowSchema {
    const char* format;
    const char* name;
    const char* metadata;
    int64_t flags;
    int64_t n_children;
    ArrowSchema** children;
    ArrowSchema* dictionary;
    void (*release)(ArrowSchema*);
    void* private_data;
};
struct ArrowArray {
    int64_t length;
    int64_t null_count;
    int64_t offset;
    int64_t n_buffers;
    int64_t n_children;
    const void** buffers;
    ArrowArray** children;
    ArrowArray* dictionary;
    void (*release)(ArrowArray*);
    void* private_data;
};
constexpr int64_t ARROW_FLAG_NULLABLE = 2;

// polars-ffi version_0
struct SeriesExport {
    ArrowSchema* field;
    ArrowArray** arrays;
    size_t len;
    void (*release)(SeriesExport*);
    void* private_data;
};
struct CallerContext {
    uint64_t bitflags;
};

thread_local std::string t_plugin_err;

struct PluginError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

[[noreturn]] void fail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void fail(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    throw PluginError(buf);
}

void check(int rc) {
    if (rc != ROGTK_OK) throw PluginError(rogtk_last_error());
}

// ------------------------------------------------------------- kwargs (pickle)
// A pickle VM restricted to what `pickle.dumps(<flat dict>, protocol=2..5)` emits for
// str / int / bool / float / None values (plus lists and tuples of them).
struct PVal {
    enum Kind { NONE, BOOL, INT, FLOAT, STR, LIST, DICT, MARK } kind = NONE;
    bool b = false;
    int64_t i = 0;
    double f = 0;
    std::string s;
    std::vector<std::shared_ptr<PVal>> items;  // LIST; DICT as key, value pairs
};
using PV = std::shared_ptr<PVal>;

struct Kwargs {
    std::map<std::string, PV> m;
    bool has(const char* k) const {
        auto it = m.find(k);
        return it != m.end() && it->second->kind != PVal::NONE;
    }
    const PVal& req(const char* k) const {
        auto it = m.find(k);
        if (it == m.end()) fail("could not parse kwargs: missing field `%s`", k);
        return *it->second;
    }
    std::string str(const char* k) const {
        const PVal& v = req(k);
        if (v.kind != PVal::STR) fail("could not parse kwargs: invalid type for `%s`, expected a string", k);
        return v.s;
    }
    int64_t uint(const char* k) const {
        const PVal& v = req(k);
        if (v.kind == PVal::INT && v.i >= 0) return v.i;
        if (v.kind == PVal::BOOL) return v.b ? 1 : 0;
        fail("could not parse kwargs: invalid type for `%s`, expected an unsigned integer", k);
    }
    bool opt_str(const char* k, std::string* out) const {
        if (!has(k)) return false;
        *out = str(k);
        return true;
    }
    int64_t opt_uint(const char* k, int64_t dflt) const { return has(k) ? uint(k) : dflt; }
    bool opt_bool(const char* k, bool dflt) const {
        if (!has(k)) return dflt;
        const PVal& v = req(k);
        if (v.kind == PVal::BOOL) return v.b;
        fail("could not parse kwargs: invalid type for `%s`, expected a boolean", k);
    }
};

Kwargs parse_kwargs(const uint8_t* p, size_t n) {
    Kwargs kw;
    if (n == 0 || p == nullptr) return kw;
    std::vector<PV> st;
    std::vector<size_t> marks;
    std::map<uint64_t, PV> memo;
    size_t i = 0;
    auto need = [&](size_t k) {
        if (i + k > n) fail("could not parse kwargs: truncated pickle");
    };
    auto u = [&](int bytes) -> uint64_t {
        need(bytes);
        uint64_t v = 0;
        for (int b = 0; b < bytes; ++b) v |= (uint64_t)p[i + b] << (8 * b);
        i += bytes;
        return v;
    };
    auto mk = [](PVal::Kind k) {
        auto v = std::make_shared<PVal>();
        v->kind = k;
        return v;
    };
    auto pop = [&]() {
        if (st.empty()) fail("could not parse kwargs: pickle stack underflow");
        PV v = st.back();
        st.pop_back();
        return v;
    };
    auto pop_mark = [&]() {
        if (marks.empty()) fail("could not parse kwargs: pickle mark underflow");
        size_t m = marks.back();
        marks.pop_back();
        std::vector<PV> out(st.begin() + m, st.end());
        st.resize(m);
        return out;
    };
    auto set_items = [&](PV d, const std::vector<PV>& kv) {
        if (d->kind != PVal::DICT || kv.size() % 2) fail("could not parse kwargs: malformed dict");
        for (const PV& x : kv) d->items.push_back(x);
    };
    for (;;) {
        need(1);
        const uint8_t op = p[i++];
        switch (op) {
            case 0x80: u(1); break;           // PROTO
            case 0x95: u(8); break;           // FRAME
            case '}': st.push_back(mk(PVal::DICT)); break;
            case ']': st.push_back(mk(PVal::LIST)); break;
            case ')': st.push_back(mk(PVal::LIST)); break;  // EMPTY_TUPLE
            case '(': marks.push_back(st.size()); break;     // MARK
            case 'N': st.push_back(mk(PVal::NONE)); break;
            case 0x88: { auto v = mk(PVal::BOOL); v->b = true; st.push_back(v); break; }
            case 0x89: { auto v = mk(PVal::BOOL); v->b = false; st.push_back(v); break; }
            case 'K': { auto v = mk(PVal::INT); v->i = (int64_t)u(1); st.push_back(v); break; }
            case 'M': { auto v = mk(PVal::INT); v->i = (int64_t)u(2); st.push_back(v); break; }
            case 'J': { auto v = mk(PVal::INT); v->i = (int64_t)(int32_t)(uint32_t)u(4); st.push_back(v); break; }
            case 0x8a: {  // LONG1: little-endian two's complement
                const uint64_t len = u(1);
                need(len);
                if (len > 8) fail("could not parse kwargs: integer too large");
                uint64_t v = 0;
                for (uint64_t b = 0; b < len; ++b) v |= (uint64_t)p[i + b] << (8 * b);
                if (len > 0 && len < 8 && (p[i + len - 1] & 0x80)) v |= ~0ull << (8 * len);
                i += len;
                auto x = mk(PVal::INT);
                x->i = (int64_t)v;
                st.push_back(x);
                break;
            }
            case 'G': {  // BINFLOAT, big-endian
                need(8);
                uint64_t bits = 0;
                for (int b = 0; b < 8; ++b) bits = (bits << 8) | p[i + b];
                i += 8;
                auto v = mk(PVal::FLOAT);
                memcpy(&v->f, &bits, 8);
                st.push_back(v);
                break;
            }
            case 0x8c: case 'X': case 0x8d: case 'C': case 'B': case 0x8e: {
                // SHORT_BINUNICODE / BINUNICODE / BINUNICODE8 / SHORT_BINBYTES / BINBYTES / BINBYTES8
                const int w = (op == 0x8c || op == 'C') ? 1 : (op == 'X' || op == 'B') ? 4 : 8;
                const uint64_t len = u(w);
                need(len);
                auto v = mk(PVal::STR);
                v->s.assign((const char*)p + i, len);
                i += len;
                st.push_back(v);
                break;
            }
            case 0x94:  // MEMOIZE
                if (st.empty()) fail("could not parse kwargs: memoize on empty stack");
                memo[memo.size()] = st.back();
                break;
            case 'q': { const uint64_t k = u(1); if (st.empty()) fail("could not parse kwargs: bad put"); memo[k] = st.back(); break; }
            case 'r': { const uint64_t k = u(4); if (st.empty()) fail("could not parse kwargs: bad put"); memo[k] = st.back(); break; }
            case 'h': case 'j': {
                const uint64_t k = u(op == 'h' ? 1 : 4);
                auto it = memo.find(k);
                if (it == memo.end()) fail("could not parse kwargs: bad memo reference");
                st.push_back(it->second);
                break;
            }
            case 's': {  // SETITEM
                PV v = pop(), k = pop();
                PV d = pop();
                set_items(d, {k, v});
                st.push_back(d);
                break;
            }
            case 'u': {  // SETITEMS
                std::vector<PV> kv = pop_mark();
                PV d = pop();
                set_items(d, kv);
                st.push_back(d);
                break;
            }
            case 'a': { PV v = pop(); PV l = pop(); l->items.push_back(v); st.push_back(l); break; }
            case 'e': { std::vector<PV> xs = pop_mark(); PV l = pop(); for (auto& x : xs) l->items.push_back(x); st.push_back(l); break; }
            case 't': { std::vector<PV> xs = pop_mark(); auto l = mk(PVal::LIST); l->items = xs; st.push_back(l); break; }
            case 0x85: case 0x86: case 0x87: {  // TUPLE1..3
                const int k = op - 0x84;
                auto l = mk(PVal::LIST);
                l->items.resize(k);
                for (int j = k - 1; j >= 0; --j) l->items[j] = pop();
                st.push_back(l);
                break;
            }
            case '.': {  // STOP
                PV d = pop();
                if (d->kind != PVal::DICT) fail("could not parse kwargs: expected a dict");
                for (size_t j = 0; j + 1 < d->items.size(); j += 2) {
                    if (d->items[j]->kind != PVal::STR) fail("could not parse kwargs: non-string key");
                    kw.m[d->items[j]->s] = d->items[j + 1];
                }
                return kw;
            }
            default:
                fail("could not parse kwargs: unsupported pickle opcode 0x%02x", op);
        }
    }
}

// ------------------------------------------------------------------ inputs
struct Chunk {
    // normalised host view of one string chunk
    int ow = 8;
    const void* offsets = nullptr;  // ow-byte offsets, n + 1
    const uint8_t* values = nullptr;
    int64_t values_len = 0;
    const uint8_t* validity = nullptr;
    int64_t voff = 0;
    int64_t n = 0;
    std::vector<int64_t> own_off;  // flattened views
    std::vector<uint8_t> own_val;
    bool valid(int64_t r) const {
        if (!validity) return true;
        const int64_t b = voff + r;
        return (validity[b >> 3] >> (b & 7)) & 1;
    }
    int64_t off(int64_t r) const {
        return ow == 4 ? ((const int32_t*)offsets)[r] : ((const int64_t*)offsets)[r];
    }
};

std::string dtype_name(const char* f) {
    if (!f) return "unknown";
    static const std::map<std::string, std::string> names = {
        {"n", "null"}, {"b", "bool"}, {"c", "i8"}, {"C", "u8"}, {"s", "i16"}, {"S", "u16"},
        {"i", "i32"}, {"I", "u32"}, {"l", "i64"}, {"L", "u64"}, {"f", "f32"}, {"g", "f64"},
        {"z", "binary"}, {"Z", "binary"}, {"vz", "binary"}, {"+s", "struct"}, {"+l", "list"},
        {"+L", "list"}};
    auto it = names.find(f);
    return it == names.end() ? std::string(f) : it->second;
}

struct StrSeries {
    std::string name;
    std::vector<Chunk> chunks;
    int64_t len() const {
        int64_t t = 0;
        for (auto& c : chunks) t += c.n;
        return t;
    }
};

// `inputs[i].str()?`: a String series or polars' dtype error.
StrSeries str_series(const SeriesExport& s) {
    StrSeries out;
    if (!s.field || !s.field->format) fail("input series has no field");
    out.name = s.field->name ? s.field->name : "";
    const std::string fmt = s.field->format;
    if (fmt != "u" && fmt != "U" && fmt != "vu")
        fail("invalid series dtype: expected `String`, got `%s`", dtype_name(fmt.c_str()).c_str());
    for (size_t c = 0; c < s.len; ++c) {
        const ArrowArray* a = s.arrays[c];
        Chunk ch;
        ch.n = a->length;
        ch.validity = a->null_count == 0 ? nullptr : (const uint8_t*)a->buffers[0];
        ch.voff = a->offset;
        if (fmt == "u" || fmt == "U") {
            ch.ow = fmt == "u" ? 4 : 8;
            ch.offsets = (const uint8_t*)a->buffers[1] + (size_t)a->offset * ch.ow;
            ch.values = (const uint8_t*)a->buffers[2];
            const int64_t base = ch.n ? ch.off(0) : 0;
            if (base != 0) {
                // the host entry points take offsets starting at 0: rebase a sliced chunk
                ch.own_off.resize(ch.n + 1);
                for (int64_t r = 0; r <= ch.n; ++r) ch.own_off[r] = ch.off(r) - base;
                ch.ow = 8;
                ch.offsets = ch.own_off.data();
                ch.values += base;
            }
            ch.values_len = ch.n ? ch.off(ch.n) : 0;
        } else {
            // Utf8View: 16-byte views {len, inline[12]} or {len, prefix, buffer, offset}
            const uint8_t* views = (const uint8_t*)a->buffers[1] + (size_t)a->offset * 16;
            const int64_t n_data = a->n_buffers - 3;
            ch.own_off.resize(ch.n + 1);
            int64_t tot = 0;
            for (int64_t r = 0; r < ch.n; ++r) {
                int32_t L;
                memcpy(&L, views + 16 * r, 4);
                if (ch.valid(r)) tot += L;
            }
            ch.own_val.resize(std::max<int64_t>(tot, 1));
            int64_t pos = 0;
            for (int64_t r = 0; r < ch.n; ++r) {
                ch.own_off[r] = pos;
                if (!ch.valid(r)) continue;
                const uint8_t* v = views + 16 * r;
                int32_t L;
                memcpy(&L, v, 4);
                if (L <= 12) {
                    memcpy(ch.own_val.data() + pos, v + 4, L);
                } else {
                    int32_t bi, bo;
                    memcpy(&bi, v + 8, 4);
                    memcpy(&bo, v + 12, 4);
                    if (bi < 0 || bi >= n_data) fail("Utf8View buffer index %d out of range", bi);
                    memcpy(ch.own_val.data() + pos, (const uint8_t*)a->buffers[2 + bi] + bo, L);
                }
                pos += L;
            }
            ch.own_off[ch.n] = pos;
            ch.ow = 8;
            ch.offsets = ch.own_off.data();
            ch.values = ch.own_val.data();
            ch.values_len = pos;
        }
        out.chunks.push_back(std::move(ch));
    }
    return out;
}

// All non-null strings of a series in order (`ca.into_iter().flatten()`), as one chunk.
Chunk flatten_non_null(const StrSeries& s) {
    Chunk g;
    g.ow = 8;
    for (const Chunk& c : s.chunks)
        for (int64_t r = 0; r < c.n; ++r) {
            if (!c.valid(r)) continue;
            const int64_t a = c.off(r), b = c.off(r + 1);
            g.own_off.push_back((int64_t)g.own_val.size());
            g.own_val.insert(g.own_val.end(), c.values + a, c.values + b);
        }
    g.own_off.push_back((int64_t)g.own_val.size());
    g.n = (int64_t)g.own_off.size() - 1;
    if (g.own_val.empty()) g.own_val.push_back(0);
    g.offsets = g.own_off.data();
    g.values = g.own_val.data();
    g.values_len = g.own_off.back();
    return g;
}

// `series.get(0)` of a String series: the first row, or nothing when empty / null.
bool first_value(const StrSeries& s, std::string* out) {
    for (const Chunk& c : s.chunks) {
        if (c.n == 0) continue;
        if (!c.valid(0)) return false;
        out->assign((const char*)c.values + c.off(0), (size_t)(c.off(1) - c.off(0)));
        return true;
    }
    return false;
}

void release_inputs(SeriesExport* in, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        SeriesExport& s = in[i];
        for (size_t c = 0; c < s.len && s.arrays; ++c)
            if (s.arrays[c] && s.arrays[c]->release) s.arrays[c]->release(s.arrays[c]);
        if (s.release) s.release(&s);
    }
}

// ----------------------------------------------------------------- outputs
// Schema: owns its strings and children.
struct SchemaHolder {
    std::string format, name;
    std::vector<ArrowSchema*> children;
};
void release_schema(ArrowSchema* s) {
    if (!s || !s->release) return;
    auto* h = (SchemaHolder*)s->private_data;
    for (ArrowSchema* c : h->children) {
        if (c->release) c->release(c);
        delete c;
    }
    delete h;
    s->release = nullptr;
}

struct FieldSpec {
    std::string name, format;
    std::vector<FieldSpec> children;
};
void fill_schema(ArrowSchema* s, const FieldSpec& f) {
    auto* h = new SchemaHolder{f.format, f.name, {}};
    for (const FieldSpec& c : f.children) {
        auto* cs = new ArrowSchema();
        fill_schema(cs, c);
        h->children.push_back(cs);
    }
    s->format = h->format.c_str();
    s->name = h->name.c_str();
    s->metadata = nullptr;
    s->flags = ARROW_FLAG_NULLABLE;
    s->n_children = (int64_t)h->children.size();
    s->children = h->children.empty() ? nullptr : h->children.data();
    s->dictionary = nullptr;
    s->release = release_schema;
    s->private_data = h;
}

// Array: owns its buffers and children.
struct ArrayHolder {
    std::vector<std::vector<uint8_t>> bufs;
    std::vector<const void*> ptrs;
    std::vector<ArrowArray*> children;
};
void release_array(ArrowArray* a) {
    if (!a || !a->release) return;
    auto* h = (ArrayHolder*)a->private_data;
    for (ArrowArray* c : h->children) {
        if (c->release) c->release(c);
        delete c;
    }
    delete h;
    a->release = nullptr;
}

// One output column under construction (buffers + children).
struct Col {
    int64_t length = 0, null_count = 0;
    std::vector<std::vector<uint8_t>> bufs;  // empty vector => NULL buffer
    std::vector<Col> children;
};
ArrowArray* to_arrow(Col&& c) {
    auto* a = new ArrowArray();
    auto* h = new ArrayHolder();
    h->bufs = std::move(c.bufs);
    for (auto& b : h->bufs) h->ptrs.push_back(b.empty() ? nullptr : b.data());
    for (Col& ch : c.children) h->children.push_back(to_arrow(std::move(ch)));
    a->length = c.length;
    a->null_count = c.null_count;
    a->offset = 0;
    a->n_buffers = (int64_t)h->ptrs.size();
    a->n_children = (int64_t)h->children.size();
    a->buffers = h->ptrs.empty() ? nullptr : h->ptrs.data();
    a->children = h->children.empty() ? nullptr : h->children.data();
    a->dictionary = nullptr;
    a->release = release_array;
    a->private_data = h;
    return a;
}

// Validity of a chunk rebased to bit offset 0 (empty when the chunk has no nulls).
std::vector<uint8_t> rebased_validity(const Chunk& c, int64_t* nulls) {
    *nulls = 0;
    if (!c.validity) return {};
    std::vector<uint8_t> v((size_t)(c.n + 7) / 8, 0);
    for (int64_t r = 0; r < c.n; ++r) {
        if (c.valid(r))
            v[r >> 3] |= (uint8_t)(1u << (r & 7));
        else
            ++*nulls;
    }
    if (*nulls == 0) return {};
    return v;
}

template <class T>
Col prim_col(const std::vector<uint8_t>& validity, int64_t nulls, std::vector<T>&& vals, int64_t n) {
    Col c;
    c.length = n;
    c.null_count = nulls;
    c.bufs.push_back(validity);
    std::vector<uint8_t> b(std::max<size_t>(vals.size() * sizeof(T), 1));
    if (!vals.empty()) memcpy(b.data(), vals.data(), vals.size() * sizeof(T));
    c.bufs.push_back(std::move(b));
    return c;
}

// Utf8View column of the given strings (all valid).
Col view_col(const std::vector<std::string>& strs) {
    Col c;
    c.length = (int64_t)strs.size();
    std::vector<uint8_t> views(std::max<size_t>(strs.size() * 16, 16), 0), data;
    for (size_t r = 0; r < strs.size(); ++r) {
        const std::string& s = strs[r];
        if (s.size() > (size_t)std::numeric_limits<int32_t>::max()) fail("string too long for a Utf8View");
        const int32_t L = (int32_t)s.size();
        uint8_t* v = views.data() + 16 * r;
        memcpy(v, &L, 4);
        if (L <= 12) {
            memcpy(v + 4, s.data(), L);
        } else {
            const int32_t bi = 0, bo = (int32_t)data.size();
            memcpy(v + 4, s.data(), 4);
            memcpy(v + 8, &bi, 4);
            memcpy(v + 12, &bo, 4);
            data.insert(data.end(), s.begin(), s.end());
        }
    }
    const int64_t dlen = (int64_t)data.size();
    if (data.empty()) data.push_back(0);
    std::vector<uint8_t> sizes(8);
    memcpy(sizes.data(), &dlen, 8);
    c.bufs.push_back({});
    c.bufs.push_back(std::move(views));
    c.bufs.push_back(std::move(data));
    c.bufs.push_back(std::move(sizes));
    return c;
}

Col struct_col(int64_t n, std::vector<Col>&& children) {
    Col c;
    c.length = n;
    c.bufs.push_back({});
    c.children = std::move(children);
    return c;
}

struct ExportHolder {
    ArrowSchema schema;
    std::vector<ArrowArray*> arrays;
};
void release_export(SeriesExport* e) {
    if (!e || !e->release) return;
    auto* h = (ExportHolder*)e->private_data;
    if (h->schema.release) h->schema.release(&h->schema);
    for (ArrowArray* a : h->arrays) delete a;  // containers only: the consumer moved the arrays out
    delete h;
    e->release = nullptr;
    e->private_data = nullptr;
}

void export_series(SeriesExport* out, const FieldSpec& f, std::vector<Col>&& chunks) {
    auto* h = new ExportHolder();
    fill_schema(&h->schema, f);
    for (Col& c : chunks) h->arrays.push_back(to_arrow(std::move(c)));
    out->field = &h->schema;
    out->arrays = h->arrays.data();
    out->len = h->arrays.size();
    out->release = release_export;
    out->private_data = h;
}

// ------------------------------------------------------------ expressions
const char* const SCORE_NAMES[7] = {"shannon_entropy",         "linguistic_complexity", "homopolymer_fraction",
                                    "dinucleotide_entropy",    "longest_homopolymer_run", "dust_score",
                                    "combined_score"};

FieldSpec complexity_struct(const std::string& name) {
    FieldSpec f{name, "+s", {}};
    for (int j = 0; j < 7; ++j) f.children.push_back({SCORE_NAMES[j], j == 4 ? "I" : "g", {}});
    return f;
}

// umi_complexity_all_expr (expressions.rs:1234-1284) when field < 0, else the
// single-field expr for SCORE_NAMES[field] (:1286-1410).
void umi_complexity(SeriesExport* in, size_t n_in, SeriesExport* out, int field) {
    if (n_in < 1) fail("expected one input series");
    StrSeries s = str_series(in[0]);
    std::vector<Col> chunks;
    for (const Chunk& c : s.chunks) {
        const int64_t n = c.n;
        std::vector<std::vector<double>> f64(7);
        std::vector<uint32_t> longest;
        void* ptrs[7] = {};
        for (int j = 0; j < 7; ++j) {
            if (field >= 0 && field != j) continue;
            if (j == 4) {
                longest.resize(std::max<int64_t>(n, 1));
                ptrs[j] = longest.data();
            } else {
                f64[j].resize(std::max<int64_t>(n, 1));
                ptrs[j] = f64[j].data();
            }
        }
        rogtk_umi_scores sc{(double*)ptrs[0], (double*)ptrs[1], (double*)ptrs[2], (double*)ptrs[3],
                            (uint32_t*)ptrs[4], (double*)ptrs[5], (double*)ptrs[6]};
        check(rogtk_umi_complexity_host(c.offsets, c.ow, c.values, c.values_len, c.validity, c.voff, n, &sc));
        int64_t nulls = 0;
        std::vector<uint8_t> vb = rebased_validity(c, &nulls);
        auto child = [&](int j) {
            if (j == 4) {
                longest.resize(n);
                return prim_col(vb, nulls, std::move(longest), n);
            }
            f64[j].resize(n);
            return prim_col(vb, nulls, std::move(f64[j]), n);
        };
        if (field >= 0) {
            chunks.push_back(child(field));
        } else {
            std::vector<Col> kids;
            for (int j = 0; j < 7; ++j) kids.push_back(child(j));
            // df.into_struct: the struct rows themselves are valid; the fields carry the nulls
            chunks.push_back(struct_col(n, std::move(kids)));
        }
    }
    if (field >= 0)
        export_series(out, {s.name, field == 4 ? "I" : "g", {}}, std::move(chunks));
    else
        export_series(out, complexity_struct(s.name), std::move(chunks));
}

// hamming_distance_expr / hamming_within_expr (expressions.rs:1048-1101).
void hamming(SeriesExport* in, size_t n_in, const Kwargs& kw, SeriesExport* out, bool within) {
    if (n_in < 1) fail("expected one input series");
    const std::string target = kw.str("target");  // HammingKwargs.target: String (:1018)
    const int64_t maxd = within ? kw.opt_uint("max_distance", 1) : 1;
    if (maxd > 0xFFFFFFFFll) fail("could not parse kwargs: max_distance does not fit in u32");
    StrSeries s = str_series(in[0]);
    std::vector<Col> chunks;
    for (const Chunk& c : s.chunks) {
        const int64_t n = c.n;
        std::vector<uint32_t> dist;
        std::vector<uint8_t> bits;
        if (within)
            bits.assign(std::max<int64_t>((n + 7) / 8, 1), 0);
        else
            dist.resize(std::max<int64_t>(n, 1));
        const uint8_t tz = 0;
        check(rogtk_hamming_host(c.offsets, c.ow, c.values, c.values_len, c.validity, c.voff, n,
                                 target.empty() ? &tz : (const uint8_t*)target.data(), (int64_t)target.size(),
                                 (uint32_t)maxd, within ? nullptr : dist.data(), within ? bits.data() : nullptr));
        int64_t nulls = 0;
        std::vector<uint8_t> vb = rebased_validity(c, &nulls);
        if (within) {
            Col col;
            col.length = n;
            col.null_count = nulls;
            col.bufs.push_back(vb);
            col.bufs.push_back(std::move(bits));
            chunks.push_back(std::move(col));
        } else {
            dist.resize(n);
            chunks.push_back(prim_col(vb, nulls, std::move(dist), n));
        }
    }
    export_series(out, {s.name, within ? "b" : "I", {}}, std::move(chunks));
}

// The assembly call of one group: contigs joined by '\n' (rogtk_assemble_host).
std::string assemble_group(const Chunk& g, int64_t k, int64_t min_cov, const std::string& method,
                           const std::string* sa, const std::string* ea, int64_t min_length, bool auto_k) {
    const int kk = (int)std::min<int64_t>(k, 1 << 20);
    int64_t cap = std::max<int64_t>(g.values_len * 2 + 1024, 4096), need = 0, nc = 0;
    for (;;) {
        std::vector<char> buf(cap);
        const int rc = rogtk_assemble_host(g.offsets, g.ow, g.values, g.values_len, nullptr, 0, g.n, kk, min_cov,
                                           method.c_str(), sa ? sa->c_str() : nullptr, ea ? ea->c_str() : nullptr,
                                           1, min_length, auto_k ? 1 : 0, buf.data(), cap, &need, &nc);
        if (rc == ROGTK_E_OVERFLOW && need > cap) {
            cap = need;
            continue;
        }
        check(rc);
        return std::string(buf.data(), (size_t)need);
    }
}

// assemble_sequences_expr (expressions.rs:695-762); with_anchors (:770-849).
void assemble(SeriesExport* in, size_t n_in, const Kwargs& kw, SeriesExport* out, bool with_anchors) {
    const int64_t k = kw.uint("k"), min_cov = kw.uint("min_coverage");
    const std::string method = kw.str("method");
    std::string sa, ea;
    const bool has_sa = kw.opt_str("start_anchor", &sa), has_ea = kw.opt_str("end_anchor", &ea);
    const int64_t min_length = kw.opt_uint("min_length", -1);
    const bool auto_k = kw.opt_bool("auto_k", false);
    if (with_anchors) {
        if (n_in < 3)
            fail("assemble_sequences_with_anchors requires 3 inputs: sequences, start_anchor, end_anchor");
        StrSeries s1 = str_series(in[1]), s2 = str_series(in[2]);
        if (!first_value(s1, &sa)) fail("start_anchor column is empty");
        if (!first_value(s2, &ea)) fail("end_anchor column is empty");
        if (method == "compression")
            fail("compression method is not supported with dynamic anchors; use shortest_path");
        if (method == "shortest_path_auto")
            fail("shortest_path_auto method is not supported with dynamic anchors; use shortest_path");
        if (method != "shortest_path") fail("Invalid assembly method for dynamic anchors. Must be 'shortest_path'");
    } else {
        if (n_in < 1) fail("expected one input series");
        if (method == "compression" && (has_sa || has_ea))
            fail("Anchor sequences should not be provided for compression method");
        if (method == "shortest_path" && !(has_sa && has_ea))
            fail("Both start_anchor and end_anchor are required for shortest_path method");
        if (method == "shortest_path_auto" && (has_sa || has_ea))
            fail("Anchor sequences should not be provided for shortest_path_auto method");
        if (method != "compression" && method != "shortest_path" && method != "shortest_path_auto")
            fail("Invalid assembly method. Must be 'compression', 'shortest_path', or 'shortest_path_auto'");
    }
    StrSeries s = str_series(in[0]);
    Chunk g = flatten_non_null(s);
    const bool anchors = with_anchors || method == "shortest_path";
    std::string contigs;
    try {
        contigs = assemble_group(g, k, min_cov, method, anchors ? &sa : nullptr, anchors ? &ea : nullptr,
                                 min_length, auto_k);
    } catch (const PluginError& e) {
        fail("Assembly failed: %s", e.what());
    }
    std::vector<Col> chunks;
    chunks.push_back(view_col({contigs}));
    export_series(out, {"assembled_sequences", "vu", {}}, std::move(chunks));
}

// sweep_assembly_params_expr (expressions.rs:880-955).
void sweep(SeriesExport* in, size_t n_in, const Kwargs& kw, SeriesExport* out) {
    if (n_in < 1) fail("expected one input series");
    const int64_t ks = kw.uint("k_start"), ke = kw.uint("k_end"), kst = kw.uint("k_step");
    const int64_t cs = kw.uint("cov_start"), ce = kw.uint("cov_end"), cst = kw.uint("cov_step");
    const std::string method = kw.str("method");
    std::string sa, ea;
    const bool has_sa = kw.opt_str("start_anchor", &sa), has_ea = kw.opt_str("end_anchor", &ea);
    // step_by(0) panics in Rust; refuse it as an error instead of aborting the host
    if (kst == 0 || cst == 0) fail("assertion failed: step != 0");
    StrSeries s = str_series(in[0]);
    Chunk g = flatten_non_null(s);
    const int64_t nk = ke >= ks ? (ke - ks) / kst + 1 : 0, nc = ce >= cs ? (ce - cs) / cst + 1 : 0;
    const int64_t cap = std::max<int64_t>(nk * nc, 1);
    std::vector<int64_t> ok(cap), oc(cap), ol(cap);
    int64_t m = 0;
    check(rogtk_assembly_sweep_host(g.offsets, g.ow, g.values, g.values_len, nullptr, 0, g.n, ks, ke, kst, cs, ce,
                                    cst, method.c_str(), has_sa ? sa.c_str() : nullptr,
                                    has_ea ? ea.c_str() : nullptr, cap, ok.data(), oc.data(), ol.data(), &m));
    ok.resize(m);
    oc.resize(m);
    ol.resize(m);
    std::vector<Col> kids;
    kids.push_back(prim_col({}, 0, std::move(ok), m));
    kids.push_back(prim_col({}, 0, std::move(oc), m));
    kids.push_back(prim_col({}, 0, std::move(ol), m));
    std::vector<Col> chunks;
    chunks.push_back(struct_col(m, std::move(kids)));
    FieldSpec f{s.name, "+s", {{"k", "l", {}}, {"min_coverage", "l", {}}, {"contig_length", "l", {}}}};
    export_series(out, f, std::move(chunks));
}

FieldSpec optimize_struct(const std::string& name) {
    return {name,
            "+s",
            {{"contig", "vu", {}},
             {"k", "I", {}},
             {"min_coverage", "I", {}},
             {"length", "I", {}},
             {"input_sequences", "I", {}}}};
}

// optimize_assembly_expr (fracture_opt.rs:283-356).
void optimize(SeriesExport* in, size_t n_in, const Kwargs& kw, SeriesExport* out) {
    if (n_in < 1) fail("expected one input series");
    std::string sa, ea;
    const std::string method = kw.str("method");
    const int64_t start_k = kw.uint("start_k"), start_cov = kw.uint("start_min_coverage");
    const int64_t max_it = kw.opt_uint("max_iterations", 50);
    const bool explore_k = kw.opt_bool("explore_k", false), prio = kw.opt_bool("prioritize_length", false);
    StrSeries s = str_series(in[0]);
    if (!kw.opt_str("start_anchor", &sa)) fail("start_anchor is required");
    if (!kw.opt_str("end_anchor", &ea)) fail("end_anchor is required");
    Chunk g = flatten_non_null(s);
    int64_t cap = std::max<int64_t>(g.values_len * 2 + 1024, 4096), need = 0;
    uint32_t out4[4] = {};
    std::string contig;
    for (;;) {
        std::vector<char> buf(cap);
        const int rc = rogtk_assembly_optimize_host(g.offsets, g.ow, g.values, g.values_len, nullptr, 0, g.n,
                                                    method.c_str(), sa.c_str(), ea.c_str(), start_k, start_cov,
                                                    max_it, explore_k, prio, buf.data(), cap, &need, out4);
        if (rc == ROGTK_E_OVERFLOW && need > cap) {
            cap = need;
            continue;
        }
        check(rc);
        contig.assign(buf.data(), (size_t)need);
        break;
    }
    std::vector<Col> kids;
    kids.push_back(view_col({contig}));
    for (int j = 0; j < 4; ++j) kids.push_back(prim_col<uint32_t>({}, 0, {out4[j]}, 1));
    std::vector<Col> chunks;
    chunks.push_back(struct_col(1, std::move(kids)));
    export_series(out, optimize_struct(s.name), std::move(chunks));
}

// ------------------------------------------- element-wise string transforms
// A whole series as one host chunk, nulls kept (the row space the reference zips over).
struct FlatCol {
    std::vector<int64_t> off;
    std::vector<uint8_t> val, valid;
    int64_t n = 0, nulls = 0;
};
FlatCol flatten_all(const StrSeries& s) {
    FlatCol f;
    f.off.push_back(0);
    for (const Chunk& c : s.chunks)
        for (int64_t r = 0; r < c.n; ++r) {
            const bool ok = c.valid(r);
            if ((f.n & 7) == 0) f.valid.push_back(0);
            if (ok) {
                f.valid.back() |= (uint8_t)(1u << (f.n & 7));
                f.val.insert(f.val.end(), c.values + c.off(r), c.values + c.off(r + 1));
            } else {
                ++f.nulls;
            }
            f.off.push_back((int64_t)f.val.size());
            ++f.n;
        }
    if (f.val.empty()) f.val.push_back(0);
    if (f.valid.empty()) f.valid.push_back(0);
    return f;
}

rogtk_str_col str_desc(const FlatCol& f) {
    return rogtk_str_col{f.off.data(), 8, f.val.data(), (int64_t)f.val.size(), f.nulls ? f.valid.data() : nullptr,
                         0, f.n};
}

// Utf8View column of a rogtk_str_result (nulls kept).
Col view_col_result(const rogtk_str_result& r) {
    Col c;
    c.length = r.n;
    c.null_count = r.null_count;
    std::vector<uint8_t> views(std::max<size_t>((size_t)r.n * 16, 16), 0), data;
    for (int64_t i = 0; i < r.n; ++i) {
        const int64_t a = r.offsets[i], b = r.offsets[i + 1];
        if (b - a > (int64_t)std::numeric_limits<int32_t>::max()) fail("string too long for a Utf8View");
        const int32_t L = (int32_t)(b - a);
        uint8_t* v = views.data() + 16 * i;
        memcpy(v, &L, 4);
        if (L <= 12) {
            if (L) memcpy(v + 4, r.values + a, L);
        } else {
            const int32_t bi = 0, bo = (int32_t)data.size();
            if (data.size() + L > (size_t)std::numeric_limits<int32_t>::max()) fail("Utf8View buffer over 2 GiB");
            memcpy(v + 4, r.values + a, 4);
            memcpy(v + 8, &bi, 4);
            memcpy(v + 12, &bo, 4);
            data.insert(data.end(), r.values + a, r.values + b);
        }
    }
    const int64_t dlen = (int64_t)data.size();
    if (data.empty()) data.push_back(0);
    std::vector<uint8_t> sizes(8);
    memcpy(sizes.data(), &dlen, 8);
    std::vector<uint8_t> vb;
    if (r.null_count) vb.assign(r.validity, r.validity + (r.n + 7) / 8);
    c.bufs.push_back(std::move(vb));
    c.bufs.push_back(std::move(views));
    c.bufs.push_back(std::move(data));
    c.bufs.push_back(std::move(sizes));
    return c;
}

// Run one op over the zipped inputs (the shortest input wins, as `.zip()`; the aligned
// exprs broadcast a 1-row reference, expressions.rs:344-349).
struct StrResultHolder {
    rogtk_str_result r{};
    ~StrResultHolder() { rogtk_str_result_free(&r); }
};
void str_transform(int op, SeriesExport* in, size_t n_in, size_t need, int64_t param, StrResultHolder* out,
                   std::string* name) {
    if (n_in < need) fail("expected %zu input series, got %zu", need, n_in);
    std::vector<FlatCol> cols;
    for (size_t k = 0; k < need; ++k) cols.push_back(flatten_all(str_series(in[k])));
    *name = str_series(in[0]).name;
    const bool aligned = op == ROGTK_STR_ALIGNED_REF || op == ROGTK_STR_ALIGNED_QUERY;
    const bool scalar_ref = aligned && cols[0].n == 1 && cols[1].n > 1;
    int64_t n = INT64_MAX;
    for (size_t k = scalar_ref ? 1 : 0; k < need; ++k) n = std::min(n, cols[k].n);
    std::vector<rogtk_str_col> d;
    for (size_t k = 0; k < need; ++k) {
        rogtk_str_col c = str_desc(cols[k]);
        if (!(scalar_ref && k == 0)) c.n = n;  // zip: rows past the shortest input are dropped
        d.push_back(c);
    }
    check(rogtk_str_transform_host(op, d.data(), (int)need, n, param, &out->r));
}

// reverse_complement_series, parse_cigar_series, cigar_aligned_*_expr,
// extract_cigar_insertions_expr, enrich_allele_insertions_expr, phred_to_numeric_series_str
void string_expr(SeriesExport* in, size_t n_in, SeriesExport* out, int op, size_t need, int64_t param) {
    StrResultHolder h;
    std::string name;
    str_transform(op, in, n_in, need, param, &h, &name);
    std::vector<Col> chunks;
    chunks.push_back(view_col_result(h.r));
    export_series(out, {name, "vu", {}}, std::move(chunks));
}

// phred_to_numeric_series (expressions.rs:598-630): List[UInt8] named "numeric_phred";
// `ca.for_each` appends nothing for null rows, so they are dropped from the output.
void phred_list_expr(SeriesExport* in, size_t n_in, SeriesExport* out, int64_t base) {
    StrResultHolder h;
    std::string name;
    str_transform(ROGTK_STR_PHRED_LIST, in, n_in, 1, base, &h, &name);
    const rogtk_str_result& r = h.r;
    std::vector<int64_t> loff{0};
    std::vector<uint8_t> vals;
    for (int64_t i = 0; i < r.n; ++i) {
        if (!((r.validity[i >> 3] >> (i & 7)) & 1)) continue;
        vals.insert(vals.end(), r.values + r.offsets[i], r.values + r.offsets[i + 1]);
        loff.push_back((int64_t)vals.size());
    }
    const int64_t m = (int64_t)loff.size() - 1;
    Col child = prim_col<uint8_t>({}, 0, std::move(vals), (int64_t)loff.back());
    Col list;
    list.length = m;
    list.bufs.push_back({});
    std::vector<uint8_t> ob(loff.size() * 8);
    memcpy(ob.data(), loff.data(), ob.size());
    list.bufs.push_back(std::move(ob));
    list.children.push_back(std::move(child));
    std::vector<Col> chunks;
    chunks.push_back(std::move(list));
    export_series(out, {"numeric_phred", "+L", {{"item", "C", {}}}}, std::move(chunks));
}

int64_t phred_base(const Kwargs& kw) {
    const int64_t b = kw.uint("base");  // Phred2NmKwargs.base: u8 (expressions.rs:493-496)
    if (b > 255) fail("could not parse kwargs: base does not fit in u8");
    return b;
}

// ----------------------------------------------------------- entry wrappers
template <class F>
void guarded(SeriesExport* in, size_t n_in, SeriesExport* out, F&& f) {
    try {
        f();
    } catch (const std::exception& e) {
        t_plugin_err = e.what();
        if (out && out->release) out->release(out);
        if (out) *out = SeriesExport{};
    } catch (...) {
        t_plugin_err = "unknown error";
        if (out) *out = SeriesExport{};
    }
    try {
        release_inputs(in, n_in);
    } catch (...) {
    }
}

std::string input_name(const ArrowSchema* fields, size_t n) {
    if (n == 0 || !fields) fail("expected at least one input field");
    return fields[0].name ? fields[0].name : "";
}

template <class F>
void guarded_field(ArrowSchema* out, F&& f) {
    try {
        FieldSpec spec = f();
        fill_schema(out, spec);
    } catch (const std::exception& e) {
        t_plugin_err = e.what();
        if (out) *out = ArrowSchema{};
    }
}

}  // namespace

// ====================================================================== ABI
extern "C" {

__attribute__((visibility("default"))) uint32_t _polars_plugin_get_version(void) {
    // polars-ffi get_version() = (0, 1), packed (major << 16) + minor as pyo3-polars does
    return (0u << 16) + 1u;
}

__attribute__((visibility("default"))) const char* _polars_plugin_get_last_error_message(void) {
    return t_plugin_err.c_str();
}

// Diagnostics (include/rogtk_hip.h): the kwargs as this library parses them, rendered
// one "key=value" per line in key order (None / True / False / integers / 'strings' /
// floats with 17 significant digits / [lists]); lets the pickle reader be tested on CPU.
static void render(const PVal& v, std::string* o) {
    char b[64];
    switch (v.kind) {
        case PVal::NONE: *o += "None"; break;
        case PVal::BOOL: *o += v.b ? "True" : "False"; break;
        case PVal::INT: snprintf(b, sizeof b, "%lld", (long long)v.i); *o += b; break;
        case PVal::FLOAT: snprintf(b, sizeof b, "%.17g", v.f); *o += b; break;
        case PVal::STR: *o += "'" + v.s + "'"; break;
        case PVal::LIST:
            *o += "[";
            for (size_t j = 0; j < v.items.size(); ++j) {
                if (j) *o += ", ";
                render(*v.items[j], o);
            }
            *o += "]";
            break;
        default: *o += "?"; break;
    }
}

__attribute__((visibility("default"))) int rogtk_plugin_kwargs_debug(const uint8_t* kwargs, int64_t len,
                                                                      char* out, int64_t cap, int64_t* out_len) {
    try {
        Kwargs kw = parse_kwargs(kwargs, (size_t)std::max<int64_t>(len, 0));
        std::string o;
        for (auto& kv : kw.m) {
            o += kv.first + "=";
            render(*kv.second, &o);
            o += "\n";
        }
        if (out_len) *out_len = (int64_t)o.size();
        if ((int64_t)o.size() > cap) {
            t_plugin_err = "output larger than cap";
            return ROGTK_E_OVERFLOW;
        }
        if (out && !o.empty()) memcpy(out, o.data(), o.size());
        return ROGTK_OK;
    } catch (const std::exception& e) {
        t_plugin_err = e.what();
        return ROGTK_E_INVALID;
    }
}

#define ROGTK_EXPR(NAME, BODY)                                                                            \
    __attribute__((visibility("default"))) void _polars_plugin_##NAME(                                    \
        SeriesExport* inputs, size_t n_inputs, const uint8_t* kwargs_ptr, size_t kwargs_len,            \
        SeriesExport* return_value, CallerContext* /*context*/) {                                          \
        guarded(inputs, n_inputs, return_value, [&] {                                                     \
            (void)kwargs_ptr;                                                                              \
            (void)kwargs_len;                                                                              \
            BODY;                                                                                          \
        });                                                                                                \
    }
#define ROGTK_FIELD(NAME, SPEC)                                                                           \
    __attribute__((visibility("default"))) void _polars_plugin_field_##NAME(                              \
        ArrowSchema* fields, size_t n_fields, ArrowSchema* return_value, const uint8_t* /*kwargs_ptr*/,   \
        size_t /*kwargs_len*/) {                                                                           \
        guarded_field(return_value, [&]() -> FieldSpec {                                                  \
            const std::string name = input_name(fields, n_fields);                                         \
            return SPEC;                                                                                   \
        });                                                                                                \
    }

// H1 (expressions.rs:1219-1410)
ROGTK_EXPR(umi_complexity_all_expr, umi_complexity(inputs, n_inputs, return_value, -1))
ROGTK_FIELD(umi_complexity_all_expr, complexity_struct(name))
ROGTK_EXPR(umi_shannon_entropy_expr, umi_complexity(inputs, n_inputs, return_value, 0))
ROGTK_FIELD(umi_shannon_entropy_expr, (FieldSpec{name, "g", {}}))
ROGTK_EXPR(umi_linguistic_complexity_expr, umi_complexity(inputs, n_inputs, return_value, 1))
ROGTK_FIELD(umi_linguistic_complexity_expr, (FieldSpec{name, "g", {}}))
ROGTK_EXPR(umi_homopolymer_fraction_expr, umi_complexity(inputs, n_inputs, return_value, 2))
ROGTK_FIELD(umi_homopolymer_fraction_expr, (FieldSpec{name, "g", {}}))
ROGTK_EXPR(umi_dinucleotide_entropy_expr, umi_complexity(inputs, n_inputs, return_value, 3))
ROGTK_FIELD(umi_dinucleotide_entropy_expr, (FieldSpec{name, "g", {}}))
ROGTK_EXPR(umi_longest_homopolymer_expr, umi_complexity(inputs, n_inputs, return_value, 4))
ROGTK_FIELD(umi_longest_homopolymer_expr, (FieldSpec{name, "I", {}}))
ROGTK_EXPR(umi_dust_score_expr, umi_complexity(inputs, n_inputs, return_value, 5))
ROGTK_FIELD(umi_dust_score_expr, (FieldSpec{name, "g", {}}))
ROGTK_EXPR(umi_combined_score_expr, umi_complexity(inputs, n_inputs, return_value, 6))
ROGTK_FIELD(umi_combined_score_expr, (FieldSpec{name, "g", {}}))

// H2 (expressions.rs:1048-1101)
ROGTK_EXPR(hamming_distance_expr,
           hamming(inputs, n_inputs, parse_kwargs(kwargs_ptr, kwargs_len), return_value, false))
ROGTK_FIELD(hamming_distance_expr, (FieldSpec{name, "I", {}}))
ROGTK_EXPR(hamming_within_expr,
           hamming(inputs, n_inputs, parse_kwargs(kwargs_ptr, kwargs_len), return_value, true))
ROGTK_FIELD(hamming_within_expr, (FieldSpec{name, "b", {}}))

// H4/H5 (expressions.rs:695-955, fracture_opt.rs:283-367)
ROGTK_EXPR(assemble_sequences_expr,
           assemble(inputs, n_inputs, parse_kwargs(kwargs_ptr, kwargs_len), return_value, false))
ROGTK_FIELD(assemble_sequences_expr, (FieldSpec{name, "vu", {}}))
ROGTK_EXPR(assemble_sequences_with_anchors_expr,
           assemble(inputs, n_inputs, parse_kwargs(kwargs_ptr, kwargs_len), return_value, true))
ROGTK_FIELD(assemble_sequences_with_anchors_expr, (FieldSpec{name, "vu", {}}))
ROGTK_EXPR(sweep_assembly_params_expr, sweep(inputs, n_inputs, parse_kwargs(kwargs_ptr, kwargs_len), return_value))
ROGTK_FIELD(sweep_assembly_params_expr,
            (FieldSpec{name, "+s", {{"k", "l", {}}, {"min_coverage", "l", {}}, {"contig_length", "l", {}}}}))
ROGTK_EXPR(optimize_assembly_expr, optimize(inputs, n_inputs, parse_kwargs(kwargs_ptr, kwargs_len), return_value))
ROGTK_FIELD(optimize_assembly_expr, optimize_struct(name))

// element-wise string expressions (expressions.rs:29-665, 957-977)
ROGTK_EXPR(reverse_complement_series, string_expr(inputs, n_inputs, return_value, ROGTK_STR_REVCOMP, 1, 0))
ROGTK_FIELD(reverse_complement_series, (FieldSpec{name, "vu", {}}))
ROGTK_EXPR(parse_cigar_series,
           string_expr(inputs, n_inputs, return_value, ROGTK_STR_PARSE_CIGAR, 1,
                       parse_kwargs(kwargs_ptr, kwargs_len).uint("block_dels") != 0))
ROGTK_FIELD(parse_cigar_series, (FieldSpec{name, "vu", {}}))
ROGTK_EXPR(cigar_aligned_ref_expr, string_expr(inputs, n_inputs, return_value, ROGTK_STR_ALIGNED_REF, 3, 0))
ROGTK_FIELD(cigar_aligned_ref_expr, (FieldSpec{name, "vu", {}}))
ROGTK_EXPR(cigar_aligned_query_expr, string_expr(inputs, n_inputs, return_value, ROGTK_STR_ALIGNED_QUERY, 3, 0))
ROGTK_FIELD(cigar_aligned_query_expr, (FieldSpec{name, "vu", {}}))
ROGTK_EXPR(extract_cigar_insertions_expr,
           string_expr(inputs, n_inputs, return_value, ROGTK_STR_CIGAR_INSERTIONS, 2, 0))
ROGTK_FIELD(extract_cigar_insertions_expr, (FieldSpec{name, "vu", {}}))
ROGTK_EXPR(enrich_allele_insertions_expr,
           string_expr(inputs, n_inputs, return_value, ROGTK_STR_ENRICH_ALLELE, 3, 0))
ROGTK_FIELD(enrich_allele_insertions_expr, (FieldSpec{name, "vu", {}}))
ROGTK_EXPR(phred_to_numeric_series_str,
           string_expr(inputs, n_inputs, return_value, ROGTK_STR_PHRED_STR, 1,
                       phred_base(parse_kwargs(kwargs_ptr, kwargs_len))))
ROGTK_FIELD(phred_to_numeric_series_str, (FieldSpec{name, "vu", {}}))
ROGTK_EXPR(phred_to_numeric_series,
           phred_list_expr(inputs, n_inputs, return_value, phred_base(parse_kwargs(kwargs_ptr, kwargs_len))))
ROGTK_FIELD(phred_to_numeric_series, (FieldSpec{name, "+L", {{"item", "C", {}}}}))

}  // extern "C"
