// fastq.cpp — paired FASTQ ingest (host C++, zlib): the producer side of the hot
// path. Restates parse_paired_fastqs (src/lib.rs:232-428)
// line for line, but emits Arrow string columns in memory (the caller stages the
// UMI column to HBM, or writes the reference's Parquet file from them):
//   lib.rs:246-252  MultiGzDecoder + BufReader::lines() + filter_map(Result::ok):
//                   lines split on '\n', a trailing '\r' dropped, a last line
//                   without '\n' kept, lines that are not valid UTF-8 skipped
//                   (gzread also reads plain text and concatenated gzip members)
//   lib.rs:286-294  limit = number of LINES taken from each file
//   lib.rs:306-310  records = chunks(4) of each file's lines, zipped pairwise
//   lib.rs:312-330  read_id = line0.trim_start_matches('@').trim_end();
//                   cbc = seq1[0..cbc_len], umi = seq1[cbc_len..cbc_len+umi_len]
//                   (and the same slices of qual1): a range outside the line or
//                   off a char boundary is the reference's panic -> an error here;
//                   seq / qual of R2 = trim_end(), reverse-complemented / reversed
//                   per char when do_rev_comp (A<->T, C<->G, N, others unchanged)
//   lib.rs:332-333  start = "0", end = "1"
// Column order = the reference schema (lib.rs:258-268).
#include <zlib.h>

#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rogtk_internal.h"

namespace rogtk {
namespace {

// Rust str::from_utf8 acceptance (no overlongs, no surrogates, <= U+10FFFF)
bool valid_utf8(const unsigned char* s, size_t n) {
    size_t i = 0;
    while (i < n) {
        const unsigned char c = s[i];
        if (c < 0x80) {
            ++i;
            continue;
        }
        size_t w;
        unsigned lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) w = 2;
        else if (c == 0xE0) { w = 3; lo = 0xA0; }
        else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) w = 3;
        else if (c == 0xED) { w = 3; hi = 0x9F; }
        else if (c == 0xF0) { w = 4; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) w = 4;
        else if (c == 0xF4) { w = 4; hi = 0x8F; }
        else return false;
        if (i + w > n) return false;
        if (s[i + 1] < lo || s[i + 1] > hi) return false;
        for (size_t k = 2; k < w; ++k)
            if (s[i + k] < 0x80 || s[i + k] > 0xBF) return false;
        i += w;
    }
    return true;
}

// decode the UTF-8 scalar that ends at s[end-1]; returns its start
size_t prev_char(const std::string& s, size_t end, uint32_t* cp) {
    size_t st = end - 1;
    while (st > 0 && (static_cast<unsigned char>(s[st]) & 0xC0) == 0x80) --st;
    const unsigned char c = static_cast<unsigned char>(s[st]);
    uint32_t v = c < 0x80 ? c : c < 0xE0 ? (c & 0x1F) : c < 0xF0 ? (c & 0x0F) : (c & 0x07);
    for (size_t k = st + 1; k < end; ++k) v = (v << 6) | (static_cast<unsigned char>(s[k]) & 0x3F);
    *cp = v;
    return st;
}

bool rust_whitespace(uint32_t c) {  // char::is_whitespace (White_Space)
    return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
           (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F ||
           c == 0x3000;
}

std::string trim_end(const std::string& s) {
    size_t end = s.size();
    while (end > 0) {
        uint32_t cp;
        const size_t st = prev_char(s, end, &cp);
        if (!rust_whitespace(cp)) break;
        end = st;
    }
    return s.substr(0, end);
}

bool char_boundary(const std::string& s, size_t i) {
    return i == 0 || i == s.size() || (i < s.size() && (static_cast<unsigned char>(s[i]) & 0xC0) != 0x80);
}

// chars of s in reverse order (optionally complemented)
std::string reverse_chars(const std::string& s, bool complement) {
    std::string out;
    out.reserve(s.size());
    size_t end = s.size();
    while (end > 0) {
        uint32_t cp;
        const size_t st = prev_char(s, end, &cp);
        if (complement && end - st == 1) {
            char c = s[st];
            switch (c) {
                case 'A': c = 'T'; break;
                case 'T': c = 'A'; break;
                case 'C': c = 'G'; break;
                case 'G': c = 'C'; break;
                default: break;  // 'N' and anything else unchanged
            }
            out.push_back(c);
        } else {
            out.append(s, st, end - st);
        }
        end = st;
    }
    return out;
}

// One FASTQ stream: BufReader::lines() over a gzip (or plain) file.
struct LineReader {
    gzFile f = nullptr;
    std::vector<char> buf = std::vector<char>(1 << 22);
    size_t pos = 0, len = 0;
    bool eof = false;
    int64_t remaining = -1;  // lines still allowed by `limit` (-1: unlimited)
    std::string err;

    bool fill() {
        if (eof) return false;
        const int r = gzread(f, buf.data(), (unsigned)buf.size());
        if (r < 0) {
            int e = 0;
            err = gzerror(f, &e);
            eof = true;
            return false;
        }
        if (r == 0) {
            eof = true;
            return false;
        }
        pos = 0;
        len = (size_t)r;
        return true;
    }
    // next valid-UTF-8 line (Result::ok filter), false at the end. Like
    // BufRead::lines(): a '\r' is dropped only before a '\n'; an unterminated last
    // line is returned as is; an empty unterminated tail is the end.
    bool next(std::string* line) {
        if (remaining == 0) return false;
        for (;;) {
            line->clear();
            bool any = false, nl_found = false;
            for (;;) {
                if (pos >= len && !fill()) break;
                any = true;
                const char* base = buf.data() + pos;
                const char* nl = static_cast<const char*>(memchr(base, '\n', len - pos));
                if (nl) {
                    line->append(base, (size_t)(nl - base));
                    pos += (size_t)(nl - base) + 1;
                    nl_found = true;
                    break;
                }
                line->append(base, len - pos);
                pos = len;
            }
            if (!nl_found && (!any || line->empty())) return false;
            if (nl_found && !line->empty() && line->back() == '\r') line->pop_back();
            if (!valid_utf8(reinterpret_cast<const unsigned char*>(line->data()), line->size())) continue;
            if (remaining > 0) --remaining;
            return true;
        }
    }
    // up to n lines
    void take(int64_t n, std::vector<std::string>* out) {
        out->clear();
        std::string l;
        while ((int64_t)out->size() < n && next(&l)) out->push_back(l);
    }
};

struct Column {
    std::vector<int64_t> off{0};
    std::vector<uint8_t> val;
    void clear() {
        off.assign(1, 0);
        val.clear();
    }
    void push(const std::string& s) {
        val.insert(val.end(), s.begin(), s.end());
        off.push_back((int64_t)val.size());
    }
};

struct PairReader {
    LineReader r1, r2;
    int64_t cbc_len = 0, umi_len = 0;
    bool rev = false, done = false;
    Column cols[9];
    std::vector<uint8_t> dummy{0};
};

}  // namespace
}  // namespace rogtk

using namespace rogtk;

extern "C" {

int rogtk_fastq_pair_open(const char* r1, const char* r2, int64_t cbc_len, int64_t umi_len, int64_t limit_lines,
                          int do_rev_comp, void** reader) {
    ROGTK_REQUIRE(r1 && r2 && reader, ROGTK_E_INVALID, "fastq: NULL argument");
    ROGTK_REQUIRE(cbc_len >= 0 && umi_len >= 0, ROGTK_E_INVALID, "fastq: cbc_len / umi_len must be >= 0");
    auto* p = new PairReader();
    p->r1.f = gzopen(r1, "rb");
    p->r2.f = gzopen(r2, "rb");
    if (!p->r1.f || !p->r2.f) {
        const bool first = !p->r1.f;
        if (p->r1.f) gzclose(p->r1.f);
        if (p->r2.f) gzclose(p->r2.f);
        delete p;
        set_error("fastq: cannot open %s", first ? r1 : r2);
        return ROGTK_E_INVALID;
    }
    gzbuffer(p->r1.f, 1 << 20);
    gzbuffer(p->r2.f, 1 << 20);
    p->r1.remaining = p->r2.remaining = limit_lines < 0 ? -1 : limit_lines;
    p->cbc_len = cbc_len;
    p->umi_len = umi_len;
    p->rev = do_rev_comp != 0;
    *reader = p;
    return ROGTK_OK;
}

/* Next batch of at most max_records records: 9 columns (read_id, start, end, cbc,
 * umi, cbc_qual, umi_qual, seq, qual). The buffers belong to the reader and stay
 * valid until the next call / close. n_records = 0 at the end. */
int rogtk_fastq_pair_next(void* reader, int64_t max_records, int64_t* n_records, const int64_t** offsets9,
                          const uint8_t** values9) {
    ROGTK_REQUIRE(reader && n_records && offsets9 && values9, ROGTK_E_INVALID, "fastq: NULL argument");
    ROGTK_REQUIRE(max_records > 0, ROGTK_E_INVALID, "fastq: max_records must be > 0");
    auto* p = static_cast<PairReader*>(reader);
    for (auto& c : p->cols) c.clear();
    *n_records = 0;
    if (!p->done) {
        // decode both files concurrently (zlib is the bottleneck)
        std::vector<std::string> l1, l2;
        std::thread t([&] { p->r1.take(4 * max_records, &l1); });
        p->r2.take(4 * max_records, &l2);
        t.join();
        ROGTK_REQUIRE(p->r1.err.empty() && p->r2.err.empty(), ROGTK_E_INVALID, "fastq: gzip error: %s",
                      (p->r1.err + p->r2.err).c_str());
        if ((int64_t)l1.size() < 4 * max_records || (int64_t)l2.size() < 4 * max_records) p->done = true;
        const size_t nch = std::min((l1.size() + 3) / 4, (l2.size() + 3) / 4);  // zip of chunks(4)
        for (size_t c = 0; c < nch; ++c) {
            ROGTK_REQUIRE(4 * c + 3 < l1.size() && 4 * c + 3 < l2.size(), ROGTK_E_INVALID,
                          "fastq: truncated record (a chunk of fewer than 4 lines)");
            const std::string &id1 = l1[4 * c], &seq1 = l1[4 * c + 1], &qual1 = l1[4 * c + 3];
            const std::string &seq2 = l2[4 * c + 1], &qual2 = l2[4 * c + 3];
            size_t a = 0;
            while (a < id1.size() && id1[a] == '@') ++a;
            const std::string rid = trim_end(id1.substr(a));
            const size_t cb = (size_t)p->cbc_len, ue = (size_t)(p->cbc_len + p->umi_len);
            for (const std::string* s : {&seq1, &qual1}) {
                ROGTK_REQUIRE(ue <= s->size() && char_boundary(*s, cb) && char_boundary(*s, ue), ROGTK_E_INVALID,
                              "fastq: invalid range of string (read %lld shorter than cbc_len + umi_len)",
                              (long long)(*n_records + 1));
            }
            p->cols[0].push(rid);
            p->cols[1].push("0");
            p->cols[2].push("1");
            p->cols[3].push(seq1.substr(0, cb));
            p->cols[4].push(seq1.substr(cb, ue - cb));
            p->cols[5].push(qual1.substr(0, cb));
            p->cols[6].push(qual1.substr(cb, ue - cb));
            const std::string s2 = trim_end(seq2), q2 = trim_end(qual2);
            p->cols[7].push(p->rev ? reverse_chars(s2, true) : s2);
            p->cols[8].push(p->rev ? reverse_chars(q2, false) : q2);
            ++*n_records;
        }
    }
    for (int i = 0; i < 9; ++i) {
        offsets9[i] = p->cols[i].off.data();
        values9[i] = p->cols[i].val.empty() ? p->dummy.data() : p->cols[i].val.data();
    }
    return ROGTK_OK;
}

int rogtk_fastq_pair_close(void* reader) {
    if (!reader) return ROGTK_OK;
    auto* p = static_cast<PairReader*>(reader);
    if (p->r1.f) gzclose(p->r1.f);
    if (p->r2.f) gzclose(p->r2.f);
    delete p;
    return ROGTK_OK;
}

}  // extern "C"
