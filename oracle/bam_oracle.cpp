// TEST INFRASTRUCTURE ONLY — C++ restatement of rogtk's BAM record -> row loop, the
// CPU baseline of config C5 and a second checker (beside oracle/pybam.py) for
// rogtk_amd/csrc/bam.hip. Single-threaded like the reference's per-record loop:
// gzread (concatenated BGZF members) + per record the row fields of
//   mode 0 noodles       extract_record_data_enhanced      src/bam.rs:170-262
//   mode 1 htslib        process_htslib_records_to_batch   src/bam.rs:3028-3148
//   mode 2 htslib_blocks process_htslib_records_to_batch   src/bam_htslib.rs:154-241
// built into std::string buffers (the reference builds Strings per field), reduced to
// an FNV-1a digest per column so callers can compare without materialising rows.
#include <zlib.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

void lossy(const uint8_t* p, int n, std::string* out) {
    out->clear();
    int i = 0;
    while (i < n) {
        const uint8_t b = p[i];
        if (b < 0x80) {
            out->push_back((char)b);
            ++i;
            continue;
        }
        int need = 0;
        uint8_t lo = 0x80, hi = 0xBF;
        if (b >= 0xC2 && b <= 0xDF) need = 1;
        else if (b == 0xE0) need = 2, lo = 0xA0;
        else if ((b >= 0xE1 && b <= 0xEC) || b == 0xEE || b == 0xEF) need = 2;
        else if (b == 0xED) need = 2, hi = 0x9F;
        else if (b == 0xF0) need = 3, lo = 0x90;
        else if (b >= 0xF1 && b <= 0xF3) need = 3;
        else if (b == 0xF4) need = 3, hi = 0x8F;
        int j = i + 1, got = 0;
        for (; need && got < need && j < n; ++got, ++j) {
            const uint8_t c = p[j];
            if (c < (got == 0 ? lo : 0x80) || c > (got == 0 ? hi : 0xBF)) break;
        }
        if (need && got == need) out->append((const char*)p + i, j - i);
        else out->append("\xEF\xBF\xBD");
        i = j;
    }
}

}  // namespace

extern "C" {

// Decodes every record; digests[7] = FNV-1a over (name, chrom, start, end, flags,
// sequence, quality) with a per-row null marker. Returns the record count, -1 on error.
int64_t oracle_bam_digest(const char* path, int mode, uint64_t* digests) {
    gzFile f = gzopen(path, "rb");
    if (!f) return -1;
    gzbuffer(f, 1 << 20);
    std::vector<uint8_t> buf(1 << 16);
    auto rd = [&](void* dst, size_t n) { return gzread(f, dst, (unsigned)n) == (int)n; };
    char magic[4];
    int32_t l_text, n_ref;
    if (!rd(magic, 4) || memcmp(magic, "BAM\1", 4) || !rd(&l_text, 4)) return gzclose(f), -1;
    std::vector<uint8_t> tmp(l_text > 0 ? l_text : 1);
    if (l_text > 0 && !rd(tmp.data(), l_text)) return gzclose(f), -1;
    if (!rd(&n_ref, 4)) return gzclose(f), -1;
    std::vector<std::string> refs(n_ref);
    for (int32_t i = 0; i < n_ref; ++i) {
        int32_t ln, lr;
        if (!rd(&ln, 4) || ln < 1) return gzclose(f), -1;
        std::vector<uint8_t> nm(ln);
        if (!rd(nm.data(), ln) || !rd(&lr, 4)) return gzclose(f), -1;
        lossy(nm.data(), ln - 1, &refs[i]);
    }
    uint64_t d[7];
    for (auto& x : d) x = 1469598103934665603ull;
    const char* nt16 = "=ACMGRSVTWYHKDBN";
    std::string name, seq, qual;
    int64_t count = 0;
    for (;;) {
        uint32_t bs;
        const int got = gzread(f, &bs, 4);
        if (got == 0) break;
        if (got != 4 || bs < 32) return gzclose(f), -1;
        if (buf.size() < bs) buf.resize(bs);
        if (!rd(buf.data(), bs)) return gzclose(f), -1;
        const uint8_t* b = buf.data();
        int32_t ref_id, pos;
        uint16_t n_cig, flag;
        uint32_t l_seq;
        memcpy(&ref_id, b, 4);
        memcpy(&pos, b + 4, 4);
        const uint32_t l_name = b[8];
        memcpy(&n_cig, b + 12, 2);
        memcpy(&flag, b + 14, 2);
        memcpy(&l_seq, b + 16, 4);
        const uint8_t* nm = b + 32;
        const uint8_t* cg = nm + l_name;
        const uint8_t* sq = cg + 4 * n_cig;
        const uint8_t* ql = sq + (l_seq + 1) / 2;
        uint32_t rlen = 0;
        for (uint32_t k = 0; k < n_cig; ++k) {
            uint32_t op;
            memcpy(&op, cg + 4 * k, 4);
            const uint32_t kind = op & 15;
            if (kind == 0 || kind == 2 || kind == 3 || kind == 7 || kind == 8) rlen += op >> 4;
        }
        if (mode == 0 && (l_name == 0 || (l_name == 2 && nm[0] == '*'))) name = "unknown";
        else lossy(nm, l_name ? (int)l_name - 1 : 0, &name);
        const bool has_chrom = ref_id >= 0 && ref_id < n_ref;
        bool vs = false, ve = false;
        uint32_t start = 0, end = 0;
        if (mode == 1) {
            vs = ve = pos >= 0;
            start = (uint32_t)pos + 1;
            end = start + l_seq - 1;
        } else if (mode == 0) {
            vs = ve = pos >= 0;
            start = (uint32_t)pos + 1;
            end = start + rlen - 1;
        } else {
            vs = pos >= 0;
            start = (uint32_t)pos;
            const int64_t re = (!(flag & 4) && n_cig > 0) ? (int64_t)pos + rlen : (int64_t)pos + 1;
            if (re > pos) ve = true, end = (uint32_t)re;
            else ve = vs, end = start;
        }
        seq.resize(l_seq);
        for (uint32_t i = 0; i < l_seq; ++i) {
            const uint32_t nib = (i & 1) ? (sq[i >> 1] & 15) : (sq[i >> 1] >> 4);
            if (mode == 2) seq[i] = nt16[nib];
            else seq[i] = nib == 1 ? 'A' : nib == 2 ? 'C' : nib == 4 ? 'G' : nib == 8 ? 'T' : 'N';
        }
        const bool vq = l_seq > 0 && !(mode == 1 && ql[0] == 0xFF);
        qual.resize(vq ? l_seq : 0);
        for (uint32_t i = 0; vq && i < l_seq; ++i) qual[i] = (char)(uint8_t)(ql[i] + 33);
        const uint8_t nul = 0xFF, one = 1;
        d[0] = fnv(fnv(d[0], name.data(), name.size()), &one, 1);
        d[1] = has_chrom ? fnv(fnv(d[1], refs[ref_id].data(), refs[ref_id].size()), &one, 1) : fnv(d[1], &nul, 1);
        d[2] = vs ? fnv(fnv(d[2], &start, 4), &one, 1) : fnv(d[2], &nul, 1);
        d[3] = ve ? fnv(fnv(d[3], &end, 4), &one, 1) : fnv(d[3], &nul, 1);
        const uint32_t fl = flag;
        d[4] = fnv(d[4], &fl, 4);
        d[5] = l_seq ? fnv(fnv(d[5], seq.data(), seq.size()), &one, 1) : fnv(d[5], &nul, 1);
        d[6] = vq ? fnv(fnv(d[6], qual.data(), qual.size()), &one, 1) : fnv(d[6], &nul, 1);
        ++count;
    }
    gzclose(f);
    memcpy(digests, d, sizeof d);
    return count;
}

}  // extern "C"
