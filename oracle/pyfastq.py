"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of parse_paired_fastqs
(src/lib.rs:232-428) for checking rogtk_amd/csrc/fastq.cpp.

MultiGzDecoder + BufReader::lines() + filter_map(Result::ok) (lib.rs:246-252),
take(limit) lines (:286-294), chunks(4) zipped (:306-310), the field slices and
trims of :312-330, start "0" / end "1" (:332-333). A Rust panic is a ValueError.
"""
from __future__ import annotations

import gzip

_WS = set(range(0x09, 0x0E)) | {0x20, 0x85, 0xA0, 0x1680, 0x2028, 0x2029, 0x202F, 0x205F, 0x3000} | set(
    range(0x2000, 0x200B))


def _lines(path):
    with open(path, "rb") as f:
        raw = f.read()
    data = gzip.decompress(raw) if raw[:2] == b"\x1f\x8b" else raw
    out = []
    for k, seg in enumerate(data.split(b"\n")):
        last = k == data.count(b"\n")
        if last and seg == b"":
            break
        if not last and seg.endswith(b"\r"):
            seg = seg[:-1]
        try:
            out.append(seg.decode("utf-8"))
        except UnicodeDecodeError:
            continue  # Result::ok filter
    return out


def _trim_end(s: str) -> str:
    while s and ord(s[-1]) in _WS:
        s = s[:-1]
    return s


def _slice(s: str, a: int, b: int) -> str:
    bs = s.encode("utf-8")
    if b > len(bs):
        raise ValueError("invalid range of string")
    try:
        return bs[a:b].decode("utf-8") if a <= b else ""
    except UnicodeDecodeError:
        raise ValueError("invalid range of string")


def _check_boundary(s: str, i: int):
    bs = s.encode("utf-8")
    if 0 < i < len(bs) and (bs[i] & 0xC0) == 0x80:
        raise ValueError("invalid range of string")


def _rc(s: str) -> str:
    m = {"A": "T", "T": "A", "C": "G", "G": "C", "N": "N"}
    return "".join(m.get(c, c) for c in reversed(s))


def parse(fn1, fn2, cbc_len, umi_len, limit=None, do_rev_comp=False):
    l1, l2 = _lines(fn1), _lines(fn2)
    if limit is not None:
        l1, l2 = l1[:limit], l2[:limit]
    rows = []
    nch = min((len(l1) + 3) // 4, (len(l2) + 3) // 4)
    for c in range(nch):
        ch1, ch2 = l1[4 * c:4 * c + 4], l2[4 * c:4 * c + 4]
        if len(ch1) < 4 or len(ch2) < 4:
            raise ValueError("truncated record")
        rid = _trim_end(ch1[0].lstrip("@"))
        seq1, qual1 = ch1[1], ch1[3]
        for s in (seq1, qual1):
            for i in (cbc_len, cbc_len + umi_len):
                _check_boundary(s, i)
        cbc, umi = _slice(seq1, 0, cbc_len), _slice(seq1, cbc_len, cbc_len + umi_len)
        cq, uq = _slice(qual1, 0, cbc_len), _slice(qual1, cbc_len, cbc_len + umi_len)
        s2, q2 = _trim_end(ch2[1]), _trim_end(ch2[3])
        if do_rev_comp:
            s2, q2 = _rc(s2), q2[::-1]
        rows.append((rid, "0", "1", cbc, umi, cq, uq, s2, q2))
    return rows
