"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of rogtk's BAM record -> row
conversion, for checking rogtk_amd/csrc/bam.hip.

The container format is SAMv1 §4 (BGZF = concatenated gzip members, decoded here with
Python's gzip; header: magic, l_text, text, n_ref, references; records: block_size +
fixed fields + read_name + cigar + 4-bit seq + qual + tags). Row semantics:

  mode "noodles"       extract_record_data_enhanced, src/bam.rs:170-262 (noodles 0.82:
                       name "*" -> missing -> "unknown"; refID/pos -1 -> None; 1-based
                       start; end = start + CIGAR ref length (M/D/N/=/X) - 1,
                       calculate_bam_alignment_length bam.rs:3238-3256; decode_base
                       :3227-3236; quality + 33 per byte)
  mode "htslib"        process_htslib_records_to_batch, src/bam.rs:3028-3148 (1-based
                       start, end = start + seq_len - 1, quality null when empty or
                       qual[0] == 0xFF, quality_to_string_zero_copy :2622-2636)
  mode "htslib_blocks" process_htslib_records_to_batch, src/bam_htslib.rs:154-241
                       (start = pos 0-based; end = bam_endpos if > pos else start, with
                       htslib bam_endpos = pos + cigar2rlen for mapped reads with a
                       CIGAR, else pos + 1; bases via seq_nt16_str "=ACMGRSVTWYHKDBN")

Names and reference names are String::from_utf8_lossy (Python's errors="replace" applies
the same maximal-subpart rule). Crate-internal choices not visible in the reference
(noodles' "*" name, its handling of 0xFF qualities) are restated as documented there and
are parity-unpinned beyond this restatement.
"""
from __future__ import annotations

import gzip
import struct
from typing import Dict, List, Optional

_DECODE = {1: "A", 2: "C", 4: "G", 8: "T", 15: "N"}
_NT16 = "=ACMGRSVTWYHKDBN"


def _lossy(b: bytes) -> str:
    return b.decode("utf-8", errors="replace")


def read_bam(path: str):
    """(reference names, list of raw record bodies) of a BAM file."""
    with open(path, "rb") as f:
        data = gzip.decompress(f.read())
    assert data[:4] == b"BAM\x01", "bad magic"
    l_text = struct.unpack_from("<i", data, 4)[0]
    o = 8 + l_text
    n_ref = struct.unpack_from("<i", data, o)[0]
    o += 4
    refs = []
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", data, o)[0]
        refs.append(_lossy(data[o + 4:o + 4 + ln - 1]))
        o += 4 + ln + 4
    recs = []
    while o < len(data):
        bs = struct.unpack_from("<I", data, o)[0]
        recs.append(data[o + 4:o + 4 + bs])
        o += 4 + bs
    return refs, recs


def _u32(x: int) -> int:
    return x & 0xFFFFFFFF


def record_row(b: bytes, refs: List[str], mode: str) -> Dict[str, Optional[object]]:
    ref_id, pos, l_name, _mapq, _bin, n_cig, flag, l_seq = struct.unpack_from("<iiBBHHHI", b, 0)
    name_raw = b[32:32 + l_name]
    o = 32 + l_name
    cigar = list(struct.unpack_from(f"<{n_cig}I", b, o)) if n_cig else []
    o += 4 * n_cig
    seq_b = b[o:o + (l_seq + 1) // 2]
    o += (l_seq + 1) // 2
    qual = b[o:o + l_seq]
    qname = name_raw[:-1] if l_name else b""
    rlen = 0
    for c in cigar:
        if c & 15 in (0, 2, 3, 7, 8):
            rlen = (rlen + (c >> 4)) & 0xFFFFFFFF
    nibbles = [(seq_b[i >> 1] >> (0 if i & 1 else 4)) & 15 for i in range(l_seq)]
    row = {}
    if mode == "noodles" and (l_name == 0 or name_raw == b"*\x00"):
        row["name"] = "unknown"
    else:
        row["name"] = _lossy(qname)
    row["chrom"] = refs[ref_id] if 0 <= ref_id < len(refs) else None
    if mode == "htslib":
        row["start"] = _u32(pos + 1) if pos >= 0 else None
        row["end"] = _u32(row["start"] + l_seq - 1) if pos >= 0 else None
    elif mode == "noodles":
        row["start"] = _u32(pos + 1) if pos >= 0 else None
        row["end"] = _u32(row["start"] + rlen - 1) if pos >= 0 else None
    else:
        row["start"] = _u32(pos) if pos >= 0 else None
        ref_end = pos + rlen if (not (flag & 4) and n_cig > 0) else pos + 1
        row["end"] = _u32(ref_end) if ref_end > pos else row["start"]
    row["flags"] = flag
    if l_seq == 0:
        row["sequence"] = None
    elif mode == "htslib_blocks":
        row["sequence"] = "".join(_NT16[x] for x in nibbles)
    else:
        row["sequence"] = "".join(_DECODE.get(x, "N") for x in nibbles)
    if l_seq == 0 or (mode == "htslib" and qual[0] == 0xFF):
        row["quality_scores"] = None
    else:
        row["quality_scores"] = bytes((q + 33) & 0xFF for q in qual)
    return row


def bam_rows(path: str, mode: str) -> List[dict]:
    refs, recs = read_bam(path)
    return [record_row(r, refs, mode) for r in recs]


_FNV0, _FNVP = 1469598103934665603, 1099511628211
_COLS = ("name", "chrom", "start", "end", "flags", "sequence", "quality_scores")


def _fnv(h: int, data: bytes) -> int:
    for x in data:
        h = ((h ^ x) * _FNVP) & 0xFFFFFFFFFFFFFFFF
    return h


def rows_digest(rows) -> list:
    """The per-column FNV-1a digests oracle_bam_digest (oracle/bam_oracle.cpp) computes."""
    d = [_FNV0] * 7
    for r in rows:
        for c, k in enumerate(_COLS):
            v = r[k]
            if k == "flags":
                d[c] = _fnv(d[c], struct.pack("<I", v))
                continue
            if v is None:
                d[c] = _fnv(d[c], b"\xff")
                continue
            if isinstance(v, int):
                v = struct.pack("<I", v)
            elif isinstance(v, str):
                v = v.encode()
            d[c] = _fnv(_fnv(d[c], v), b"\x01")
    return d


def cpp_digest(path: str, mode: str):
    """(record count, 7 column digests) from the C++ restatement (single core)."""
    import ctypes
    import numpy as np
    from . import pyoracle
    out = np.zeros(7, dtype=np.uint64)
    n = pyoracle.lib().oracle_bam_digest(path.encode(), {"noodles": 0, "htslib": 1, "htslib_blocks": 2}[mode],
                                         ctypes.c_void_p(out.ctypes.data))
    return int(n), [int(x) for x in out]
