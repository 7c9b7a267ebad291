"""Synthetic BAM files (SAMv1 §4: BGZF-compressed binary records) for tests and the C5
bench. Pure Python + zlib; `write_bam` takes explicit records (edge cases), and
`synth_bam` writes N uniform 150-bp reads of the synth-v1 UMI workload fast (numpy-built
fixed-size records, blocks compressed on threads: zlib releases the GIL).
"""
from __future__ import annotations

import struct
import zlib
from concurrent.futures import ThreadPoolExecutor
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
_NT16 = {c: i for i, c in enumerate("=ACMGRSVTWYHKDBN")}
_CIGAR_OPS = "MIDNSHP=X"
MAX_BLOCK_DATA = 0xFF00


def bgzf_block(data: bytes, level: int = 6) -> bytes:
    co = zlib.compressobj(level, zlib.DEFLATED, -15)
    cdata = co.compress(data) + co.flush()
    bsize = 18 + len(cdata) + 8
    hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize - 1)
    return hdr + cdata + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


def bgzf_compress(stream: bytes, level: int = 6, threads: int = 8, block: int = MAX_BLOCK_DATA) -> bytes:
    chunks = [stream[i:i + block] for i in range(0, len(stream), block)]
    if threads > 1 and len(chunks) > 8:
        with ThreadPoolExecutor(threads) as ex:
            blocks = list(ex.map(lambda c: bgzf_block(c, level), chunks))
    else:
        blocks = [bgzf_block(c, level) for c in chunks]
    return b"".join(blocks) + BGZF_EOF


def header_bytes(text: str, refs: Sequence[Tuple[bytes, int]]) -> bytes:
    t = text.encode() if isinstance(text, str) else text
    out = [b"BAM\x01", struct.pack("<i", len(t)), t, struct.pack("<i", len(refs))]
    for name, length in refs:
        out += [struct.pack("<i", len(name) + 1), name + b"\x00", struct.pack("<i", length)]
    return b"".join(out)


def record_bytes(name: bytes = b"r", ref_id: int = -1, pos: int = -1, mapq: int = 255, flag: int = 4,
                 cigar: Iterable[Tuple[int, str]] = (), seq: str = "", qual: Optional[bytes] = None,
                 next_ref_id: int = -1, next_pos: int = -1, tlen: int = 0, tags: bytes = b"",
                 raw_cigar: Optional[List[int]] = None, bin_: int = 4680) -> bytes:
    """One BAM record (block_size included). qual None = missing (0xFF * l_seq)."""
    cig = raw_cigar if raw_cigar is not None else [(n << 4) | _CIGAR_OPS.index(op) for n, op in cigar]
    l_seq = len(seq)
    packed = bytearray((l_seq + 1) // 2)
    for i, ch in enumerate(seq):
        code = _NT16[ch]
        packed[i >> 1] |= code << (0 if i & 1 else 4)
    q = b"\xff" * l_seq if qual is None else qual
    assert len(q) == l_seq
    body = struct.pack("<iiBBHHHIiii", ref_id, pos, len(name) + 1, mapq, bin_, len(cig), flag, l_seq, next_ref_id,
                       next_pos, tlen)
    body += name + b"\x00" + b"".join(struct.pack("<I", c) for c in cig) + bytes(packed) + q + tags
    return struct.pack("<I", len(body)) + body


def write_bam(path: str, refs: Sequence[Tuple[bytes, int]], records: Iterable[bytes], text: str = "",
              level: int = 6, block: int = MAX_BLOCK_DATA) -> None:
    stream = header_bytes(text, refs) + b"".join(records)
    with open(path, "wb") as f:
        f.write(bgzf_compress(stream, level, block=block))


def synth_bam(path: str, n: int, read_len: int = 150, umi_len: int = 12, seed: int = 0x524F47544B,
              n_refs: int = 24, level: int = 1, threads: int = 16) -> np.ndarray:
    """n mapped reads, 150 bp, M:150 CIGAR, name "r<9 digits>_<UMI>", sequence = UMI
    (synth-v1 UMI of read i, rogtk_amd.synth) + random template bases. Returns the packed
    UMI codes of the reads (first base most significant) for checking the UMI column."""
    from . import synth
    codes = synth.umi_codes(n, umi_len, seed)
    rng = np.random.default_rng(seed ^ 0xBA)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    # sequence bases as 2-bit codes
    bases = rng.integers(0, 4, size=(n, read_len), dtype=np.uint8)
    shifts = 2 * (umi_len - 1 - np.arange(umi_len, dtype=np.uint32))
    bases[:, :umi_len] = ((codes[:, None] >> shifts[None, :]) & 3).astype(np.uint8)
    nt16 = np.array([1, 2, 4, 8], np.uint8)[bases]
    packed = (nt16[:, 0::2] << 4) | nt16[:, 1::2] if read_len % 2 == 0 else None
    assert packed is not None, "even read length"
    qual = rng.integers(2, 41, size=(n, read_len), dtype=np.uint8)
    name_len = 1 + 9 + 1 + umi_len  # r + 9 digits + _ + UMI
    idx = np.arange(n, dtype=np.int64)
    digits = np.zeros((n, 9), np.uint8)
    v = idx.copy()
    for d in range(8, -1, -1):
        digits[:, d] = (v % 10) + 48
        v //= 10
    names = np.concatenate([np.full((n, 1), ord("r"), np.uint8), digits, np.full((n, 1), ord("_"), np.uint8),
                            acgt[bases[:, :umi_len]], np.zeros((n, 1), np.uint8)], axis=1)
    body_len = 32 + (name_len + 1) + 4 + read_len // 2 + read_len
    rec = np.zeros((n, 4 + body_len), np.uint8)
    hdr = np.zeros(n, dtype=np.dtype([("bs", "<u4"), ("ref", "<i4"), ("pos", "<i4"), ("lrn", "u1"), ("mapq", "u1"),
                                      ("bin", "<u2"), ("ncig", "<u2"), ("flag", "<u2"), ("lseq", "<u4"),
                                      ("nref", "<i4"), ("npos", "<i4"), ("tlen", "<i4")]))
    hdr["bs"] = body_len
    hdr["ref"] = rng.integers(0, n_refs, size=n)
    hdr["pos"] = rng.integers(0, 100_000_000, size=n)
    hdr["lrn"] = name_len + 1
    hdr["mapq"] = 60
    hdr["bin"] = 4680
    hdr["ncig"] = 1
    hdr["flag"] = rng.choice(np.array([0, 16, 99, 147, 83, 163], np.uint16), size=n)
    hdr["lseq"] = read_len
    hdr["nref"] = -1
    hdr["npos"] = -1
    rec[:, :36] = hdr.view(np.uint8).reshape(n, 36)
    o = 36
    rec[:, o:o + name_len + 1] = names
    o += name_len + 1
    rec[:, o:o + 4] = np.frombuffer(struct.pack("<I", (read_len << 4) | 0), np.uint8)
    o += 4
    rec[:, o:o + read_len // 2] = packed
    o += read_len // 2
    rec[:, o:o + read_len] = qual
    refs = [(f"chr{i + 1}".encode(), 250_000_000) for i in range(n_refs)]
    stream = header_bytes("@HD\tVN:1.6\tSO:unsorted\n", refs) + rec.tobytes()
    with open(path, "wb") as f:
        f.write(bgzf_compress(stream, level, threads))
    return codes
