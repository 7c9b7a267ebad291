"""BAM -> Arrow: GPU record decoding (rogtk_amd/csrc/bam.hip) vs
the pure-Python restatement (oracle/pybam.py) of the reference's three record semantics.

The reference ships no BAM fixtures; files are written here (rogtk_amd/synth_bam.py,
SAMv1 layout) with the edge cases its code distinguishes: unmapped / out-of-range refIDs,
pos -1 and < -1, '*' names, non-UTF-8 names, CIGARs with every op (and invalid op codes),
empty and odd-length sequences, IUPAC bases, missing (0xFF) and > 93 qualities, records
spanning BGZF blocks and decode batches.
"""
import os

import numpy as np
import pyarrow as pa
import pytest

from oracle import pybam
from rogtk_amd import synth_bam

MODES = ("noodles", "htslib", "htslib_blocks")
REFS = [(b"chr1", 1000), (b"chrX", 500), (b"contig_\xff\xfe", 10)]


def _random_records(seed, n):
    rng = np.random.default_rng(seed)
    iupac = "=ACMGRSVTWYHKDBN"
    recs = []
    for i in range(n):
        kind = int(rng.integers(0, 12))
        name = f"read{i}".encode()
        if kind == 0:
            name = b"*"
        elif kind == 1:
            name = b"bad\xff\xc3(x\xe2\x82" + bytes([int(rng.integers(128, 256))])
        elif kind == 2:
            name = bytes(rng.integers(33, 127, size=int(rng.integers(100, 250)), dtype=np.uint8))
        ref_id = int(rng.choice([-1, 0, 1, 2, 3, -5]))
        pos = int(rng.choice([-1, -2, 0, int(rng.integers(0, 10**6))]))
        flag = int(rng.integers(0, 1 << 16))
        l_seq = int(rng.choice([0, 1, 7, 12, 150, int(rng.integers(0, 300))]))
        alphabet = iupac if kind in (3, 4) else "ACGTN"
        seq = "".join(rng.choice(list(alphabet), l_seq)) if l_seq else ""
        if kind == 5 and l_seq:
            qual = None
        elif kind == 6 and l_seq:
            qual = bytes([0]) + b"\xff" * (l_seq - 1)
        elif kind == 7 and l_seq:
            qual = bytes(rng.integers(90, 255, size=l_seq, dtype=np.uint8))
        else:
            qual = bytes(rng.integers(0, 42, size=l_seq, dtype=np.uint8))
        n_cig = int(rng.integers(0, 6))
        raw_cigar = [int(rng.integers(0, 200)) << 4 | int(rng.integers(0, 16 if kind == 8 else 9)) for _ in range(n_cig)]
        tags = b"NMi\x01\x00\x00\x00" if kind % 2 else b""
        recs.append(synth_bam.record_bytes(name=name, ref_id=ref_id, pos=pos, flag=flag, seq=seq, qual=qual,
                                           raw_cigar=raw_cigar, tags=tags))
    return recs


@pytest.fixture(scope="module")
def edge_bam(tmp_path_factory):
    p = str(tmp_path_factory.mktemp("bam") / "edge.bam")
    # small BGZF blocks so records straddle block boundaries
    synth_bam.write_bam(p, REFS, _random_records(7, 3000), text="@HD\tVN:1.6\n", block=997)
    return p


# ------------------------------------------------------------------ CPU
def _stream_map(path):
    """(compressed block offset -> stream offset of its first byte, the record starts in
    the inflated stream) of a BAM file, from a plain walk of its blocks."""
    import gzip
    import struct

    raw = open(path, "rb").read()
    offs, o, u = {}, 0, 0
    while o < len(raw):
        bsize = struct.unpack_from("<H", raw, o + 16)[0] + 1
        offs[o] = u
        u += struct.unpack_from("<I", raw, o + bsize - 4)[0]
        o += bsize
    data = gzip.decompress(raw)
    q = 8 + struct.unpack_from("<i", data, 4)[0]
    nref = struct.unpack_from("<i", data, q)[0]
    q += 4
    for _ in range(nref):
        q += 8 + struct.unpack_from("<i", data, q)[0]
    starts = []
    while q < len(data):
        starts.append(q)
        q += 4 + struct.unpack_from("<I", data, q)[0]
    return offs, np.array(starts, dtype=np.int64)


@pytest.mark.parametrize("block,long_names", [(997, False), (65280, False), (4093, True)])
def test_split_points_and_record_starts(tmp_path, block, long_names):
    """One BAM cut at BGZF block starts (the reference's discover_split_points,
    bam_htslib.rs:247): every split point is a block start past the header's blocks, and
    rogtk_bam_find_record finds exactly the first record that starts in each range (the
    straddling record's tail skipped), for 2..17 ranges and records that span blocks.
    Host-only entry points: no GPU."""
    from rogtk_amd import bam as B

    p = str(tmp_path / "s.bam")
    recs = _random_records(11, 2500)
    if long_names:  # records of 300-600 B spanning many small blocks
        recs = [synth_bam.record_bytes(name=b"n" * 200 + str(i).encode(), seq="ACGT" * 60) for i in range(800)]
    synth_bam.write_bam(p, REFS, recs, text="@HD\tVN:1.6\n", block=block)
    offs, starts = _stream_map(p)
    size = os.path.getsize(p)
    for n in (1, 2, 3, 5, 8, 17):
        pts = B.bam_split_points(p, n)
        assert pts[0] == 0 and pts[-1] == size and len(pts) - 1 <= n
        assert all(a < b for a, b in zip(pts, pts[1:]))
        for c in pts[1:-1]:
            assert c in offs
            uo = offs[c]
            assert uo > starts[0]  # past the header
            nxt = starts[starts >= uo]
            assert B.bam_find_record(p, c) == (int(nxt[0] - uo) if nxt.size else 0)



def test_oracle_known_answers(tmp_path):
    p = str(tmp_path / "kat.bam")
    recs = [
        # mapped, 5S10M2D3I4M (ref length 16), pos 99 (0-based)
        synth_bam.record_bytes(name=b"q1", ref_id=1, pos=99, flag=0, cigar=[(5, "S"), (10, "M"), (2, "D"),
                                                                          (3, "I"), (4, "M")],
                               seq="ACGTNACGTAACGTAACGTAC", qual=bytes(range(21))),
        # unmapped, no CIGAR, missing qualities, name "*"
        synth_bam.record_bytes(name=b"*", ref_id=-1, pos=-1, flag=4, seq="ACGR", qual=None),
        # empty sequence
        synth_bam.record_bytes(name=b"e", ref_id=0, pos=0, flag=0, cigar=[(3, "N")], seq="", qual=b""),
    ]
    synth_bam.write_bam(p, REFS, recs)
    n, h, b = (pybam.bam_rows(p, m) for m in MODES)
    assert n[0] == {"name": "q1", "chrom": "chrX", "start": 100, "end": 115, "flags": 0,
                    "sequence": "ACGTNACGTAACGTAACGTAC", "quality_scores": bytes(range(33, 54))}
    assert h[0]["start"] == 100 and h[0]["end"] == 120  # start + seq_len - 1
    assert b[0]["start"] == 99 and b[0]["end"] == 115  # 0-based, bam_endpos
    assert n[1]["name"] == "unknown" and h[1]["name"] == "*" and b[1]["name"] == "*"
    assert n[1]["chrom"] is None and n[1]["start"] is None and n[1]["end"] is None
    assert b[1]["start"] is None and b[1]["end"] == 0  # bam_endpos(pos -1) = 0 > -1
    assert h[1]["quality_scores"] is None and n[1]["quality_scores"] == b"\x20" * 4
    assert n[1]["sequence"] == "ACGN" and b[1]["sequence"] == "ACGR"
    assert n[2]["sequence"] is None and n[2]["quality_scores"] is None
    assert n[2]["start"] == 1 and n[2]["end"] == 3 and h[2]["end"] == 0
    assert pybam.read_bam(p)[0] == ["chr1", "chrX", "contig_��"]


def test_bgzf_writer_round_trip(tmp_path):
    import gzip
    p = str(tmp_path / "rt.bam")
    recs = _random_records(1, 200)
    synth_bam.write_bam(p, REFS, recs, block=333)
    refs, got = pybam.read_bam(p)
    assert [r[4:] for r in recs] == got
    raw = open(p, "rb").read()
    assert raw.endswith(synth_bam.BGZF_EOF)
    assert gzip.decompress(raw)[:4] == b"BAM\x01"


# ------------------------------------------------------------------ GPU
def _rows_of(batches, mode):
    out = []
    for rb in batches:
        cols = {n: rb.column(n) for n in rb.schema.names}
        for n in ("sequence", "quality_scores"):
            if n in cols:
                cols[n] = cols[n].view(pa.binary())
        d = {k: v.to_pylist() for k, v in cols.items()}
        for i in range(rb.num_rows):
            out.append({k: d[k][i] for k in d})
    return out


def _expect(rows, include_sequence, include_quality):
    out = []
    for r in rows:
        r = dict(r)
        if r["sequence"] is not None:
            r["sequence"] = r["sequence"].encode()
        if not include_sequence:
            del r["sequence"]
        if not include_quality:
            del r["quality_scores"]
        out.append(r)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("max_records", [1, 97, 1 << 20])
def test_gpu_decode_matches_oracle(edge_bam, mode, max_records):
    from rogtk_amd.bam import BamReader
    ref = _expect(pybam.bam_rows(edge_bam, mode), True, True)
    got = []
    with BamReader(edge_bam, n_threads=4) as r:
        assert r.reference_names() == ["chr1", "chrX", "contig_��"]
        while True:
            rb = r.next_batch(max_records if max_records != 1 else 13 if got else 1, mode)
            if rb is None:
                break
            got += _rows_of([rb], mode)
    assert len(got) == len(ref)
    bad = [i for i in range(len(ref)) if got[i] != ref[i]]
    assert not bad, (bad[:3], got[bad[0]], ref[bad[0]])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 5, 13])
def test_gpu_range_readers_cover_the_file(edge_bam, n):
    """The ranges of one file (split points + found record starts) decoded by range readers
    are the whole file's rows exactly once, in order; each range's tail equals the next
    range's skip (what bams_umi_cluster checks across ranks)."""
    from rogtk_amd import bam as B
    ref = _expect(pybam.bam_rows(edge_bam, "htslib_blocks"), True, True)
    pts = B.bam_split_points(edge_bam, n)
    got, tails, skips = [], [], []
    for i in range(len(pts) - 1):
        skip = 0 if i == 0 else B.bam_find_record(edge_bam, pts[i])
        skips.append(skip)
        with B.BamReader(edge_bam, 4, rng=(pts[i], pts[i + 1], skip)) as r:
            while True:
                rb = r.next_batch(101, "htslib_blocks")
                if rb is None:
                    break
                got += _rows_of([rb], "htslib_blocks")
            tails.append(r.tail())
    assert len(pts) - 1 == n and tails[-1] == -1
    assert tails[:-1] == skips[1:]
    assert got == ref


@pytest.mark.gpu
@pytest.mark.parametrize("inc", [(False, False), (True, False), (False, True)])
def test_gpu_decode_column_selection(edge_bam, inc):
    from rogtk_amd.bam import iter_bam_batches
    ref = _expect(pybam.bam_rows(edge_bam, "htslib"), *inc)
    got = _rows_of(iter_bam_batches(edge_bam, 500, inc[0], inc[1], mode="htslib"), "htslib")
    assert got == ref


@pytest.mark.gpu
def test_synth_bam_umis_and_large_batches(tmp_path):
    from rogtk_amd.bam import iter_bam_batches
    p = str(tmp_path / "s.bam")
    codes = synth_bam.synth_bam(p, 60_000, level=1)
    ref = _expect(pybam.bam_rows(p, "noodles"), True, True)
    got = _rows_of(iter_bam_batches(p, 50_000, mode="noodles"), "noodles")
    assert got == ref
    acgt = "ACGT"
    umi0 = "".join(acgt[(int(codes[0]) >> (2 * (11 - j))) & 3] for j in range(12))
    assert got[0]["sequence"][:12].decode() == umi0 and got[0]["name"].endswith("_" + umi0)


@pytest.mark.gpu
@pytest.mark.parametrize("readahead", ["1", "0"])
@pytest.mark.parametrize("chunk", ["4096", "70000", "1000000"])
def test_bgzf_readahead_and_chunks(edge_bam, tmp_path, monkeypatch, readahead, chunk):
    """The BGZF read-ahead thread (default) and the synchronous path give the oracle's
    records for every compressed chunk size: chunks smaller than one block (4096), a few
    blocks per chunk (many read-ahead steps and buffer moves per batch) and whole files."""
    from rogtk_amd.bam import BamReader, iter_bam_batches
    monkeypatch.setenv("ROGTK_BAM_READAHEAD", readahead)
    monkeypatch.setenv("ROGTK_BAM_CHUNK", chunk)
    p = str(tmp_path / "s.bam")
    synth_bam.synth_bam(p, 40_000, level=1)
    for path, mode, batch in ((p, "htslib", 7_000), (edge_bam, "noodles", 333)):
        ref = _expect(pybam.bam_rows(path, mode), True, True)
        got = _rows_of(iter_bam_batches(path, batch, mode=mode), mode)
        assert len(got) == len(ref)
        assert got == ref
    with BamReader(p, n_threads=3) as r:  # a reader closed mid-file joins its read-ahead thread
        assert r.next_batch(100, "htslib").num_rows == 100


@pytest.mark.gpu
def test_converters_write_the_reference_schema(edge_bam, tmp_path):
    import pyarrow.parquet as pq
    from rogtk_amd import bam as B
    ipc = str(tmp_path / "out" / "a.arrow")
    B.bam_to_arrow_ipc_htslib_optimized(edge_bam, ipc, batch_size=700, limit=2500)
    with pa.ipc.open_file(ipc) as f:
        t = f.read_all()
    assert t.schema == B.bam_schema(True, True)
    assert t.num_rows == 2500 and max(b.num_rows for b in t.to_batches()) == 700
    ref = _expect(pybam.bam_rows(edge_bam, "htslib"), True, True)[:2500]
    assert _rows_of(t.to_batches(), "htslib") == ref
    pqp = str(tmp_path / "b.parquet")
    B.bams_to_parquet([edge_bam, edge_bam], pqp, batch_size=1000, include_quality=False, limit=4000,
                      include_source_file=True)
    t = pq.read_table(pqp)
    assert t.schema.names == ["name", "chrom", "start", "end", "flags", "sequence", "source_file"]
    assert t.num_rows == 4000 and set(t.column("source_file").to_pylist()) == {os.path.basename(edge_bam)}
    nref = _expect(pybam.bam_rows(edge_bam, "noodles"), True, False)
    got = _rows_of(t.drop_columns(["source_file"]).to_batches(), "noodles")
    assert got == (nref + nref)[:4000]
    B.bam_to_arrow_ipc_htslib_bgzf_blocks(edge_bam, ipc, include_sequence=False)
    with pa.ipc.open_file(ipc) as f:
        t = f.read_all()
    assert _rows_of(t.to_batches(), "htslib_blocks") == _expect(pybam.bam_rows(edge_bam, "htslib_blocks"), False,
                                                                True)


@pytest.mark.gpu
def test_errors(edge_bam, tmp_path):
    from rogtk_amd import RogtkError
    from rogtk_amd import bam as B
    with pytest.raises(RogtkError, match="BAM file does not exist"):
        B.bam_to_arrow_ipc(str(tmp_path / "nope.bam"), str(tmp_path / "x.arrow"))
    with pytest.raises(RogtkError, match="batch_size must be greater than 0"):
        B.bam_to_parquet(edge_bam, str(tmp_path / "x.parquet"), batch_size=0)
    raw = open(edge_bam, "rb").read()
    cut = str(tmp_path / "cut.bam")
    with open(cut, "wb") as f:
        f.write(raw[: len(raw) // 2])
    with pytest.raises(RogtkError, match="truncated"):
        list(B.iter_bam_batches(cut))
    notbam = str(tmp_path / "plain.bam")
    with open(notbam, "wb") as f:
        f.write(synth_bam.bgzf_compress(b"SAM\x01" + b"\x00" * 64))
    with pytest.raises(RogtkError, match="bad magic"):
        list(B.iter_bam_batches(notbam))


def _oracle_umis(rows, source, umi_len, sep="_"):
    out = []
    for r in rows:
        if source == "sequence":
            s = r["sequence"]
            out.append(None if s is None else s[:umi_len].encode())
        else:
            nm = r["name"].encode()
            k = nm.rfind(sep.encode())
            out.append(None if k < 0 else nm[k + 1:])
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["sequence", "name"])
@pytest.mark.parametrize("md", [0, 1])
def test_bam_umi_cluster_matches_oracle(tmp_path, monkeypatch, source, md):
    from oracle import pyoracle as P
    from rogtk_amd import bam as B
    p = str(tmp_path / "c5.bam")
    synth_bam.synth_bam(p, 30_000, level=1)
    # a few irregular UMIs (N in the UMI, short reads, names without the separator)
    extra = [synth_bam.record_bytes(name=b"x_ACGNACGTACGT", seq="ACGNACGTACGTAAAA", qual=None),
             synth_bam.record_bytes(name=b"noumi", seq="ACG", qual=b"\x01\x02\x03"),
             synth_bam.record_bytes(name=b"y_ACGTACGTAC", seq="", qual=b"")]
    raw = open(p, "rb").read()
    import gzip
    body = gzip.decompress(raw)
    with open(p, "wb") as f:
        f.write(synth_bam.bgzf_compress(body + b"".join(extra), level=1))
    monkeypatch.setattr(B, "DECODE_RECORDS", 7_000)  # several device batches
    t = B.bam_umi_cluster(p, umi_len=12, max_distance=md, source=source, mode="htslib")
    rows = pybam.bam_rows(p, "htslib")
    umis = _oracle_umis(rows, source, 12)
    assert t.column("umi").to_pylist() == [None if u is None else u.decode() for u in umis]
    rc, rv, rk, _ = P.umi_cluster(P.StrCol.from_list(umis), 12, md)
    got = t.column("cluster_id").to_numpy(zero_copy_only=False)
    valid = np.array([u is not None for u in umis])
    assert int(t.schema.metadata[b"n_clusters"]) == rk
    assert np.array_equal(np.asarray(t.column("cluster_id").is_valid()), valid)
    assert np.array_equal(got[rv].astype(np.uint32), rc[rv])
    assert t.column("name").to_pylist() == [r["name"] for r in rows]


@pytest.mark.parametrize("mode", MODES)
def test_cpp_restatement_matches_python_oracle(edge_bam, mode):
    """The single-core C++ restatement (CPU baseline of C5) = the Python oracle."""
    rows = pybam.bam_rows(edge_bam, mode)
    n, d = pybam.cpp_digest(edge_bam, mode)
    assert n == len(rows)
    assert d == pybam.rows_digest(rows)
