"""Paired FASTQ ingest (host C++, no GPU needed) vs the Python restatement of
parse_paired_fastqs (oracle/pyfastq.py): every field of every record."""
from __future__ import annotations

import gzip

import numpy as np
import pytest


def _write(path, lines, gz=True, crlf=False, members=1, final_newline=True):
    body = ("\r\n" if crlf else "\n").join(lines)
    if final_newline:
        body += "\r\n" if crlf else "\n"
    data = body.encode("utf-8") if isinstance(body, str) else body
    if gz:
        parts = np.array_split(np.frombuffer(data, dtype=np.uint8), members)
        with open(path, "wb") as f:
            for p in parts:
                f.write(gzip.compress(p.tobytes()))
    else:
        with open(path, "wb") as f:
            f.write(data)


def _records(rng, n, r1_len=40, r2_len=90):
    l1, l2 = [], []
    for i in range(n):
        s1 = "".join(rng.choice(list("ACGTN"), r1_len))
        s2 = "".join(rng.choice(list("ACGTNx"), r2_len))
        ids = ["@read%d extra" % i, "@@read%d\t " % i, "@r%d " % i][i % 3]
        l1 += [ids, s1, "+", "".join(rng.choice(list("FFFF:#,"), r1_len))]
        l2 += [ids, s2 + ("  " if i % 2 else ""), "+", "".join(rng.choice(list("FFFF:#,"), r2_len)) + " "]
    return l1, l2


def _run(p1, p2, cbc, umi, limit=None, rev=False, batch=7):
    from rogtk_amd import iter_paired_fastqs

    rows = []
    for b in iter_paired_fastqs(str(p1), str(p2), cbc, umi, limit, rev, batch_records=batch):
        cols = [b.column(i).to_pylist() for i in range(9)]
        rows += list(zip(*cols))
    return rows


@pytest.mark.parametrize("rev", [False, True])
@pytest.mark.parametrize("crlf,members,final_nl", [(False, 1, True), (True, 3, True), (False, 2, False)])
def test_matches_restatement(tmp_path, rev, crlf, members, final_nl):
    from oracle import pyfastq

    rng = np.random.default_rng(7)
    l1, l2 = _records(rng, 50)
    p1, p2 = tmp_path / "r1.fq.gz", tmp_path / "r2.fq.gz"
    _write(p1, l1, crlf=crlf, members=members, final_newline=final_nl)
    _write(p2, l2, crlf=crlf, members=members, final_newline=final_nl)
    for cbc, umi in ((16, 12), (0, 10), (28, 12)):
        assert _run(p1, p2, cbc, umi, rev=rev) == pyfastq.parse(p1, p2, cbc, umi, do_rev_comp=rev)
    for limit in (0, 8, 40, 1000):
        assert _run(p1, p2, 16, 12, limit=limit) == pyfastq.parse(p1, p2, 16, 12, limit=limit)


def test_unequal_files_invalid_utf8_and_plain(tmp_path):
    from oracle import pyfastq

    rng = np.random.default_rng(3)
    l1, l2 = _records(rng, 30)
    raw1 = ("\n".join(l1[:20]) + "\n").encode() + b"\xff\xfe broken line\n" + ("\n".join(l1[20:]) + "\n").encode()
    p1, p2 = tmp_path / "a.fq.gz", tmp_path / "b.fq"
    with open(p1, "wb") as f:
        f.write(gzip.compress(raw1))
    _write(p2, l2[:80], gz=False)  # plain text, fewer records: zip stops early
    assert _run(p1, p2, 16, 12) == pyfastq.parse(p1, p2, 16, 12)


def test_errors(tmp_path):
    from rogtk_amd import RogtkError

    rng = np.random.default_rng(5)
    l1, l2 = _records(rng, 4, r1_len=20)
    p1, p2 = tmp_path / "a.fq.gz", tmp_path / "b.fq.gz"
    _write(p1, l1)
    _write(p2, l2)
    with pytest.raises(RogtkError, match="invalid range"):
        _run(p1, p2, 16, 12)  # 28 > 20-byte reads: the reference's expect() panic
    with pytest.raises(RogtkError, match="truncated"):
        _run(p1, p2, 4, 4, limit=10)  # 10 lines: a 2-line chunk
    with pytest.raises(RogtkError, match="cannot open"):
        _run(tmp_path / "missing.gz", p2, 4, 4)


def test_parquet_output(tmp_path):
    import pyarrow.parquet as pq

    from oracle import pyfastq
    from rogtk_amd import parse_paired_fastqs

    rng = np.random.default_rng(11)
    l1, l2 = _records(rng, 25)
    p1, p2, out = tmp_path / "a.fq.gz", tmp_path / "b.fq.gz", tmp_path / "o.parquet"
    _write(p1, l1)
    _write(p2, l2)
    parse_paired_fastqs(str(p1), str(p2), 16, 12, str(out), do_rev_comp=True)
    t = pq.read_table(out)
    assert t.schema.names == ["read_id", "start", "end", "cbc", "umi", "cbc_qual", "umi_qual", "seq", "qual"]
    assert list(zip(*(t.column(i).to_pylist() for i in range(9)))) == pyfastq.parse(p1, p2, 16, 12, do_rev_comp=True)


@pytest.mark.gpu
def test_umi_column_feeds_h1_h3(tmp_path):
    """FASTQ -> umi column -> H1 scores and H3 ids on the GPU, bit-exact vs the oracle."""
    from oracle import pyoracle as P
    from rogtk_amd import iter_paired_fastqs, umi_cluster, umi_complexity_scores
    from rogtk_amd import synth

    n = 20000
    umis = synth.umi_ascii(n, 12, p_n=0.001)
    rng = np.random.default_rng(1)
    l1, l2 = [], []
    for i in range(n):
        cbc = "".join(rng.choice(list("ACGT"), 16))
        l1 += ["@r%d" % i, cbc + umis[i].tobytes().decode() + "TTTTT", "+", "F" * 33]
        l2 += ["@r%d" % i, "ACGT" * 20, "+", "F" * 80]
    p1, p2 = tmp_path / "a.fq.gz", tmp_path / "b.fq.gz"
    _write(p1, l1)
    _write(p2, l2)
    umi = next(iter_paired_fastqs(str(p1), str(p2), 16, 12)).column("umi")
    col = P.StrCol.from_fixed(umis)
    got = umi_complexity_scores(umi)
    ref = P.umi_complexity(col)
    for f in P.FIELDS:
        g = np.asarray(got.field(f))
        assert np.array_equal(g.view(np.uint64) if g.dtype == np.float64 else g, ref[f].view(np.uint64)
                              if ref[f].dtype == np.float64 else ref[f]), f
    cid, k, _ = umi_cluster(umi, 12, 1)
    rc, _, rk, _ = P.umi_cluster(col, 12, 1)
    assert k == rk and np.array_equal(np.asarray(cid), rc)
