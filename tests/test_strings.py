"""Element-wise string expressions: reverse complement, CIGAR
parsing / expansion / insertions / allele enrichment, PHRED conversion.

CPU: the oracle (oracle/pystrings.py) against known answers taken from the
reference's own docstrings (rogtk/__init__.py:536-660, expressions.rs:81-83) and
hand-derived cases of its Rust semantics. GPU (-m gpu): rogtk_amd.strings through
the C ABI against the oracle on the same rows, bit-exact (bytes, offsets, nulls).
"""
from __future__ import annotations

import numpy as np
import pyarrow as pa
import pytest

from oracle import pystrings as O


# ------------------------------------------------------------------ oracle KATs
def test_oracle_docstring_alignments():
    # CigarNamespace.align_to_ref / align_to_query docstrings (rogtk/__init__.py:604-606, 643-645)
    r, q = O.expand_cigar_alignment("ATCGTACG", "ATCGACTGTACG", "4M4I4M")
    assert (r, q) == ("ATCG----TACG", "ATCGACTGTACG")
    r, q = O.expand_cigar_alignment("ATCGTACG", "ATCGATCGTACG", "4S8M")
    assert (r, q) == ("----ATCGTACG", "atcgATCGTACG")


def test_oracle_docstring_enrich():
    # enrich_allele_with_insertions doc (expressions.rs:81-83): [78:5I] -> [78:5I:GCTAG]
    seq = "A" * 77 + "GCTAG" + "T" * 20
    assert O.enrich_row("TAGTCATTAC[78:5I]ACTTAGACAGGTG", seq, "77M5I20M") == \
        "TAGTCATTAC[78:5I:GCTAG]ACTTAGACAGGTG"
    # not an insertion / None / unparsable / missing / unclosed stay as they are
    assert O.enrich_row("A[20:432D]C[None]G[x:5I]T[3:2I]", seq, "77M5I20M") == "A[20:432D]C[None]G[x:5I]T[3:2I]"
    assert O.enrich_row("AC[78:5I", seq, "77M5I20M") == "AC[78:5I"
    assert O.enrich_row("AC[78:5I]", None, "77M5I20M") == "AC[78:5I]"
    assert O.enrich_row(None, seq, "77M5I20M") is None
    # pos (1-based) -> 0-based first, then pos itself; '+' sign parses as usize
    assert O.enrich_row("[+78:5I]", seq, "77M5I20M") == "[+78:5I:GCTAG]"
    assert O.enrich_row("[77:5I]", seq, "77M5I20M") == "[77:5I:GCTAG]"


def test_oracle_parse_cigar_and_insertions():
    assert O.parse_cigar("10M2D5M3I4M", True) == "D,10,2|I,17,3"
    assert O.parse_cigar("10M2D5M3I4M", False) == "D,10,1|D,11,1|I,17,3"
    assert O.parse_cigar("10M", False) == ""
    assert O.parse_cigar("3S2D", True) == "D,3,2"  # S advances the position here
    assert O.parse_cigar("M2D", True) == "D,0,2"  # empty number: op skipped
    assert O.cigar_insertions("AACCGGTTAA", "2M2I2M2I2M") == "2:CC|4:TT"
    assert O.cigar_insertions("AACCGGTT", "2M2I0M2I") == "2:GG"  # same ref_pos: the later wins
    assert O.cigar_insertions("AAC", "2M5I") == ""  # insertion past the end of seq
    assert O.cigar_insertions("", "") == ""


def test_oracle_revcomp_phred():
    assert O.reverse_complement("ACGTNacgtX") == "XtgcaNACGT"
    assert O.reverse_complement("AÉC") == "GÉT"
    assert O.phred_str("II#", 33) == "40|40|2"
    assert O.phred_str(" ", 33) == "255"  # u8 wraps in the release build
    assert O.phred_str("", 33) == ""


# ------------------------------------------------------------------ GPU parity
def _rand_dna(rng, n, lo, hi, alphabet="ACGT"):
    al = np.frombuffer(alphabet.encode(), np.uint8)
    return [bytes(rng.choice(al, int(rng.integers(lo, hi + 1)))).decode() for _ in range(n)]


def _rand_cigar(rng, qlen, ops="MIDNSHP=X"):
    parts, used = [], 0
    while used < qlen:
        op = ops[int(rng.integers(len(ops)))]
        k = int(rng.integers(0, 12))
        parts.append(f"{k}{op}")
        used += k if op in "MIS=X" else 0
    return "".join(parts)


def _check_strings(got: pa.Array, want):
    assert len(got) == len(want)
    g = got.to_pylist()
    for i, (a, b) in enumerate(zip(g, want)):
        assert a == b, (i, a, b)


@pytest.fixture(scope="module")
def S():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from rogtk_amd import strings

    return strings


@pytest.mark.gpu
def test_gpu_revcomp(S):
    rng = np.random.default_rng(1)
    rows = _rand_dna(rng, 5000, 0, 300, "ACGTNacgtn") + ["AÉC", "日本ACGT", "", None, "X"]
    _check_strings(S.reverse_complement(pa.array(rows, type=pa.large_string())),
                   O.column("revcomp", [rows]))
    # int32 offsets, sliced with nulls
    arr = pa.array(rows, type=pa.string()).slice(7, 3000)
    _check_strings(S.reverse_complement(arr), O.column("revcomp", [rows[7:3007]]))


@pytest.mark.gpu
@pytest.mark.parametrize("block_dels", [False, True])
def test_gpu_parse_cigar(S, block_dels):
    rng = np.random.default_rng(2)
    rows = [_rand_cigar(rng, 150) for _ in range(4000)]
    rows += ["", None, "M", "5", "5Z3D", "3D日2I", "99999999999999999999999D1I", "18446744073709551615M1I",
             "0D0I", "+3D", "1000D"]
    _check_strings(S.parse_cigar(rows, block_dels=block_dels), O.column("parse_cigar", [rows], int(block_dels)))


@pytest.mark.gpu
@pytest.mark.parametrize("side", ["ref", "query"])
def test_gpu_aligned(S, side):
    rng = np.random.default_rng(3)
    n = 3000
    ref = _rand_dna(rng, n, 0, 200, "ACGTacgtN")
    qry = _rand_dna(rng, n, 0, 200, "ACGTacgtN")
    cig = [_rand_cigar(rng, len(q)) for q in qry]
    ref += ["AÉG", None, "ACGT", "ACGT", "ACGT"]
    qry += ["aéé", "ACGT", None, "ACGT", "ACGT"]
    cig += ["1M1S1M1D1I", "4M", "4M", None, "2H2P2M99999I"]
    op = "aligned_ref" if side == "ref" else "aligned_query"
    ns = S.CigarNamespace(ref)
    got = ns.align_to_ref(qry, cig) if side == "ref" else ns.align_to_query(qry, cig)
    _check_strings(got, O.column(op, [ref, qry, cig]))
    # scalar reference broadcast (pl.lit(ref_seq)), expressions.rs:344-349
    ns1 = S.CigarNamespace(["ACGTACGTAAcc"])
    got = ns1.align_to_ref(qry[:500], cig[:500]) if side == "ref" else ns1.align_to_query(qry[:500], cig[:500])
    _check_strings(got, O.column(op, [["ACGTACGTAAcc"], qry[:500], cig[:500]]))


@pytest.mark.gpu
def test_gpu_insertions_and_enrich(S):
    rng = np.random.default_rng(4)
    n = 3000
    seq = _rand_dna(rng, n, 0, 160) + ["AÉCÉGG", "AÉCÉGG", "ACGT", None]
    cig = [_rand_cigar(rng, len(s), "MIDS") for s in seq[:n]] + ["1M1I2I", "2M2I", "1M2I0M1I", "2I"]
    _check_strings(S.extract_cigar_insertions(seq, cig), O.column("cigar_insertions", [seq, cig]))
    # alleles that reference the insertions (1-based and 0-based positions), plus junk
    alleles = []
    for s, c in zip(seq, cig):
        ins = O.extract_insertions(s, c) if s is not None and c is not None else {}
        parts = ["AC"]
        for p in list(ins)[:3]:
            parts.append(f"[{p + int(rng.integers(0, 2))}:{len(ins[p])}I]")
        parts += ["[5:3D]", "[None]", "[x:1I]", "TT"]
        if rng.random() < 0.05:
            parts.append("[12:")
        alleles.append("".join(parts))
    alleles[5] = None
    cig2 = list(cig)
    cig2[6] = None
    _check_strings(S.CigarNamespace(alleles).enrich_insertions(seq, cig2),
                   O.column("enrich", [alleles, seq, cig2]))


@pytest.mark.gpu
def test_gpu_phred(S):
    rng = np.random.default_rng(5)
    rows = [bytes(rng.integers(33, 75, int(rng.integers(0, 200)), dtype=np.uint8)).decode() for _ in range(3000)]
    rows += ["", None, " ", "É~"]
    _check_strings(S.phred_to_numeric_str(rows), O.column("phred_str", [rows], 33))
    _check_strings(S.phred_to_numeric_str(rows, base=64), O.column("phred_str", [rows], 64))
    got = S.phred_to_numeric(rows, base=33).to_pylist()
    want = [v for v in O.column("phred_list", [rows], 33) if v is not None]  # null rows dropped
    assert got == want


@pytest.mark.gpu
def test_gpu_strings_large_batch(S):
    """1M reads of 150 bp: reverse complement twice is the identity; one pass equals the
    oracle on a sample of rows."""
    from rogtk_amd import synth

    rng = np.random.default_rng(6)
    raw = synth.reads(1_000_000, 150, seed=6)
    n = len(raw)
    # a LargeString column straight from the (n, 150) byte matrix, no Python strings
    offs = np.arange(n + 1, dtype=np.int64) * 150
    arr = pa.Array.from_buffers(pa.large_string(), n, [None, pa.py_buffer(offs), pa.py_buffer(raw.tobytes())])
    rc = S.reverse_complement(arr)
    back = S.reverse_complement(rc)
    assert back.equals(arr)
    for i in rng.integers(0, n, 2000):
        assert rc[int(i)].as_py() == O.reverse_complement(bytes(raw[int(i)]).decode())
