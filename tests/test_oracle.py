"""CPU: the oracle pinned against SURVEY.md Appendix A, the pure-Python restatement,
the committed golden vectors, and (for H3) an O(n^2) brute force."""
from __future__ import annotations

import math
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import pyoracle as P

# hand-derived known answers (dinucleotide terms summed in
# first-occurrence order, as printed there). Fields: shannon, linguistic,
# homopolymer, dinuc, longest, dust, combined.
APPENDIX_A = {
    b"AAAAAAAAAAAA": (0.0, 0.1, 1.0, 0.0, 12, 0.0, 0.125),
    b"ACGTACGTACGT": (2.0, 0.4, 0.0, 0.49520648405726964, 1, 0.0, 1.015947639275257),
    b"AACCGGTTAACC": (1.9182958340544893, 0.8, 0.0, 0.7284942682956881, 2, 0.0, 1.122181432091309),
    b"ACGTTGCAACGT": (2.0, 0.8, 0.0, 0.7284942682956881, 2, 0.0, 1.1426074735776865),
    b"GATTACAGATTA": (1.7841591278514217, 0.7, 0.0, 0.6830397228411426, 2, 0.0, 1.0568290737223602),
    b"NNNNNNNNNNNN": (0.0, 0.1, 1.0, 0.0, 12, 0.0, 0.125),
    b"ACGTNACGTACG": (1.930827083453526, 0.7, 0.0, 0.6032721091064395, 1, 0.0, 1.0898642538960142),
    b"acgtacgtacgt": (0.0, 0.4, 0.0, 0.49520648405726964, 1, 0.0, 0.5159476392752571),
}


def _ulp_diff(a: float, b: float) -> int:
    ia = np.array([a]).view(np.int64)[0]
    ib = np.array([b]).view(np.int64)[0]
    return abs(int(ia) - int(ib))


@pytest.mark.parametrize("umi", list(APPENDIX_A))
def test_appendix_a_first_occurrence_order_exact(umi):
    got = P.umi_complexity_one(umi, dinuc_order=1)
    exp = APPENDIX_A[umi]
    for f, e in zip(P.FIELDS, exp):
        assert got[f] == e, (umi, f, got[f], e)


@pytest.mark.parametrize("umi", list(APPENDIX_A))
def test_appendix_a_canonical_order_within_2ulp(umi):
    """The canonical (ascending pair) order differs from any HashMap order by <= 2 ULP
    on dinucleotide/combined only; all other fields exact."""
    got = P.umi_complexity_one(umi, dinuc_order=0)
    exp = APPENDIX_A[umi]
    for f, e in zip(P.FIELDS, exp):
        if f in ("dinucleotide_entropy", "combined_score"):
            assert _ulp_diff(got[f], e) <= 2, (umi, f)
        else:
            assert got[f] == e, (umi, f)


def test_empty_umi_is_x86_default_nan():
    r = P.umi_complexity_one(b"", 0)
    assert math.isnan(r["combined_score"])
    assert np.array([r["combined_score"]]).view(np.uint64)[0] == 0xFFF8000000000000
    assert r["longest_homopolymer_run"] == 0 and r["shannon_entropy"] == 0.0


def _random_bytes(rng, n, lengths, alphabet):
    return [bytes(rng.choice(list(alphabet), size=int(rng.choice(lengths))).astype(np.uint8)) for _ in range(n)]


@pytest.mark.parametrize("order", [0, 1])
def test_cpp_oracle_matches_python_restatement(order):
    rng = np.random.default_rng(1)
    umis = _random_bytes(rng, 300, list(range(0, 30)), b"ACGTNacgt")
    umis += _random_bytes(rng, 20, [64, 65, 80, 130], b"ACGT")  # DUST windows
    umis += _random_bytes(rng, 10, [100], b"AC")
    for u in umis:
        a = P.umi_complexity_one(u, order)
        b = P.py_umi_complexity(u, order)
        for f in P.FIELDS:
            va, vb = a[f], b[f]
            if isinstance(vb, float) and math.isnan(vb):
                assert math.isnan(va)
            else:
                assert va == vb, (u, f, va, vb)


def test_dust_nonzero_for_long_reads():
    r = P.umi_complexity_one(b"A" * 100, 0)
    # every 64-byte window holds 62 identical triplets: 62*61/2 pairs
    assert r["dust_score"] == 62 * 61 / 2
    assert r["combined_score"] == P.py_umi_complexity(b"A" * 100)["combined_score"]


def test_hamming_semantics():
    t = b"ACGTACGTACGT"
    assert P.py_hamming(b"ACGTACGTACGT", t) == 0
    assert P.py_hamming(b"ACGTACGTACGA", t) == 1
    assert P.py_hamming(b"ACGT", t) == 0xFFFFFFFF  # byte-length mismatch -> u32::MAX
    # same byte length, fewer chars: zip stops at the shorter char sequence
    assert P.py_hamming("ACGTACGTACé".encode(), t) == 1
    col = P.StrCol.from_list([b"ACGTACGTACGT", None, b"ACGTNCGTACGT", b"ACG", "ACGTACGTACé".encode()])
    d, w, valid = P.hamming(col, t, 1)
    assert list(valid) == [True, False, True, True, True]
    assert d[0] == 0 and d[2] == 1 and d[3] == 0xFFFFFFFF and d[4] == 1
    assert list(w[[0, 2, 3, 4]]) == [True, True, False, True]


@pytest.mark.parametrize("fixture", ["c1_clean", "c1_stress"])
def test_golden_vectors_reproduce(fixture):
    """The committed fixtures are exactly what the oracle computes (no drift)."""
    z = np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False)
    offs, vals, valid = z["offsets"], z["values"], z["valid"]
    n = len(valid)
    validity = None if valid.all() else np.packbits(valid, bitorder="little")
    col = P.StrCol(offs, vals, validity, n)
    res = P.umi_complexity(col)
    for f in P.FIELDS:
        a = res[f].view(np.uint64) if res[f].dtype == np.float64 else res[f]
        assert np.array_equal(a[valid], z["f_" + f][valid]), f
    for md in (0, 1):
        cid, cv, k, _ = P.umi_cluster(col, 12, md)
        assert k == int(z[f"n_clusters_{md}"][0])
        assert np.array_equal(cid[cv], z[f"cluster_{md}"][cv])


def test_golden_stress_covers_edge_cases():
    z = np.load(os.path.join(GOLDEN, "c1_stress.npz"), allow_pickle=False)
    lens = np.diff(z["offsets"])
    valid = z["valid"]
    assert (~valid).sum() >= 1  # nulls
    assert (lens[valid] == 0).any()  # empty string
    assert (lens[valid] >= 64).any()  # DUST windows
    assert (lens[valid] < 3).any()  # below the 3-mer window
    vals = z["values"]
    assert (vals == ord("N")).any() and (vals >= 0x80).any() and ((vals >= ord("a")) & (vals <= ord("z"))).any()


@pytest.mark.parametrize("md", [0, 1])
def test_cluster_oracle_vs_bruteforce(md):
    rng = np.random.default_rng(4 + md)
    umis = _random_bytes(rng, 1500, [5], b"ACGT")
    umis += [None, b"ACGTN", b"acgta", b"ACGT", b"ACGTAC", b"ACGTN"]
    ref, rk = P.py_cluster_bruteforce(umis, 5, md)
    cid, valid, k, L = P.umi_cluster(P.StrCol.from_list(umis), 5, md)
    assert L == 5 and k == rk
    assert [int(c) if v else None for c, v in zip(cid, valid)] == ref


def test_cluster_spec_properties():
    """Ids are dense, ordered by each cluster's smallest UMI, transitive for d=1; strings
    with N join the regular clusters they are 1 byte away from."""
    umis = [b"AAAA", b"AAAC", b"AACC", b"TTTT", b"GGGG", b"GGGA", b"CCCC", b"AAAN", b"AAAN", None, b"NNCN", b"NNNN"]
    cid, valid, k, _ = P.umi_cluster(P.StrCol.from_list(umis), 4, 1)
    ids = dict(zip(umis, cid))
    assert ids[b"AAAA"] == ids[b"AAAC"] == ids[b"AACC"] == ids[b"AAAN"] == 0  # AAAN ~ AAAA
    assert ids[b"CCCC"] == 1 and ids[b"GGGA"] == ids[b"GGGG"] == 2 and ids[b"TTTT"] == 3
    assert ids[b"NNCN"] == ids[b"NNNN"] == 4  # irregular-only cluster after the regular ones
    assert k == 5 and not valid[-3]
    cid0, _, k0, _ = P.umi_cluster(P.StrCol.from_list(umis), 4, 0)
    assert k0 == 10  # 7 distinct regular + 3 irregular


def test_cluster_irregular_bridges_regular_clusters():
    """AAGT ~ ANGT ~ ANNT ~ ACNT ~ ACAT: two regular clusters (2 bytes apart) merge
    through strings with N; the merged id is the one of the smaller code."""
    umis = [b"ACAT", b"AAGT", b"ANGT", b"ANNT", b"ACNT", b"TTTT"]
    cid, valid, k, _ = P.umi_cluster(P.StrCol.from_list(umis), 4, 1)
    assert list(cid) == [0, 0, 0, 0, 0, 1] and k == 2
    cid, valid, k, _ = P.umi_cluster(P.StrCol.from_list(umis[:2] + umis[5:]), 4, 1)
    assert list(cid) == [1, 0, 2] and k == 3
    # lowercase and other lengths: ordinary bytes; other lengths cluster among themselves
    umis = [b"acgt", b"acga", b"ACGTA", b"ACGTC", b"ACG", b"ACGT", b"aCGT"]
    cid, valid, k, _ = P.umi_cluster(P.StrCol.from_list(umis), 4, 1)
    ids = dict(zip(umis, cid))
    assert ids[b"ACGT"] == ids[b"aCGT"] == 0
    assert ids[b"acgt"] == ids[b"acga"] and ids[b"ACGTA"] == ids[b"ACGTC"]
    assert len({ids[b"ACG"], ids[b"ACGTA"], ids[b"acgt"], 0}) == 4 and k == 4


def test_cluster_oracle_threads_identical():
    """oracle_umi_cluster_mt (bench.py's multi-threaded CPU baseline) == the serial oracle."""
    from conftest import irregular_families
    from rogtk_amd import synth

    cols = [P.StrCol.from_fixed(synth.umi_ascii(300_000, 12, p_n=1e-3, p_lower=5e-4)),
            P.StrCol.from_list(irregular_families(9, 3000, 10))]
    for col in cols:
        for md in (0, 1):
            ref = P.umi_cluster(col, 0, md, threads=1)
            for t in (2, 7, 16):
                got = P.umi_cluster(col, 0, md, threads=t)
                assert got[2] == ref[2] and np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])


@pytest.mark.parametrize("seed,L,utf8", [(1, 4, 0), (2, 6, 0), (3, 12, 0), (4, 20, 0), (5, 33, 0), (6, 6, 0.1),
                                         (7, 12, 0.1)])
def test_cluster_oracle_vs_bruteforce_irregular_families(seed, L, utf8):
    """utf8 > 0: multi-byte UTF-8 members; H3 is byte-wise, so the pin pair
    A^(L-2)+U+00E9 / A^L has H2.1 distance 1 (py_hamming zips chars) but no H3 edge."""
    from conftest import irregular_families

    umis = irregular_families(seed, 120 if L <= 6 else 250, L, p_utf8=utf8)
    for md in (0, 1):
        ref, rk = P.py_cluster_bruteforce(umis, L, md)
        cid, valid, k, rl = P.umi_cluster(P.StrCol.from_list(umis), L, md)
        assert rl == L and k == rk
        assert [int(c) if v else None for c, v in zip(cid, valid)] == ref
        if utf8 and md == 1:
            assert ref[-2] != ref[-1]
    if utf8:
        d, _, _ = P.hamming(P.StrCol.from_list(umis[-2:]), b"A" * L, 1)
        assert list(d) == [1, 0]


# ---------------------------------------------------------------- H4 k-mer oracle
def test_kmer_oracle_matches_python_restatement():
    """oracle/kmer_oracle.cpp vs the independent Python restatement (pyoracle.py)."""
    import random

    rng = random.Random(1)
    for trial in range(300):
        items = []
        for _ in range(rng.randint(0, 12)):
            if rng.random() < 0.1:
                items.append(None)
                continue
            alpha = b"ACGTacgtN" if rng.random() < 0.2 else b"ACGT"
            items.append(bytes(rng.choice(alpha) for _ in range(rng.randint(0, 40))))
        k = rng.choice([0, 1, 3, 4, 5, 8, 9, 16, 17, 31, 32, 33, 64, 65])
        mc = rng.choice([0, 1, 1, 2, 3])
        ak = rng.random() < 0.2
        r = P.kmer_spectrum(P.StrCol.from_list(items), k, mc, ak)
        py, st = P.py_kmer_spectrum(items, k, mc, ak)
        got = [(P.kmer_to_str(h, l, st[0]), int(e), int(c))
               for h, l, e, c in zip(r["kmer_hi"], r["kmer_lo"], r["exts"], r["counts"])]
        assert got == py and tuple(r["stats"][0]) == st, (trial, items, k, mc, ak)


def test_kmer_oracle_reference_fixture():
    """fracture.rs:611-626: the two test reads assemble to the 44-bp contig in the
    comment; at k=13 (effective 16) their valid k-mers are exactly its 29 16-mers,
    forming one unbranched path (2 terminal ends, 0 isolated)."""
    seqs = [b"GAGACTGCATGGGCTGGTGGGCGTCCGTCTGC", b"GGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"]
    r = P.kmer_spectrum(P.StrCol.from_list(seqs), 13, 1)
    contig = "GAGACTGCATGGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"
    want = sorted({contig[i:i + 16] for i in range(len(contig) - 15)})
    have = [P.kmer_to_str(h, l, 16) for h, l in zip(r["kmer_hi"], r["kmer_lo"])]
    assert have == want
    assert tuple(r["stats"][0]) == (16, 2, 29, 2, 0)
    # k=4 (fracture.rs:685 test_compare_assembly_methods): non-empty spectrum
    r4 = P.kmer_spectrum(P.StrCol.from_list(seqs), 4, 1)
    assert r4["stats"][0][0] == 4 and r4["stats"][0][2] > 0


# ---------------------------------------------------------------- H5 assembly restatement
def test_assembly_restatement_reference_tests():
    """oracle/pyassembly.py against the reference's own assembly tests (fracture.rs:593-761)."""
    from oracle import pyassembly as A

    seqs = [b"GAGACTGCATGGGCTGGTGGGCGTCCGTCTGC", b"GGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"]
    # :630-681 + the expected contig in the comment at :611
    assert A.assemble(seqs, 13, 1, "shortest_path", "GAGACTGCATGG", "TTTAGTGAGGGT") == [
        "GAGACTGCATGGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"]
    # :684-707 anchors absent -> no contig
    assert A.assemble([b"AAAACCCCCAAAAA", b"TTTTTGGGGGTTTT"], 4, 1, "shortest_path", "NONEXISTENT",
                      "ALSONOTHERE") == []
    # :710-761 compression at k=4 yields a contig
    assert A.assemble(seqs, 4, 1, "compression") != []
    # Rust std BinaryHeap order (sift_up / sift_down_to_bottom) of the restated heap
    h = A.RustHeap()
    for s in (3.0, 1.0, 2.0, 1.0, 5.0, 0.5):
        h.push((s, int(s * 10)))
    assert [h.pop()[0] for _ in range(6)] == [0.5, 1.0, 1.0, 2.0, 3.0, 5.0]
