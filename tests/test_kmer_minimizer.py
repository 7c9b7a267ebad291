"""CPU check of the minimizer filter's argument (kmer_kernels.hip
k_minimizer_filter): in a group whose rows all carry the repeat certificate, a K-mer
(K = 31, 32) counted min_coverage times implies a window minimizer (the smallest 16-mer of
a window of K - 15 of them, as a 2-bit code) counted min_coverage times, each row adding a
minimizer once per run of consecutive windows that share it. Brute force over groups of
random templates read at shifted offsets with errors; a poly-A row shows why the rows must
be certified. (The GPU filter is pinned by the oracle in tests/test_gpu_c3.py.)"""
import random
from collections import Counter

from test_kmer_cert import norep

CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def code16(s: str) -> int:
    v = 0
    for ch in s:
        v = (v << 2) | CODE[ch]
    return v


def kmer_counts(rows, k):
    c = Counter()
    for r in rows:
        for p in range(len(r) - k + 1):
            c[r[p:p + k]] += 1
    return c


def minimizer_counts(rows, k):
    """What the filter counts: per row, a window's minimizer added once per run of
    consecutive windows that share it."""
    c = Counter()
    w = k - 15
    for r in rows:
        h = [code16(r[q:q + 16]) for q in range(len(r) - 15)]
        prev = None
        for p in range(len(r) - k + 1):
            m = min(h[p:p + w])
            if m != prev:
                c[m] += 1
            prev = m
    return c


def _group(rnd, mc):
    rows = []
    for _ in range(rnd.randint(1, 4)):  # templates, each read 1..2 mc times at offsets
        tpl = "".join(rnd.choice("ACGT") for _ in range(rnd.randint(150, 200)))
        for _ in range(rnd.randint(1, 2 * mc)):
            L = rnd.randint(60, 150)
            o = rnd.randint(0, len(tpl) - L)
            x = list(tpl[o:o + L])
            for _ in range(rnd.randint(0, 2)):
                x[rnd.randrange(L)] = rnd.choice("ACGT")
            rows.append("".join(x))
    return rows


def test_minimizer_filter_is_sound_on_certified_groups():
    rnd = random.Random(5)
    checked = filtered = kept_valid = 0
    for g in range(300):
        mc = rnd.choice((2, 3, 5, 8))
        rows = _group(rnd, mc)
        if not all(norep(r) for r in rows):
            continue
        for k in (31, 32):
            valid = max(kmer_counts(rows, k).values(), default=0) >= mc
            passes = max(minimizer_counts(rows, k).values(), default=0) >= mc
            assert passes or not valid, (g, k, mc)  # empty by the filter => nothing valid
            checked += 1
            filtered += not passes
            kept_valid += valid
    assert checked > 300 and filtered > 50 and kept_valid > 50, (checked, filtered, kept_valid)


def test_filter_needs_certified_rows():
    """A poly-A row holds A^32 (len - 31) times but its every window shares one minimizer,
    counted once: without the row certificate the count would not bound the K-mer's."""
    row = "A" * 60
    assert not norep(row)
    assert kmer_counts([row], 32)["A" * 32] == 29
    assert minimizer_counts([row], 32)[0] == 1
