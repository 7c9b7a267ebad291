"""Generate the committed golden vectors under tests/golden/ (run on CPU).

The reference (Rust + polars plugin) cannot be built or imported in this image
(SURVEY.md §8c), so the vectors come from the C++ oracle (oracle/rogtk_oracle.cpp),
which is itself pinned by SURVEY.md Appendix A's hand-derived known answers
(tests/test_oracle.py) and cross-checked against an independent pure-Python
restatement. The inputs are stored explicitly, so the fixtures do not depend on
the synthetic generator staying byte-stable.

Fixtures (npz, allow_pickle=False):
  c1_clean.npz   config C1: 10,000 synthetic 12-bp UMIs (synth-v1), no N
  c1_stress.npz  10,000 UMIs with N (p=5e-3/base), lowercase (2e-3/base), plus hand
                 edge cases: nulls, empty, short (1..3 bytes), long (64..300 bytes,
                 DUST windows), non-ASCII UTF-8, other lengths.
Each holds: offsets int64[n+1], values u8, valid bool[n]; every complexity field
(f64 as raw u64 bits); hamming distance/within for TARGETS; cluster ids + counts
for max_distance 0 and 1 (umi_len 12).

Usage: python tests/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import pyoracle as P  # noqa: E402
from rogtk_amd import synth  # noqa: E402

TARGETS = [b"ACGTACGTACGT", b"AAAAAAAAAAAA", b"ACGTNACGTACG", b"ACGT", "ACGTACGTACGé".encode(),
           "éCGTACGTAC".encode()]


def edge_cases():
    rng = np.random.default_rng(7)
    e = [None, b"", b"A", b"AC", b"ACG", b"NNNN", b"acgt", b"ACGTN", "ACGTéACGTAC".encode(),
         "日本語ACGTAC".encode(), b"ACGTACGTACGTA", b"ACGTACGTACG"]
    for L in (63, 64, 65, 80, 150, 300):
        e.append(rng.choice(list(b"ACGT"), size=L).astype(np.uint8).tobytes())
        e.append(b"ACGTTT" * (L // 6) + b"A" * (L % 6))
    e.append(b"A" * 150)
    e.append(b"AC" * 75)
    return e


def make(name: str, umis, path: str):
    col = P.StrCol.from_list(umis)
    out = {"offsets": col.offsets, "values": col.values, "valid": col.valid_mask()}
    res = P.umi_complexity(col)
    for f in P.FIELDS:
        a = res[f]
        out["f_" + f] = a.view(np.uint64) if a.dtype == np.float64 else a
    for k, t in enumerate(TARGETS):
        d, w, _ = P.hamming(col, t, 1)
        out[f"ham_target_{k}"] = np.frombuffer(t, dtype=np.uint8)
        out[f"ham_dist_{k}"] = d
        out[f"ham_within_{k}"] = w
    for md in (0, 1):
        cid, cvalid, k, L = P.umi_cluster(col, 12, md)
        out[f"cluster_{md}"] = cid
        out[f"cluster_valid_{md}"] = cvalid
        out[f"n_clusters_{md}"] = np.array([k], dtype=np.int64)
    np.savez_compressed(path, **out)
    print(f"{name}: {len(umis)} rows -> {path} ({os.path.getsize(path)} bytes)")


def main():
    gdir = os.path.join(ROOT, "tests", "golden")
    os.makedirs(gdir, exist_ok=True)
    n = 10_000
    clean = [bytes(r) for r in synth.umi_ascii(n, 12)]
    make("c1_clean", clean, os.path.join(gdir, "c1_clean.npz"))
    stress = [bytes(r) for r in synth.umi_ascii(n, 12, p_n=5e-3, p_lower=2e-3, seed=synth.DEFAULT_SEED + 1)]
    ec = edge_cases()
    idx = np.random.default_rng(11).choice(n, size=len(ec), replace=False)
    for i, e in zip(sorted(idx), ec):
        stress[i] = e
    make("c1_stress", stress, os.path.join(gdir, "c1_stress.npz"))
    # Appendix A known answers, first-occurrence dinucleotide order (as printed there)
    kats = [b"AAAAAAAAAAAA", b"ACGTACGTACGT", b"AACCGGTTAACC", b"ACGTTGCAACGT", b"GATTACAGATTA",
            b"NNNNNNNNNNNN", b"ACGTNACGTACG", b"acgtacgtacgt"]
    print("Appendix A rows (first-occurrence order):")
    for k in kats:
        r = P.umi_complexity_one(k, 1)
        print(k.decode(), [repr(float(r[f])) if f != "longest_homopolymer_run" else r[f] for f in P.FIELDS])


if __name__ == "__main__":
    main()
