#!/usr/bin/env python3
"""Writes tests/golden/c4_union_x8.json: the oracle's H3 over the union of the 8 shards of
BASELINE C4 (500M synth-v1 reads, 12-bp UMIs, Hamming <= 1). The union covers 96.4% of the
code space and is one cluster; tests/test_gpu_bench.py::test_c4_rank_of_8_against_the_union
checks the device run against this fixture instead of re-running the 45-s oracle union-find
on every GPU test pass (the non-degenerate N = 8 ids are checked against the oracle live,
at 13 bp, by test_c2_weak_scaling_rank_of_8_union). Test infrastructure: oracle only."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as P  # noqa: E402
from rogtk_amd import dist as RD  # noqa: E402
from rogtk_amd import synth  # noqa: E402


def main():
    n_total, world, L = 500_000_000, 8, 12
    present = np.zeros(4 ** L, dtype=bool)
    for r in range(world):
        s0, c0 = RD.shard_range(n_total, r, world)
        present[synth.umi_codes(n_total, L, start=s0, count=c0)] = True
    union = np.flatnonzero(present).astype(np.uint32)
    rc, _, rk, _ = P.umi_cluster(P.StrCol.from_fixed(synth.codes_to_ascii(union, L)), L, 1,
                                 threads=os.cpu_count() or 1)
    sizes = np.bincount(rc)
    out = {"config": "C4: 500M synth-v1 reads (seed default), 8 shards, 12-bp UMIs, max_distance 1",
           "n_total": n_total, "world": world, "umi_len": L, "max_distance": 1,
           "n_distinct": int(len(union)), "n_clusters": int(rk), "largest_cluster": int(sizes.max()),
           "max_cluster_id": int(rc.max()), "union_digest": int(np.bitwise_xor.reduce(union.astype(np.uint64) *
                                                                                     np.uint64(0x9E3779B1)))}
    path = os.path.join(ROOT, "tests", "golden", "c4_union_x8.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
