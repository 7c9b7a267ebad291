#!/usr/bin/env python3
"""Level-2 (host Arrow buffers) rates, PCIe included: what a polars plugin sees.

Times the three host entry points on a 10M-row pyarrow UMI column (synth-v1 C2
UMIs as 12-byte strings): H2D copy of the column, the kernels and the D2H copy
of the results are all inside the timed region. Never bench.py's `value`.
"""
import json
import os
import sys
import time

import numpy as np
import pyarrow as pa

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rogtk_amd as rg  # noqa: E402
from rogtk_amd import synth  # noqa: E402


def timed(fn, reps=3):
    fn()  # warm (allocations, LUT upload)
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t)
    return best


def main():
    n = int(os.environ.get("N", "10000000"))
    L = 12
    umis = synth.umi_ascii(n, L)
    offsets = pa.py_buffer((np.arange(n + 1, dtype=np.int64) * L).tobytes())
    col = pa.Array.from_buffers(pa.large_binary(), n, [None, offsets, pa.py_buffer(umis.reshape(-1).tobytes())])
    out = {}
    out["umi_complexity_host"] = n / timed(lambda: rg.umi_complexity_scores(col))
    out["hamming_host"] = n / timed(lambda: rg.hamming_within(col, "ACGTACGTACGT", 1))
    out["umi_cluster_host"] = n / timed(lambda: rg.umi_cluster(col, L, 1))
    print(json.dumps({"metric": "Level-2 host-buffer rate (PCIe H2D + kernels + D2H), rows/s", "rows": n,
                      "rates": {k: round(v, 1) for k, v in out.items()},
                      "note": "pyarrow column in host memory; results copied back into Arrow buffers"}))


if __name__ == "__main__":
    main()
