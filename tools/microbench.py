"""Kernel-level micro-benchmarks on the GPU box (not part of the product).

Times each phase of the hot path in isolation with torch events around calls on
torch's current stream, plus reference ceilings (torch fill / copy) for the
achievable HBM write and copy bandwidth on this device.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rogtk_amd import device as D  # noqa: E402
from rogtk_amd import synth  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1000.0  # us


def main():
    n = int(os.environ.get("N", 10_000_000))
    L = 12
    res = {}
    big = torch.empty(n * 7, dtype=torch.float64, device="cuda")
    us = timeit(lambda: big.fill_(1.0))
    res["torch_fill_GBps"] = big.numel() * 8 / us / 1e3
    src = torch.empty(n * 7, dtype=torch.float64, device="cuda").fill_(2.0)
    us = timeit(lambda: big.copy_(src))
    res["torch_copy_GBps(r+w)"] = 2 * big.numel() * 8 / us / 1e3
    del big, src
    codes = torch.from_numpy(synth.umi_codes(n, L).view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    scores = D.alloc_scores(n, "cuda")
    within = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    eng = D.ClusterEngine(L, n, "cuda")
    t = b"ACGTACGTACGT"
    res["score_only_us"] = timeit(lambda: D.score_packed(batch, scores))
    res["score_within_us"] = timeit(lambda: D.score_packed(batch, scores, t, 1, None, within))
    res["score_within_mark_us"] = timeit(lambda: (D.score_packed(batch, scores, t, 1, None, within, cluster=eng),
                                                  eng.build_local_bitmap()))
    res["mark_only_us"] = timeit(lambda: (eng.mark(batch), eng.build_local_bitmap()))
    res["bitmap_only_us"] = timeit(lambda: eng.build_local_bitmap())
    eng.mark(batch)
    bm = eng.build_local_bitmap().clone()
    for md in (0, 1):
        res[f"resolve_md{md}_us"] = timeit(lambda: eng.resolve(bm, 1, md))
    res["assign_us"] = timeit(lambda: eng.assign(batch, cid))
    D.profile_reset()
    D.profile_enable(True)
    for _ in range(5):
        eng.resolve(bm, 1, 1)
    torch.cuda.synchronize()
    D.profile_enable(False)
    for k in ("cluster_scan", "cluster_compact", "cluster_union", "cluster_flatten", "cluster_label"):
        ms, c = D.profile_read(k)
        res[f"resolve_{k}_us"] = 1000 * ms / max(c, 1)
    bpr = 56.125
    res["score_within_GBps"] = n * bpr / res["score_within_us"] / 1e3
    res["score_only_GBps"] = n * 56 / res["score_only_us"] / 1e3
    print(json.dumps({k: round(v, 2) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
