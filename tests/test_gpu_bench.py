"""GPU: bench.py's launcher and BASELINE config C4's per-rank shard.

* `python bench.py --gpus 2` with no WORLD_SIZE starts the two ranks itself
  (rogtk_amd.launch); on a one-GPU box they share cuda:0 over gloo
  (ROGTK_DIST_BACKEND=gloo, tests only). The JSON line must report the world size the
  process group saw.
* C4 = 500M reads over 8 GPUs: one rank's 62.5M-read shard runs through UmiPipeline
  exactly as bench.py --workload C4 --gpus 8 runs it per rank. H1/H2 are checked on the
  distinct codes broadcast back (a regular row's scores are a function of its code), H3
  against the oracle's union-find over the shard's distinct codes (ids depend only on the
  distinct set), mapped back to the rows.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _last_json(text):
    for line in reversed(text.strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError("no JSON line:\n" + text[-2000:])


def test_bench_launcher_two_ranks():
    env = dict(os.environ, ROGTK_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--reads-per-gpu", "1000000", "--no-cpu-baseline", "--iso-launches", "2"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["config"]["total_reads"] == 2_000_000
    assert line["value"] > 0 and line["scaling"] == "weak"


def test_c4_rank_shard_62m():
    import torch

    from oracle import pyoracle as P
    from rogtk_amd import device as D
    from rogtk_amd import dist as RD
    from rogtk_amd import synth
    from rogtk_amd.pipeline import UmiPipeline

    n_total, world, rank, L = 500_000_000, 8, 3, 12
    start, count = RD.shard_range(n_total, rank, world)
    assert count == 62_500_000
    codes_h = synth.umi_codes(n_total, L, start=start, count=count)
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    pipe = UmiPipeline(L, min(n_total, 4 ** L), count, "cuda", depth=2, target=b"ACGTACGTACGT", max_distance=1,
                       score_alone=True)
    slot = pipe.submit(batch)
    pipe.drain()
    torch.cuda.synchronize()
    cid = slot.cid[:count].cpu().numpy().view(np.uint32)
    comb = slot.scores["combined_score"][:count].cpu().numpy().view(np.uint64)
    longest = slot.scores["longest_homopolymer_run"][:count].cpu().numpy().view(np.uint32)
    within = np.unpackbits(slot.within.cpu().numpy().view(np.uint8), bitorder="little")[:count].astype(bool)
    stats = slot.eng.stats()
    del pipe, slot, batch, codes
    print(f"C4 shard on GPU done: {stats}", flush=True)
    uniq, inv = np.unique(codes_h, return_inverse=True)
    ucol = P.StrCol.from_fixed(synth.codes_to_ascii(uniq, L))
    threads = min(16, os.cpu_count() or 1)
    rc, _, rk, _ = P.umi_cluster(ucol, L, 1, threads=threads)
    print(f"oracle H3 on {len(uniq)} distinct codes done", flush=True)
    assert stats["n_clusters"] == rk and stats["overflow"] == 0
    assert np.array_equal(cid, rc[inv])
    ref = P.umi_complexity(ucol)
    assert np.array_equal(comb, ref["combined_score"].view(np.uint64)[inv])
    assert np.array_equal(longest, ref["longest_homopolymer_run"].astype(np.uint32)[inv])
    _, rw, _ = P.hamming(ucol, b"ACGTACGTACGT", 1)
    assert np.array_equal(within, rw[inv])
