"""GPU: bench.py's launcher and BASELINE config C4's per-rank shard.

* `python bench.py --gpus 2` with no WORLD_SIZE starts the two ranks itself
  (rogtk_amd.launch); on a one-GPU box they share cuda:0 over gloo
  (ROGTK_DIST_BACKEND=gloo, tests only). The JSON line must report the world size the
  process group saw.
* C4 = 500M reads over 8 GPUs: one rank's 62.5M-read shard runs through UmiPipeline
  exactly as bench.py --workload C4 --gpus 8 runs it per rank, against the all-gathered
  bitmaps of all 8 shards (the other 7 built on the same GPU). Every output is compared:
  H1/H2 on the distinct codes broadcast back (a regular row's scores are a function of its
  code), H3 against the oracle's union-find over the union's distinct codes (ids depend
  only on the global distinct set), mapped back to the rows.
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


@pytest.mark.timeout(900)
def test_c4_rank_of_8_against_the_union():
    """C4 at N = 8 (500M reads, 62.5M per rank), emulated on one GPU exactly as each rank
    runs it: rank 3's shard goes through UmiPipeline (bench.py's defaults) with the
    exchange returning the all-gathered bitmaps of all 8 shards (the other 7 built here,
    ~95% of the 4^12 codes present in their union). Every output is compared: all 7 H1
    fields and the Hamming-within bits on the rank's distinct codes (a regular row's scores
    are a function of its code), and the ids against the oracle's union-find over the
    union's distinct codes (ids depend only on the global distinct set)."""
    import torch

    import bench
    from oracle import pyoracle as P
    from rogtk_amd import device as D
    from rogtk_amd import dist as RD
    from rogtk_amd import synth
    from rogtk_amd.pipeline import UmiPipeline

    n_total, world, rank, L = 500_000_000, 8, 3, 12
    dev = torch.device("cuda", 0)
    bitmaps = [bench.emulated_shard_bitmap(n_total, r, world, L, dev) if r != rank else None for r in range(world)]
    start, count = RD.shard_range(n_total, rank, world)
    assert count == 62_500_000
    codes_h = synth.umi_codes(n_total, L, start=start, count=count)
    codes = torch.from_numpy(codes_h.view(np.int32)).to(dev)
    batch = D.PackedBatch(codes, L)
    gathered = torch.zeros(world * bitmaps[0].numel(), dtype=bitmaps[0].dtype, device=dev)
    for r in range(world):
        if r != rank:
            gathered[r * bitmaps[0].numel():(r + 1) * bitmaps[0].numel()].copy_(bitmaps[r])

    def exchange(bm):  # the all-gather of rank `rank`: its own bitmap in its slot
        gathered[rank * bm.numel():(rank + 1) * bm.numel()].copy_(bm)
        return gathered, world

    pipe = UmiPipeline(L, min(n_total, 4 ** L), count, dev, depth=2, target=b"ACGTACGTACGT", max_distance=1,
                       score_alone=True, exchange=exchange)
    slot = pipe.submit(batch)
    pipe.drain()
    torch.cuda.synchronize()
    got = {f: slot.scores[f][:count].cpu().numpy() for f in P.FIELDS}
    cid = slot.cid[:count].cpu().numpy().view(np.uint32)
    within = np.unpackbits(slot.within.cpu().numpy().view(np.uint8), bitorder="little")[:count].astype(bool)
    stats = slot.eng.stats()
    del pipe, slot, batch, codes, gathered, bitmaps
    torch.cuda.empty_cache()
    print(f"C4 rank {rank} of {world} on GPU done: {stats}", flush=True)
    # H1 / H2 on the rank's distinct codes
    uniq, inv = np.unique(codes_h, return_inverse=True)
    ucol = P.StrCol.from_fixed(synth.codes_to_ascii(uniq, L))
    ref = P.umi_complexity(ucol)
    for f in P.FIELDS:
        r = ref[f]
        g = got[f]
        if r.dtype == np.float64:
            assert np.array_equal(g.view(np.uint64), r.view(np.uint64)[inv]), f
        else:
            assert np.array_equal(g.view(np.uint32), r.astype(np.uint32)[inv]), f
    _, rw, _ = P.hamming(ucol, b"ACGTACGTACGT", 1)
    assert np.array_equal(within, rw[inv])
    del ucol, ref
    # H3 over the union of the 8 shards' distinct codes
    union = uniq
    for r in range(world):
        if r != rank:
            s0, c0 = RD.shard_range(n_total, r, world)
            union = np.union1d(union, np.unique(synth.umi_codes(n_total, L, start=s0, count=c0)))
    assert stats["n_distinct"] == len(union) and len(union) > 0.9 * 4 ** L
    threads = min(16, os.cpu_count() or 1)
    rc, _, rk, _ = P.umi_cluster(P.StrCol.from_fixed(synth.codes_to_ascii(union, L)), L, 1, threads=threads)
    print(f"oracle H3 on the union's {len(union)} distinct codes done", flush=True)
    assert stats["n_clusters"] == rk and stats["overflow"] == 0
    assert np.array_equal(cid, rc[np.searchsorted(union, codes_h)])
