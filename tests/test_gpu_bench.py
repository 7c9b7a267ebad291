"""GPU: bench.py's launcher and BASELINE config C4's per-rank shard.

* `python bench.py --gpus 2` with no WORLD_SIZE starts the two ranks itself
  (rogtk_amd.launch); on a one-GPU box they share cuda:0 over gloo
  (ROGTK_DIST_BACKEND=gloo, tests only). The JSON line must report the world size the
  process group saw.
* C2 weak scaling at N = 8 (10M reads per rank): one rank's ids against the oracle over the
  union of the 8 shards, at 12 bp (one cluster) and 13 bp (36,893 clusters).
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


def _rank_of_world(n_total, world, rank, L, scores=True):
    """Rank `rank` of `world` emulated on one GPU exactly as it runs under bench.py: its shard
    through UmiPipeline (bench.py's defaults) with the exchange returning the all-gathered
    bitmaps of every shard (the others built here, as bench.emulated_shard_bitmap does).
    Returns (codes_h, slot outputs, stats, union): union = the sorted distinct codes of all
    shards, from a presence array torch fills on the device (index_put; none of the
    library's kernels), each shard's codes generated once."""
    import torch

    from oracle import pyoracle as P
    from rogtk_amd import device as D
    from rogtk_amd import dist as RD
    from rogtk_amd import synth
    from rogtk_amd.pipeline import UmiPipeline

    import time

    t0 = time.perf_counter()
    dev = torch.device("cuda", 0)
    present = torch.zeros(4 ** L, dtype=torch.bool, device=dev)
    nw = 4 ** L // 64
    gathered = torch.zeros(world * nw, dtype=torch.int64, device=dev)
    for r in range(world):
        if r == rank:
            continue
        s0, c0 = RD.shard_range(n_total, r, world)
        cr = torch.from_numpy(synth.umi_codes(n_total, L, start=s0, count=c0).view(np.int32)).to(dev)
        present[cr.long()] = True
        eng = D.ClusterEngine(L, min(n_total, 4 ** L), dev)
        eng.mark(D.PackedBatch(cr, L))
        gathered[r * nw:(r + 1) * nw].copy_(eng.build_local_bitmap())
        del cr, eng
    start, count = RD.shard_range(n_total, rank, world)
    codes_h = synth.umi_codes(n_total, L, start=start, count=count)
    codes = torch.from_numpy(codes_h.view(np.int32)).to(dev)
    present[codes.long()] = True
    union = torch.nonzero(present).flatten().to(torch.int64).cpu().numpy().astype(np.uint32)
    del present
    print(f"shards and union ({time.perf_counter() - t0:.1f} s)", flush=True)
    batch = D.PackedBatch(codes, L)

    def exchange(bm):  # the all-gather of rank `rank`: its own bitmap in its slot
        gathered[rank * nw:(rank + 1) * nw].copy_(bm)
        return gathered, world

    pipe = UmiPipeline(L, min(n_total, 4 ** L), count, dev, depth=2, target=b"ACGTACGTACGT", max_distance=1,
                       score_alone=True, exchange=exchange, with_scores=scores)
    slot = pipe.submit(batch)
    pipe.drain()
    torch.cuda.synchronize()
    out = {"cid": slot.cid[:count].cpu().numpy().view(np.uint32)}
    if scores:
        out.update({f: slot.scores[f][:count].cpu().numpy() for f in P.FIELDS})
        out["within"] = np.unpackbits(slot.within.cpu().numpy().view(np.uint8), bitorder="little")[:count].astype(bool)
    stats = slot.eng.stats()
    del pipe, slot, batch, codes, gathered
    torch.cuda.empty_cache()
    return codes_h, out, stats, union


def _check_union_ids(codes_h, cid, stats, union, L):
    from oracle import pyoracle as P
    from rogtk_amd import synth

    threads = min(16, os.cpu_count() or 1)
    rc, _, rk, _ = P.umi_cluster(P.StrCol.from_fixed(synth.codes_to_ascii(union, L)), L, 1, threads=threads)
    assert stats["n_distinct"] == len(union)
    assert stats["n_clusters"] == rk and stats["overflow"] == 0
    assert np.array_equal(cid, rc[np.searchsorted(union, codes_h)])
    return rk


@pytest.mark.timeout(600)
def test_c4_rank_of_8_against_the_union():
    """C4 at N = 8 (500M reads, 62.5M per rank), emulated on one GPU exactly as each rank
    runs it: rank 3's shard goes through UmiPipeline (bench.py's defaults) with the
    exchange returning the all-gathered bitmaps of all 8 shards (the other 7 built here,
    ~95% of the 4^12 codes present in their union). Every output is compared: all 7 H1
    fields and the Hamming-within bits on the rank's distinct codes (a regular row's scores
    are a function of its code), and the ids against the oracle's union-find over the
    union's distinct codes (ids depend only on the global distinct set). At this density
    the union is one cluster: the non-degenerate N = 8 ids are the C2 test below."""
    from oracle import pyoracle as P
    from rogtk_amd import synth

    import time

    t0 = time.perf_counter()
    n_total, world, rank, L = 500_000_000, 8, 3, 12
    codes_h, got, stats, union = _rank_of_world(n_total, world, rank, L)
    assert len(codes_h) == 62_500_000
    print(f"C4 rank {rank} of {world} on GPU done ({time.perf_counter() - t0:.1f} s): {stats}", flush=True)
    # H1 / H2 on the rank's distinct codes (distinct set and row -> distinct index from a
    # presence array: no sort of the 62.5M codes)
    pres = np.zeros(4 ** L, dtype=bool)
    pres[codes_h] = True
    uniq = np.flatnonzero(pres).astype(np.uint32)
    inv = (np.cumsum(pres, dtype=np.int64) - 1)[codes_h]
    del pres
    threads = min(16, os.cpu_count() or 1)
    ucol = P.StrCol.from_fixed(synth.codes_to_ascii(uniq, L))
    ref = P.umi_complexity(ucol, threads=threads)
    for f in P.FIELDS:
        r = ref[f]
        g = got[f]
        if r.dtype == np.float64:
            assert np.array_equal(g.view(np.uint64), r.view(np.uint64)[inv]), f
        else:
            assert np.array_equal(g.view(np.uint32), r.astype(np.uint32)[inv]), f
    _, rw, _ = P.hamming(ucol, b"ACGTACGTACGT", 1)
    assert np.array_equal(got["within"], rw[inv])
    del ucol, ref, uniq, inv
    print(f"H1/H2 checked ({time.perf_counter() - t0:.1f} s)", flush=True)
    assert len(union) > 0.9 * 4 ** L
    # H3 against the oracle's union-find over the union, pinned in a fixture
    # (tools/gen_union_fixture.py: 45 s of oracle at this density): the same union (size and
    # digest), one cluster, so every id is 0
    with open(os.path.join(ROOT, "tests", "golden", "c4_union_x8.json")) as f:
        fx = json.load(f)
    digest = int(np.bitwise_xor.reduce(union.astype(np.uint64) * np.uint64(0x9E3779B1)))
    assert (fx["n_total"], fx["world"], fx["umi_len"]) == (n_total, world, L)
    assert len(union) == fx["n_distinct"] and digest == fx["union_digest"]
    assert stats["n_distinct"] == fx["n_distinct"] and stats["n_clusters"] == fx["n_clusters"]
    assert stats["overflow"] == 0 and fx["max_cluster_id"] == 0
    assert int(got["cid"].max()) == 0 and int(got["cid"].min()) == 0
    print(f"H3 checked ({time.perf_counter() - t0:.1f} s)", flush=True)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("L,min_clusters", [(12, 1), (13, 10_000)])
def test_c2_weak_scaling_rank_of_8_union(L, min_clusters):
    """C2 weak scaling at N = 8 (what bench.py --gpus 8 runs: 10M reads per rank, 80M in all),
    rank 5 emulated on one GPU against the all-gathered bitmaps of the 8 shards; the ids
    against the oracle's union-find over the union's distinct codes. At 12 bp the union is
    41% of the code space and Hamming-1 joins all of it into ONE cluster (6.94M codes; a
    site percolation far above threshold: 36 neighbours per code), so the same shards with
    13-bp UMIs (12.6% dense, 36,893 clusters, the largest 8.41M codes) pin the merge where
    the answer is not degenerate."""
    n_total, world, rank = 80_000_000, 8, 5
    codes_h, got, stats, union = _rank_of_world(n_total, world, rank, L, scores=False)
    assert len(codes_h) == 10_000_000
    print(f"C2 x8 rank {rank}, {L} bp: {stats}", flush=True)
    rk = _check_union_ids(codes_h, got["cid"], stats, union, L)
    assert rk >= min_clusters
    if L == 13:
        assert rk > 10_000 and len(np.unique(got["cid"])) > 10_000
