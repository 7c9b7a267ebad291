"""GPU: rogtk_amd.dist.umi_cluster_sharded with the HIP steps (rogtk_amd/csrc/dist_cluster.hip).

world 1 in-process, and world 2 as two gloo ranks sharing cuda:0 (collective buffers
staged on the host; the same exchange plan the driver runs over RCCL). Ids must equal
the oracle on the whole column and the single-GPU engines (umi_cluster).
"""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_dist_sharded import _arrow, _free_port, make_column

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rg():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import rogtk_amd

    assert rogtk_amd.device_count() >= 1
    return rogtk_amd


@pytest.mark.parametrize("L,md,n,irr", [(12, 1, 30_000, 0), (12, 0, 30_000, 0), (20, 1, 30_000, 0),
                                        (32, 1, 20_000, 0), (7, 1, 5_000, 0), (1, 1, 300, 0), (16, 1, 40_000, 0),
                                        (6, 1, 3_000, 1), (12, 1, 3_000, 1), (24, 1, 3_000, 1)])
def test_sharded_world1_matches_oracle_and_engine(rg, L, md, n, irr):
    """irr: N / lowercase / length-change families (Hamming-1 edges of irregular strings)."""
    import pyarrow as pa

    from oracle import pyoracle as P
    from rogtk_amd import dist as RD

    col = make_column(n, L, seed=-(L * 3 + md) if irr else L * 3 + md)
    off, vals, vbits = (t.cuda() for t in _arrow(col))
    cid, k = RD.umi_cluster_sharded(off, vals, n, L, md, validity=vbits)
    torch.cuda.synchronize()
    got = cid.cpu().numpy().view(np.uint32)
    ref, valid, rk, _ = P.umi_cluster(P.StrCol.from_list(col), L, md)
    assert k == rk
    assert np.array_equal(got[valid], ref[valid])
    assert (got[~valid] == 0xFFFFFFFF).all()
    eng, ek, _ = rg.umi_cluster(pa.array(col, type=pa.large_binary()), L, md)
    assert ek == k
    assert np.array_equal(np.asarray(eng.fill_null(0).to_numpy(zero_copy_only=False)).astype(np.uint32)[valid],
                          got[valid])


def test_sharded_empty_and_all_irregular(rg):
    from rogtk_amd import dist as RD

    for col in ([], [None, None], [b"NNNN", b"acgt", b"ACG", None, b"NNNN"]):
        off, vals, vbits = (t.cuda() for t in _arrow(col))
        cid, k = RD.umi_cluster_sharded(off, vals, len(col), 4, 1, validity=vbits)
        got = cid.cpu().numpy().view(np.uint32).tolist()
        if len(col) == 5:
            assert k == 3 and got == [1, 2, 0, 0xFFFFFFFF, 1]  # b"ACG" < b"NNNN" < b"acgt"
        else:
            assert k == 0 and all(g == 0xFFFFFFFF for g in got)


def _worker(rank, world, port, L, md, n, seed, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rogtk_amd import dist as RD
        col = make_column(n, L, seed)
        start, count = RD.shard_range(n, rank, world)
        off, vals, vbits = (t.cuda() for t in _arrow(col[start:start + count]))
        cid, k = RD.umi_cluster_sharded(off, vals, count, L, md, validity=vbits)
        out_q.put((rank, start, cid.cpu().numpy().view(np.uint32).copy(), k))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("L,md,irr", [(12, 1, 0), (24, 1, 0), (32, 0, 0), (12, 1, 1), (24, 1, 1)])
def test_sharded_world2_matches_oracle(rg, L, md, irr):
    from oracle import pyoracle as P

    world, n, seed = 2, (4_000 if irr else 20_000), (-(11 + L) if irr else 11 + L)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, L, md, n, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    col = make_column(n, L, seed)
    ref, valid, rk, _ = P.umi_cluster(P.StrCol.from_list(col), L, md)
    got = np.zeros(n, dtype=np.uint32)
    for rank, start, ids, k in results:
        assert k == rk
        got[start:start + len(ids)] = ids
    assert np.array_equal(got[valid], ref[valid])


# ---- config C5 across ranks: BAM files sharded over ranks, clusters merged by all-to-all

def _bam_files(tmp, k):
    from rogtk_amd import synth_bam
    paths = []
    for i in range(k):
        p = os.path.join(tmp, f"part{i}.bam")
        synth_bam.synth_bam(p, 4000 + 997 * i, seed=0x524F47544B + i, level=1)
        paths.append(p)
    return paths


def _bam_oracle(paths, md):
    from oracle import pybam
    from oracle import pyoracle as P
    umis, names = [], []
    for p in paths:
        for r in pybam.bam_rows(p, "htslib"):
            s = r["sequence"]
            umis.append(None if s is None else s[:12].encode())
            names.append((p, r["name"]))
    rc, rv, rk, _ = P.umi_cluster(P.StrCol.from_list(umis), 12, md)
    return {key: (int(c), bool(v)) for key, c, v in zip(names, rc, rv)}, rk


def _bam_worker(rank, world, port, paths, md, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rogtk_amd import bam as B
        t = B.bams_umi_cluster(paths, umi_len=12, max_distance=md)
        out_q.put((rank, t.column("source").to_pylist(), t.column("name").to_pylist(),
                   t.column("cluster_id").to_pylist(), int(t.schema.metadata[b"n_clusters"])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("md", [0, 1])
def test_bams_umi_cluster_sharded_matches_oracle(rg, tmp_path, world, md):
    """Every record of 3 BAM files, decoded on the rank that owns its file, gets the id the
    oracle gives it over all files' UMIs together."""
    paths = _bam_files(str(tmp_path), 3)
    want, rk = _bam_oracle(paths, md)
    if world == 1:
        from rogtk_amd import bam as B
        t = B.bams_umi_cluster(paths, umi_len=12, max_distance=md)
        results = [(0, t.column("source").to_pylist(), t.column("name").to_pylist(),
                    t.column("cluster_id").to_pylist(), int(t.schema.metadata[b"n_clusters"]))]
    else:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_bam_worker, args=(r, world, port, paths, md, q)) for r in range(world)]
        for p in procs:
            p.start()
        results = [q.get(timeout=100) for _ in range(world)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    seen = 0
    for rank, src, names, ids, k in results:
        assert k == rk
        for s, nm, c in zip(src, names, ids):
            wc, wv = want[(s, nm)]
            assert (c is None) == (not wv)
            if wv:
                assert c == wc
            seen += 1
    assert seen == len(want)


def _bam_split_worker(rank, world, port, paths, md, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rogtk_amd import bam as B
        t = B.bams_umi_cluster(paths, umi_len=12, max_distance=md)
        out_q.put((rank, t.column("source").to_pylist(), t.column("name").to_pylist(),
                   t.column("cluster_id").to_pylist(), int(t.schema.metadata[b"n_clusters"])))
    finally:
        dist.destroy_process_group()


def _check_bam_results(results, want, rk):
    seen = set()
    for rank, src, names, ids, k in results:
        assert k == rk
        for s, nm, c in zip(src, names, ids):
            assert (s, nm) not in seen  # every record on exactly one rank
            seen.add((s, nm))
            wc, wv = want[(s, nm)]
            assert (c is None) == (not wv)
            if wv:
                assert c == wc
    assert seen == set(want)


@pytest.mark.parametrize("md", [0, 1])
def test_one_bam_split_over_two_ranks(rg, tmp_path, md):
    """Config C5 with ONE BAM over 2 ranks: the file is cut at a BGZF block start, each rank
    decodes its range (the second from the record it finds, checked against the first
    range's tail), and every record gets the oracle's id."""
    from rogtk_amd import synth_bam
    p = os.path.join(str(tmp_path), "one.bam")
    synth_bam.synth_bam(p, 30000, seed=0x524F47544B + 9, level=1)
    want, rk = _bam_oracle([p], md)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bam_split_worker, args=(r, 2, port, [p], md, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    results = [q.get(timeout=100) for _ in range(2)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert all(len(r[1]) > 0 for r in results)  # both ranks decoded part of the file
    _check_bam_results(results, want, rk)


def test_bam_ranges_recover_from_wrong_record_guesses(rg, tmp_path, monkeypatch):
    """A range whose guessed first record is wrong (forced here) is decoded again from the
    previous range's exact tail: the rows and ids still equal the oracle's."""
    from rogtk_amd import bam as B
    from rogtk_amd import synth_bam
    p = os.path.join(str(tmp_path), "g.bam")
    synth_bam.synth_bam(p, 20000, seed=0x524F47544B + 5, level=1)
    want, rk = _bam_oracle([p], 1)
    real = B.bam_find_record
    monkeypatch.setattr(B, "bam_find_record", lambda path, c: real(path, c) + 7)  # mid-record
    t = B.bams_umi_cluster([p], umi_len=12, max_distance=1, ranges_per_file=4)
    results = [(0, t.column("source").to_pylist(), t.column("name").to_pylist(),
                t.column("cluster_id").to_pylist(), int(t.schema.metadata[b"n_clusters"]))]
    _check_bam_results(results, want, rk)


# ---- the streaming pipeline across ranks (the bench path at N > 1): bitmap all-gather on
# its own stream, resolve of the merged bitmaps, labels of each rank's own reads

def _pipe_worker(rank, world, port, n_total, seeds, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rogtk_amd import device as D
        from rogtk_amd import dist as RD
        from rogtk_amd import synth
        from rogtk_amd.pipeline import UmiPipeline
        start, count = RD.shard_range(n_total, rank, world)
        outs = []
        pipe = UmiPipeline(12, n_total, count, "cuda", depth=2, target=b"ACGTACGTACGT", max_distance=1,
                           score_alone=True, on_assigned=lambda slot, b: outs.append(slot.cid[:count].clone()))
        assert pipe.s_comm is not None
        keep = []
        for s in seeds:
            codes = synth.umi_codes(n_total, 12, seed=s, start=start, count=count)
            keep.append(D.PackedBatch(torch.from_numpy(codes.view(np.int32)).cuda(), 12))
            pipe.submit(keep[-1])
        pipe.drain()
        torch.cuda.synchronize()
        out_q.put((rank, start, [o.cpu().numpy().view(np.uint32).copy() for o in outs]))
    finally:
        dist.destroy_process_group()


def test_pipeline_world2_matches_oracle(rg):
    """Two gloo ranks on cuda:0, 4 batches each through UmiPipeline: every batch's ids on
    every rank equal the oracle over the union of both ranks' reads of that batch."""
    from oracle import pyoracle as P
    from rogtk_amd import synth

    world, n_total = 2, 120_000
    seeds = [synth.DEFAULT_SEED + 101 * k for k in range(4)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, n_total, seeds, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k, s in enumerate(seeds):
        codes = synth.umi_codes(n_total, 12, seed=s)
        ref, _, _, _ = P.umi_cluster(P.StrCol.from_fixed(synth.codes_to_ascii(codes, 12)), 12, 1)
        got = np.zeros(n_total, dtype=np.uint32)
        for rank, start, outs in results:
            assert len(outs) == len(seeds)
            got[start:start + len(outs[k])] = outs[k]
        assert np.array_equal(got, ref), k


@pytest.mark.parametrize("n", [1_000_000, 4_000_000])
def test_sharded_world1_matches_engine_at_scale(rg, n):
    """The all-to-all H3 at world 1 on synth-v1 UMIs at the C5 sizes (1M and 4M rows,
    N / lowercase families included) gives the single-GPU engine's ids and count."""
    import pyarrow as pa

    from rogtk_amd import dist as RD
    from rogtk_amd import synth

    umis = synth.umi_ascii(n, 12, p_n=1e-4, p_lower=1e-4)
    offs = np.arange(0, 12 * (n + 1), 12, dtype=np.int64)
    col = pa.Array.from_buffers(pa.large_binary(), n, [None, pa.py_buffer(offs), pa.py_buffer(umis.reshape(-1))])
    eng, ek, _ = rg.umi_cluster(col, 12, 1)
    e = np.asarray(eng.fill_null(0xFFFFFFFF).to_numpy(zero_copy_only=False)).astype(np.uint32)
    off = torch.from_numpy(offs).cuda()
    vals = torch.from_numpy(umis.reshape(-1).copy()).cuda()
    cid, k = RD.umi_cluster_sharded(off, vals, n, 12, 1)
    torch.cuda.synchronize()
    got = cid.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != e)[0]
    detail = ""
    if len(bad) or k != ek:  # which side is wrong: the oracle on the same column
        from oracle import pyoracle as P

        ref, valid, rk, _ = P.umi_cluster(P.StrCol.from_list([bytes(r) for r in umis]), 12, 1)
        i = bad[:5]
        detail = (f"{len(bad)} rows differ, k sharded {k} engine {ek} oracle {rk}; sharded wrong on "
                  f"{int(np.count_nonzero(got[valid] != ref[valid]))}, engine wrong on "
                  f"{int(np.count_nonzero(e[valid] != ref[valid]))}; first: " + ", ".join(
                      f"{int(j)}:{bytes(umis[j])!r} {int(got[j])} vs {int(e[j])} (oracle {int(ref[j])})" for j in i))
    assert k == ek and not len(bad), detail


@pytest.mark.parametrize("n", [1_000_000, 4_000_000])
def test_bam_ranges_match_whole_file_at_scale(rg, tmp_path, n):
    """tools/bench_bam.py's C5 check at its size: one synthetic BAM cut into 4 ranges at
    BGZF block starts gives the whole-file run's rows (names, UMIs) and cluster ids."""
    from rogtk_amd import bam as B
    from rogtk_amd import synth_bam

    path = str(tmp_path / "c5.bam")
    synth_bam.synth_bam(path, n, level=6, threads=16)
    t1 = B.bam_umi_cluster(path, umi_len=12, max_distance=1, source="sequence", n_threads=16)
    t4 = B.bams_umi_cluster([path], umi_len=12, max_distance=1, source="sequence", n_threads=16, ranges_per_file=4)
    assert t1.num_rows == t4.num_rows == n
    msgs = []
    for c in ("name", "umi", "cluster_id"):
        a, b = t1.column(c).combine_chunks(), t4.column(c).combine_chunks()
        if not a.equals(b):
            neq = np.nonzero(~np.asarray(pa_equal(a, b)))[0]
            msgs.append(f"{c}: {len(neq)} rows differ, first {neq[:3].tolist()}: "
                        f"{[a[int(i)].as_py() for i in neq[:3]]} vs {[b[int(i)].as_py() for i in neq[:3]]}")
    k1, k4 = int(t1.schema.metadata[b"n_clusters"]), int(t4.schema.metadata[b"n_clusters"])
    assert not msgs and k1 == k4, "; ".join(msgs) + f"; n_clusters {k1} vs {k4}"


def pa_equal(a, b):
    import pyarrow.compute as pc

    eq = pc.equal(a, b)
    both_null = pc.and_(pc.is_null(a), pc.is_null(b))
    return pc.or_(pc.fill_null(eq, False), both_null).to_numpy(zero_copy_only=False)
