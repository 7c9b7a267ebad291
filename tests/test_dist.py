"""CPU, world_size 2 and 4 over gloo: the multi-GPU H3 exchange path.

Each rank takes its record shard (rogtk_amd.dist.shard_range), builds the 4^L-bit
presence bitmap of its UMIs in the layout rogtk_cluster_local_bitmap produces
(bit code%64 of word code//64), all-gathers the bitmaps with
rogtk_amd.dist.gather_bitmaps (the same call bench.py makes over RCCL), ORs them as
rogtk_cluster_resolve does, resolves the components of the merged distinct set with
the oracle and labels its own reads. Every rank's ids must equal the single-process
oracle run on the whole dataset, for any world size.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_TOTAL = 60_000
L = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bitmap(codes: np.ndarray, L: int) -> np.ndarray:
    words = max(1, 4 ** L // 64)
    bm = np.zeros(words, dtype=np.uint64)
    np.bitwise_or.at(bm, codes >> 6, np.left_shift(np.uint64(1), (codes & 63).astype(np.uint64)))
    return bm


def _worker(rank, world, port, md, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle as P
        from rogtk_amd import dist as RD
        from rogtk_amd import synth

        start, count = RD.shard_range(N_TOTAL, rank, world)
        codes = synth.umi_codes(N_TOTAL, L, start=start, count=count)
        local = torch.from_numpy(_bitmap(codes, L).view(np.int64))
        gathered, nb = RD.gather_bitmaps(local)
        assert nb == world and gathered.numel() == world * local.numel()
        merged = np.bitwise_or.reduce(gathered.numpy().view(np.uint64).reshape(world, -1), axis=0)
        bits = np.unpackbits(merged.view(np.uint8), bitorder="little")
        distinct = np.nonzero(bits)[0].astype(np.uint32)  # ascending == lexicographic
        col = P.StrCol.from_fixed(synth.codes_to_ascii(distinct, L))
        dids, _, k, _ = P.umi_cluster(col, L, md)
        ids = dids[np.searchsorted(distinct, codes)]
        out_q.put((rank, start, ids, k))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("md", [0, 1])
def test_sharded_exchange_matches_single_process(world, md):
    from oracle import pyoracle as P
    from rogtk_amd import synth

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, md, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    codes = synth.umi_codes(N_TOTAL, L)
    ref, _, rk, _ = P.umi_cluster(P.StrCol.from_fixed(synth.codes_to_ascii(codes, L)), L, md)
    got = np.zeros(N_TOTAL, dtype=np.uint32)
    for rank, start, ids, k in results:
        assert k == rk
        got[start:start + len(ids)] = ids
    assert np.array_equal(got, ref)
