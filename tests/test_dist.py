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


def _route_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle as P
        from rogtk_amd import dist as RD
        reads, keys = _route_data()
        start, count = RD.shard_range(len(reads), rank, world)
        mine = reads[start:start + count]
        off = torch.tensor(np.concatenate([[0], np.cumsum([len(r) for r in mine])]), dtype=torch.int64)
        vals = torch.tensor(np.frombuffer(b"".join(mine), np.uint8).copy())
        k = torch.tensor(keys[start:start + count], dtype=torch.int32)
        o, v, rk, srank, srow = RD.route_rows(off, vals, k)
        o, v, rk = o.numpy(), v.numpy().tobytes(), rk.numpy()
        got = [v[o[i]:o[i + 1]] for i in range(len(rk))]
        # every key this rank received is owned here, with all of its rows, in source order
        owned = {int(x) for x in rk}
        dest = RD.route_destination(torch.tensor(keys, dtype=torch.int32), world).numpy()
        assert owned == {int(x) for x in np.asarray(keys)[dest == rank]}
        src_global = [RD.shard_range(len(reads), int(q), world)[0] + int(r) for q, r in zip(srank, srow)]
        assert [reads[g] for g in src_global] == got
        assert [keys[g] for g in src_global] == rk.tolist()
        # per-group k-mer spectra of the owned groups (the work each rank then does alone)
        order = np.argsort(rk, kind="stable")
        gk, go = np.unique(rk[order], return_index=True)
        go = np.concatenate([go, [len(rk)]]).astype(np.int64)
        spec = P.kmer_spectrum(P.StrCol.from_list([got[i] for i in order]), 17, 2, False, go)
        out_q.put((rank, gk.tolist(), {f: spec[f].tolist() for f in ("kmer_lo", "exts", "counts")},
                   spec["group_offsets"].tolist()))
    finally:
        dist.destroy_process_group()


def _route_data():
    rng = np.random.default_rng(5)
    reads, keys = [], []
    for g in range(120):
        tpl = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 120))
        for _ in range(int(rng.integers(1, 12))):
            a = int(rng.integers(0, 40))
            reads.append(tpl[a:a + int(rng.integers(40, 80))])
            keys.append(int(g * 7919 % 100003))
    perm = rng.permutation(len(reads))
    return [reads[i] for i in perm], [keys[i] for i in perm]


@pytest.mark.parametrize("world", [2, 4])
def test_route_rows_colocates_groups(world):
    """H4 exchange: after one all-to-all every group lives on exactly one
    rank, and the per-group spectra computed there equal the single-process spectra."""
    from oracle import pyoracle as P
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_route_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    reads, keys = _route_data()
    keys = np.asarray(keys)
    order = np.argsort(keys, kind="stable")
    gk, go = np.unique(keys[order], return_index=True)
    go = np.concatenate([go, [len(keys)]]).astype(np.int64)
    ref = P.kmer_spectrum(P.StrCol.from_list([reads[i] for i in order]), 17, 2, False, go)
    eo = ref["group_offsets"]
    seen = set()
    for rank, rgk, spec, reo in results:
        for j, key in enumerate(rgk):
            assert key not in seen
            seen.add(key)
            g = int(np.searchsorted(gk, key))
            for f in ("kmer_lo", "exts", "counts"):
                assert spec[f][reo[j]:reo[j + 1]] == ref[f][eo[g]:eo[g + 1]].tolist(), (key, f)
    assert seen == set(gk.tolist())
