"""H4 exchange on the GPU: rogtk_route_pack (HIP) == the torch counting sort used for CPU
tensors, and a 2-rank gloo rehearsal on one GPU with device tensors end to end."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _column(seed, n, maxlen=90):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen, size=n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    vals = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    return off, vals


@pytest.mark.parametrize("world", [1, 2, 3, 8, 64])
@pytest.mark.parametrize("n", [0, 1, 1000, 200_000])
def test_route_pack_matches_torch(world, n):
    from rogtk_amd import dist as RD
    off, vals = _column(world * 31 + n, n)
    keys = torch.from_numpy(np.random.default_rng(n).integers(0, 2**31, size=n).astype(np.int32))
    dest = RD.route_destination(keys, world)
    c = RD._pack(torch.from_numpy(off), torch.from_numpy(vals), dest, world)
    g = RD._pack(torch.from_numpy(off).cuda(), torch.from_numpy(vals).cuda(), dest.cuda(), world)
    assert torch.equal(g[0].cpu(), c[0])
    assert list(g[1]) == list(c[1]) and list(g[2]) == list(c[2])
    assert torch.equal(g[3].cpu(), c[3])
    assert torch.equal(g[4].cpu(), c[4])


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rogtk_amd import dist as RD
        off, vals = _column(7, 5000)
        keys = (np.arange(5000) * 7919 % 613).astype(np.int32)
        s, c = RD.shard_range(5000, rank, world)
        o = torch.from_numpy(off[s:s + c + 1] - off[s]).cuda()
        v = torch.from_numpy(vals[off[s]:off[s + c]].copy()).cuda()
        ro, rv, rk, sr, srow = RD.route_rows(o, v, torch.from_numpy(keys[s:s + c]).cuda())
        ro, rv = ro.cpu().numpy(), rv.cpu().numpy()
        rows = []
        for i, (q_, r_) in enumerate(zip(sr.cpu().tolist(), srow.cpu().tolist())):
            g = RD.shard_range(5000, q_, world)[0] + r_
            rows.append((g, rv[ro[i]:ro[i + 1]].tobytes() == vals[off[g]:off[g + 1]].tobytes(),
                         int(rk[i]) == int(keys[g])))
        q.put((rank, rows))
    finally:
        dist.destroy_process_group()


def test_route_rows_two_ranks_one_gpu():
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=100) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    seen = []
    for rank, rows in res:
        assert all(ok and kk for _, ok, kk in rows)
        seen += [g for g, _, _ in rows]
    assert sorted(seen) == list(range(5000))
