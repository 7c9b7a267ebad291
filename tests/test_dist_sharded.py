"""CPU, world_size 1/2/3 over gloo: the exchange plan of rogtk_amd.dist.umi_cluster_sharded
(the all-to-all H3 merge for any UMI length).

The device steps (rogtk_amd/csrc/dist_cluster.hip) need a GPU; here they are replaced by
numpy statements of the same contracts (NumpyOps, test-only), so that the routing, the
variable all-to-alls / all-gathers and the id assembly run with real gloo collectives.
Every rank's ids must equal the oracle (oracle/pyoracle.umi_cluster) run on the whole
column, for umi_len 8 / 20 / 32, with nulls, N, lowercase and wrong-length rows. The
GPU twin (tests/test_gpu_dist_sharded.py) runs the HIP steps.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_column(n: int, L: int, seed: int):
    """UMI strings with Hamming-1 families, irregular rows and nulls (list of bytes|None).
    A negative seed gives irregular_families (N / lowercase / length changes at high rates)."""
    if seed < 0:
        from conftest import irregular_families
        out = irregular_families(-seed, n, L)  # >= n rows; keep the edge rows at the end
        return out[:n - 4] + out[-4:]
    rng = np.random.default_rng(seed)
    parents = rng.integers(0, 4, size=(max(n // 6, 1), L))
    acgt = np.frombuffer(b"ACGT", np.uint8)
    out = []
    for i in range(n):
        u = parents[rng.integers(len(parents))].copy()
        if rng.random() < 0.3:
            u[rng.integers(L)] = rng.integers(4)
        s = bytearray(acgt[u].tobytes())
        r = rng.random()
        if r < 0.02:
            out.append(None)
            continue
        if r < 0.04:
            s[rng.integers(L)] = ord("N")
        elif r < 0.05:
            s = s.lower()
        elif r < 0.06:
            s = s[:-1]
        out.append(bytes(s))
    return out


class NumpyOps:
    """The contracts of the rogtk_* sharded-H3 entry points, restated in numpy (CPU)."""

    def long_codes(self, offsets, values, validity, voff, n, L):
        off = offsets.numpy().astype(np.int64)
        val = values.numpy()
        codes = np.zeros(n, np.uint64)
        kind = np.zeros(n, np.uint8)
        lut = np.full(256, -1, np.int64)
        for i, ch in enumerate(b"ACGT"):
            lut[ch] = i
        vb = None if validity is None else validity.numpy()
        for i in range(n):
            if vb is not None and not (vb[(voff + i) >> 3] >> ((voff + i) & 7)) & 1:
                continue
            s = val[off[i]:off[i + 1]]
            b = lut[s] if len(s) else np.zeros(0, np.int64)
            if len(s) == L and (b >= 0).all():
                c = 0
                for x in b:
                    c = (c << 2) | int(x)
                codes[i] = c
                kind[i] = 1
            else:
                kind[i] = 2
        return torch.from_numpy(codes.view(np.int64)), torch.from_numpy(kind)

    def unique(self, codes, kind, L):
        c = codes.numpy().view(np.uint64)
        if kind is not None:
            c = c[kind.numpy() == 1]
        return torch.from_numpy(np.unique(c).view(np.int64))

    def owner_counts(self, sorted_codes, L, W):
        c = sorted_codes.numpy().view(np.uint64)
        starts = [-(-(r * (1 << (2 * L))) // W) for r in range(W + 1)]
        b = [int(np.searchsorted(c, np.uint64(min(s, (1 << 64) - 1)))) if s < (1 << 64) else len(c)
             for s in starts]
        b[W] = len(c)
        return [b[r + 1] - b[r] for r in range(W)]

    def masked_records(self, D, L, W):
        d = D.numpy().view(np.uint64)
        rec = []
        for c in d.tolist():
            for p in range(L):
                mk = c & ~(3 << (2 * p))
                rec.append((hash((mk, p)) % W, mk, p, c))
        rec.sort(key=lambda r: r[0])
        counts = [sum(1 for r in rec if r[0] == w) for w in range(W)]
        mk = np.array([r[1] for r in rec], np.uint64)
        pos = np.array([r[2] for r in rec], np.int32)
        code = np.array([r[3] for r in rec], np.uint64)
        return (torch.from_numpy(mk.view(np.int64)), torch.from_numpy(pos), torch.from_numpy(code.view(np.int64)),
                counts)

    def clique_edges(self, mk, pos, code, L, G):
        g = G.numpy().view(np.uint64)
        groups = {}
        for m, p, c in zip(mk.numpy().view(np.uint64).tolist(), pos.numpy().tolist(),
                           code.numpy().view(np.uint64).tolist()):
            groups.setdefault((p, m), []).append(c)
        E = []
        for members in groups.values():
            for a, b in zip(members, members[1:]):
                E.append((int(np.searchsorted(g, np.uint64(a))), int(np.searchsorted(g, np.uint64(b)))))
        return torch.tensor(E, dtype=torch.int32).reshape(-1, 2)

    def cc_labels(self, nv, E):
        f = list(range(nv))

        def find(x):
            while f[x] != x:
                f[x] = f[f[x]]
                x = f[x]
            return x

        for a, b in E.numpy().tolist():
            ra, rb = find(a), find(b)
            if ra != rb:
                f[max(ra, rb)] = min(ra, rb)
        roots = sorted({find(v) for v in range(nv)})
        lab = {r: i for i, r in enumerate(roots)}
        return torch.tensor([lab[find(v)] for v in range(nv)], dtype=torch.int32), len(roots)

    def assign(self, codes, kind, G, labels, cid):
        g = G.numpy().view(np.uint64)
        c = codes.numpy().view(np.uint64)
        k = kind.numpy()
        out = cid.numpy()
        for i in range(len(c)):
            if k[i] == 0:
                out[i] = -1
            elif k[i] == 1:
                j = int(np.searchsorted(g, c[i]))
                assert j < len(g) and g[j] == c[i]
                out[i] = labels[j]

    def irregular_merge(self, offsets, values, n, max_len, L, md, G, labels, n_reg):
        """rogtk_irregular_merge: exact bytes (md 0) or Hamming-1 edges among the strings
        and to G's codes, components with the regular clusters (md 1)."""
        off = offsets.numpy()
        val = values.numpy().tobytes()
        strs = [val[off[i]:off[i + 1]] for i in range(n)]
        order = sorted(set(strs))
        rank = {s: i for i, s in enumerate(order)}
        if md == 0:
            return torch.tensor([n_reg + rank[s] for s in strs], dtype=torch.int32), n_reg + len(order)
        g = G.numpy().view(np.uint64)
        lab = labels.numpy()
        f = list(range(n_reg + len(order)))

        def find(x):
            while f[x] != x:
                x = f[x]
            return x

        def unite(a, b):
            ra, rb = find(a), find(b)
            if ra != rb:
                f[max(ra, rb)] = min(ra, rb)

        first = {}
        for j, s in enumerate(order):
            for p in range(len(s)):
                key = (p, s[:p] + s[p + 1:])
                if key in first:
                    unite(n_reg + first[key], n_reg + j)
                else:
                    first[key] = j
            bad = [q for q in range(len(s)) if s[q] not in b"ACGT"]
            if len(s) == L and len(bad) == 1:
                for x in b"ACGT":
                    t = s[:bad[0]] + bytes([x]) + s[bad[0] + 1:]
                    c = 0
                    for ch in t:
                        c = (c << 2) | b"ACGT".index(ch)
                    i = int(np.searchsorted(g, np.uint64(c)))
                    if i < len(g) and g[i] == c:
                        unite(int(lab[i]), n_reg + j)
        roots = sorted({find(v) for v in range(len(f))})
        dense = {r: i for i, r in enumerate(roots)}
        for i in range(len(lab)):
            lab[i] = dense[find(int(lab[i]))]
        return torch.tensor([dense[find(n_reg + rank[s])] for s in strs], dtype=torch.int32), len(roots)

    def group_strings(self, offsets, values, n, max_len, base):
        off = offsets.numpy()
        val = values.numpy().tobytes()
        strs = [val[off[i]:off[i + 1]] for i in range(n)]
        order = sorted(set(strs))
        rank = {s: i for i, s in enumerate(order)}
        return torch.tensor([base + rank[s] for s in strs], dtype=torch.int32), len(order)


def _arrow(col):
    n = len(col)
    lens = [0 if s is None else len(s) for s in col]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    vals = np.frombuffer(b"".join(s for s in col if s is not None), np.uint8).copy()
    valid = np.array([s is not None for s in col], dtype=bool)
    vbits = np.packbits(np.concatenate([valid, np.zeros((-n) % 8, bool)]), bitorder="little")
    return torch.from_numpy(off), torch.from_numpy(vals if len(vals) else np.zeros(1, np.uint8)), \
        torch.from_numpy(vbits)


def _worker(rank, world, port, L, md, n, seed, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rogtk_amd import dist as RD
        col = make_column(n, L, seed)
        start, count = RD.shard_range(n, rank, world)
        off, vals, vbits = _arrow(col[start:start + count])
        cid, k = RD.umi_cluster_sharded(off, vals, count, L, md, validity=vbits, ops=NumpyOps())
        out_q.put((rank, start, cid.numpy().view(np.uint32).copy(), k))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("L,md,irr", [(8, 1, 0), (20, 1, 0), (32, 1, 0), (20, 0, 0), (6, 1, 1), (12, 1, 1)])
def test_sharded_cluster_plan_matches_oracle(world, L, md, irr):
    from oracle import pyoracle as P

    n, seed = 900, (-(3 + L) if irr else 7 + L)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, L, md, n, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    col = make_column(n, L, seed)
    ref, valid, rk, _ = P.umi_cluster(P.StrCol.from_list(col), L, md)
    got = np.zeros(n, dtype=np.uint32)
    for rank, start, ids, k in results:
        assert k == rk, (rank, k, rk)
        got[start:start + len(ids)] = ids
    assert np.array_equal(got[valid], ref[valid])
    assert (got[~valid] == 0xFFFFFFFF).all()
