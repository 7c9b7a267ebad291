"""GPU: the RCCL call sequence of the multi-GPU path, executed once at world 1.

bench.py --gpus 8 issues, per step, the presence-bitmap all-gather on the pipeline's comm
stream (rogtk_amd.pipeline, dist.gather_bitmaps: all_gather_into_tensor); the H4 route
(dist.route_rows) and the sharded H3 merge (dist.umi_cluster_sharded) add all_to_all_single
and all-gathers. Every multi-rank test elsewhere runs gloo; here a child process
initialises the "nccl" backend (RCCL) at world 1 on cuda:0, so each of those calls goes
through RCCL on device tensors, and checks the results against the oracle / the
single-GPU engines (with a process group the exchanges always run, at world 1 too).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, {root!r})
from rogtk_amd import device as D, dist as RD, synth
from rogtk_amd.pipeline import UmiPipeline
from oracle import pyoracle as P

torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:{port}", rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl" and RD.collective() and RD.world() == 1
dev = torch.device("cuda", 0)

# 1. the bitmap all-gather (all_gather_into_tensor on device tensors)
bm = torch.randint(-2**62, 2**62, (262144,), dtype=torch.int64, device=dev)
out, nb = RD.gather_bitmaps(bm)
assert nb == 1 and out.data_ptr() != bm.data_ptr() and torch.equal(out, bm)
print("all_gather ok", flush=True)

# 2. the H4 route: all_to_all_single of the packed rows + three metadata all-to-alls
n = 20011
lens = torch.randint(0, 200, (n,), dtype=torch.int64)
offs = torch.zeros(n + 1, dtype=torch.int64)
offs[1:] = torch.cumsum(lens, 0)
vals = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8)
keys = torch.randint(0, 5000, (n,), dtype=torch.int32)
o2, v2, k2, src_rank, src_row = RD.route_rows(offs.to(dev), vals.to(dev), keys.to(dev))
assert torch.equal(o2.cpu(), offs) and torch.equal(v2.cpu(), vals) and torch.equal(k2.cpu(), keys)
assert int(src_rank.abs().sum()) == 0 and torch.equal(src_row.cpu(), torch.arange(n))
print("route ok", flush=True)

# 3. the pipeline's comm stream: the all-gather behind every mark, the resolve waiting for it
L, m, nbatch = 12, 1_000_003, 3
assert UmiPipeline(L, m, m, dev, depth=2).s_comm is not None
seeds = [synth.DEFAULT_SEED + 7 * k for k in range(nbatch)]
got = []
pipe = UmiPipeline(L, m, m, dev, depth=2, target=b"ACGTACGTACGT", max_distance=1,
                   on_assigned=lambda slot, b: got.append(slot.cid[:m].clone()))
keep = []
for s in seeds:
    keep.append(D.PackedBatch(torch.from_numpy(synth.umi_codes(m, L, seed=s).view(np.int32)).to(dev), L))
    pipe.submit(keep[-1])
pipe.drain()
torch.cuda.synchronize()
assert len(got) == nbatch
for s, cid in zip(seeds, got):
    codes_h = synth.umi_codes(m, L, seed=s)
    rc, _, _, _ = P.umi_cluster(P.StrCol.from_fixed(synth.codes_to_ascii(codes_h, L)), L, 1)
    assert np.array_equal(cid.cpu().numpy().view(np.uint32), rc)
print("pipeline ok", flush=True)

# 4. the sharded H3 merge (all-to-alls of distinct codes and masked records, all-gathers of
#    the owned sets and edges) for a 12-bp and a 20-bp column
for L2 in (12, 20):
    k = 200_003
    rng = np.random.default_rng(L2)
    base = rng.integers(0, 4, (k // 10, L2))
    pick = base[rng.integers(0, len(base), k)]
    flip = rng.random((k, L2)) < 0.01
    pick[flip] = rng.integers(0, 4, int(flip.sum()))
    asc = np.frombuffer(b"ACGT", np.uint8)[pick].reshape(-1)
    offs = torch.arange(0, (k + 1) * L2, L2, dtype=torch.int64, device=dev)
    cid, nc = RD.umi_cluster_sharded(offs, torch.from_numpy(asc).to(dev), k, L2, 1)
    rc, _, rk, _ = P.umi_cluster(P.StrCol.from_fixed(asc.reshape(k, L2)), L2, 1)
    assert nc == rk and np.array_equal(cid.cpu().numpy().view(np.uint32), rc), L2
print("sharded ok", flush=True)
dist.destroy_process_group()
print("rccl-ok", flush=True)
"""


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world1_call_sequence():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-u", "-c", CHILD.format(root=ROOT, port=_free_port())], env=env,
                       capture_output=True, text=True, timeout=240)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "rccl-ok" in r.stdout
