"""CPU: the one-process-per-GPU launcher of bench.py (rogtk_amd.launch) at world 2 over
gloo: every rank sees WORLD_SIZE / RANK / LOCAL_RANK as torchrun sets them, the process
group has exactly N ranks, and a failing rank fails the launch instead of hanging it."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from rogtk_amd.launch import run_local_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(out_dir):
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    t = torch.tensor([float(dist.get_rank() + 1)])
    dist.all_reduce(t)
    with open(os.path.join(out_dir, f"r{dist.get_rank()}.json"), "w") as f:
        json.dump({"world": dist.get_world_size(), "rank": int(os.environ["RANK"]),
                   "local": int(os.environ["LOCAL_RANK"]), "sum": float(t.item())}, f)
    dist.barrier()
    dist.destroy_process_group()


def _fail_on_rank1():
    import torch.distributed as dist

    dist.init_process_group("gloo")
    if dist.get_rank() == 1:
        raise SystemExit(3)
    dist.barrier()  # rank 0 blocks here until the launcher kills it


@pytest.mark.parametrize("world", [2, 3])
def test_launcher_world(tmp_path, world):
    assert run_local_ranks(world, _rank, (str(tmp_path),), timeout=120) == 0
    got = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    for r, g in enumerate(got):
        assert g == {"world": world, "rank": r, "local": r, "sum": world * (world + 1) / 2}


def test_launcher_failed_rank_fails_launch():
    # rank 1 exits 3; rank 0, blocked in the barrier, is killed by the launcher or sees the
    # closed connection and fails first (gloo raises): either way the launch fails, promptly
    rc = run_local_ranks(2, _fail_on_rank1, (), timeout=120)
    assert rc in (1, 3)


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)
