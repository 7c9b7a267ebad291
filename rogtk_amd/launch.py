"""One process per GPU on one node, started before anything touches the GPU.

`python bench.py --gpus N` with no WORLD_SIZE in the environment uses run_local_ranks to
start N fresh worker processes (multiprocessing "spawn": new interpreters, so no HIP state
is inherited and nothing is exec'd over a process that initialised the GPU). Each worker
gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT exactly as torchrun would
set them, binds cuda:LOCAL_RANK and joins the process group (nccl = RCCL over xGMI). The
parent only waits and returns the workers' worst exit code.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import socket
import time
from multiprocessing.connection import wait
from typing import Callable, Sequence


def visible_gpus():
    """GPUs this process could use, counted WITHOUT initialising HIP (the launcher must not
    touch the GPU before it spawns the ranks): the KFD topology nodes with a GPU id,
    narrowed by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES. None
    when the topology is not readable (the ranks then find out themselves)."""
    n = 0
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "gpu_id")) as f:
                    n += int(f.read().strip() or 0) != 0
            except (OSError, ValueError):
                pass
    except OSError:
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _entry(rank: int, world: int, port: int, target: Callable, args: Sequence):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    target(*args)


def run_local_ranks(world: int, target: Callable, args: Sequence = (), timeout: float | None = None) -> int:
    """Run target(*args) in `world` spawned processes (ranks 0..world-1 of one node).
    Returns 0 when every rank exited 0, else the first non-zero exit code (a rank killed
    by a signal reports 128 + signal). Ranks still running after `timeout` are killed."""
    if world < 1:
        raise ValueError("world must be >= 1")
    ctx = mp.get_context("spawn")
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, target, tuple(args))) for r in range(world)]
    for p in procs:
        p.start()
    deadline = None if timeout is None else time.monotonic() + timeout
    rc = 0
    live = list(procs)
    while live:
        left = None if deadline is None else max(0.0, deadline - time.monotonic())
        wait([p.sentinel for p in live], left)
        done = [p for p in live if not p.is_alive()]
        for p in done:
            p.join()
            code = p.exitcode if p.exitcode is not None else 1
            if code < 0:
                code = 128 - code
            if code and not rc:
                rc = code
        live = [p for p in live if p.is_alive()]
        timed_out = deadline is not None and time.monotonic() >= deadline
        if live and (rc or timed_out):  # a failed rank leaves its peers blocked in collectives
            for p in live:
                p.kill()
            for p in live:
                p.join()
            rc = rc or 124
            live = []
    return rc
