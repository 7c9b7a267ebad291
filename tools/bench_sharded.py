"""Throughput of the sharded H3 (rogtk_amd.dist.umi_cluster_sharded, all-to-all merge) next to
the single-GPU engines, on synth-v1 UMIs of several lengths (columns resident in HBM).

Usage: python tools/bench_sharded.py [--n 10000000] [--lens 12,20,32] [--reps 3]
       torchrun --nproc-per-node N tools/bench_sharded.py ...   (one rank per GPU, RCCL)
Prints one JSON line per length: reads/s of the sharded path (all ranks' reads / max rank
time) and, at world 1, of the single-GPU engine on the same column (rogtk_umi_cluster_dev:
the bitmap engine for umi_len <= 16, the sort engine for 17..32).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rogtk_amd import _lib  # noqa: E402
from rogtk_amd import dist as RD  # noqa: E402
from rogtk_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000, help="reads per rank")
    ap.add_argument("--lens", type=str, default="12,20,32")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    dev = torch.device("cuda", torch.cuda.current_device())
    for L in [int(x) for x in a.lens.split(",")]:
        n_total = a.n * world
        start, count = RD.shard_range(n_total, rank, world)
        asc = synth.umi_ascii(n_total, L, start=start, count=count)
        off = torch.arange(count + 1, dtype=torch.int64, device=dev) * L
        vals = torch.from_numpy(asc.reshape(-1)).to(dev)
        best = 1e9
        k = 0
        for _ in range(a.reps):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            cid, k = RD.umi_cluster_sharded(off, vals, count, L, 1)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            if world > 1:
                t = torch.tensor([el], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el = float(t.item())
            best = min(best, el)
        line = {"umi_len": L, "reads_per_rank": count, "world": world, "n_clusters": k,
                "sharded_reads_per_s": round(n_total / best, 1), "sharded_s": round(best, 4)}
        if world == 1:
            out = torch.empty(count, dtype=torch.int32, device=dev)
            nc = ctypes.c_int64(0)
            s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            eb = 1e9
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                _lib.call("rogtk_umi_cluster_dev", ctypes.c_void_p(off.data_ptr()), ctypes.c_void_p(vals.data_ptr()),
                          None, count, L, 1, ctypes.c_void_p(out.data_ptr()), ctypes.byref(nc), s)
                torch.cuda.synchronize()
                eb = min(eb, time.perf_counter() - t0)
            line["engine_reads_per_s"] = round(count / eb, 1)
            line["engine_s"] = round(eb, 4)
            line["ids_equal"] = bool(torch.equal(out, cid)) and nc.value == k
        if rank == 0:
            print(json.dumps(line), flush=True)
        del off, vals
        torch.cuda.empty_cache()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
