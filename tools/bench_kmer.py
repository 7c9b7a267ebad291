#!/usr/bin/env python3
"""C3 measurement (BASELINE.json configs[2]): UMI grouping + k-mer front end on 1 MI355X.

One step = one batch of synthetic 150-bp reads with 12-bp UMIs, resident in HBM:
  H3 exact UMI ids    (mark -> bitmap -> resolve(max_distance 0) -> assign; the
                       caller-side group_by('umi') of rogtk/__init__.py:206-214)
  group_spectra       rogtk_amd.device.group_spectra: rogtk_group_by_key (stable radix
                       sort of the ids -> row permutation + group offsets), then
                       rogtk_kmer_spectrum_dev, k = 17 (effective 32), min_coverage
                       20 (rogtk/__init__.py:212): filter_kmers + CountFilter +
                       censored exts per group (LDS path for small groups), in calls of
                       <= 10M rows; tests/test_gpu_c3.py checks this path vs the oracle
Prints one JSON line: reads/s over the timed steps, per-phase HIP-event times and
the LDS / global path split. Not the driver's bench (bench.py is C2).

Usage: python tools/bench_kmer.py [--reads 10000000 --steps 5 --warmup 1]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rogtk_amd import _lib  # noqa: E402
from rogtk_amd import device as D  # noqa: E402
from rogtk_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--k", type=int, default=17)
    ap.add_argument("--min-coverage", type=int, default=20)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--global-only", action="store_true", help="route every group through the radix-sort path")
    ap.add_argument("--ascii", action="store_true",
                    help="stage grouped rows from their ASCII bytes (no rogtk_pack_reads block column)")
    ap.add_argument("--group-batch-rows", type=int, default=100_000_000,
                    help="k-mer spectra run over consecutive groups of at most this many rows per call "
                         "(bounds the output capacity: 19 B x (read_len - 3) / min_coverage per row)")
    args = ap.parse_args()
    n, RL, L = args.reads, args.read_len, 12
    dev = torch.device("cuda", 0)
    t0 = time.time()
    codes = torch.from_numpy(synth.umi_codes(n, L).view(np.int32)).to(dev)
    reads = torch.empty(n * RL, dtype=torch.uint8, device=dev)
    chunk = 2_000_000
    for a in range(0, n, chunk):  # host generator (OpenMP), streamed to HBM
        b = min(n, a + chunk)
        reads[a * RL:b * RL] = torch.from_numpy(synth.reads(n, RL, start=a, count=b - a).reshape(-1)).to(dev)
    offsets = torch.arange(0, (n + 1) * RL, RL, dtype=torch.int64, device=dev)
    gen_s = time.time() - t0
    batch = D.PackedBatch(codes, L)
    eng = D.ClusterEngine(L, min(n, 4 ** L), dev)
    cid = torch.empty(n, dtype=torch.int32, device=dev)
    br = min(n, args.group_batch_rows)
    _lib.call("rogtk_kmer_set_path", 0 if args.global_only else 1)
    ev = lambda: torch.cuda.Event(enable_timing=True)
    phases = {"cluster": 0.0, "group_by+kmer": 0.0}
    out = None
    path_groups = [0, 0]

    def step(record):
        nonlocal out
        e0, e1, e3 = ev(), ev(), ev()
        e0.record()
        D.cluster_batch(eng, batch, cid, 0)
        e1.record()
        path_groups[:] = [0, 0]
        acc = {"valid": 0, "stats": [], "calls": 0}

        def consume(g0, g1, r):  # per spectrum call (the same path tests/test_gpu_c3.py checks)
            acc["valid"] += int(r["entry_offsets"][-1].item())
            acc["stats"].append(r["stats"].clone())
            acc["calls"] += 1
            ps = (ctypes.c_int64 * 2)()
            _lib.call("rogtk_kmer_path_stats", ps)
            path_groups[0] += ps[0]
            path_groups[1] += ps[1]

        _, _, G, _ = D.group_spectra(offsets, reads, cid, args.k, args.min_coverage, batch_rows=br, consume=consume,
                                     packed=None if args.ascii else "auto")
        out = {"n_calls": acc["calls"], "valid": acc["valid"],
               "stats": acc["stats"][0] if len(acc["stats"]) == 1 else torch.cat(acc["stats"])}
        e3.record()
        torch.cuda.synchronize()
        if record:
            phases["cluster"] += e0.elapsed_time(e1)
            phases["group_by+kmer"] += e1.elapsed_time(e3)
        return G

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        G = step(True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    paths = path_groups
    st = out["stats"].cpu().numpy()
    step_s = el / args.steps
    obs_per_s = n * (RL - int(st[:, 0].max()) + 1) * args.steps / el
    # C3 roofline. Algorithmic HBM bytes per read: the ASCII read once, its
    # UMI code read and its cluster id written (RL + 8). Staged bytes per read as built:
    # the pack pass (RL in, one 64-B block out), the grouped gather (64-B block in, 40 B
    # staged + 12 B of row metadata). The step is bound by the LDS k-mer table, stated as
    # k-mer observations per CU clock (256 CUs, 2.4 GHz).
    alg_b, staged_b, peak = RL + 8, RL + 64 + 64 + 40 + 12, 8000.0
    ach = lambda b: n * b / step_s / 1e9
    roofline = {
        "bound": "lds", "kernel": "k_kmer_lds<3>",
        "obs_per_cu_clock": round(obs_per_s / (256 * 2.4e9), 3),
        "step": {"bound": "hbm", "algorithmic_bytes_per_read": alg_b, "achieved": round(ach(alg_b), 1),
                 "peak": peak, "unit": "GB/s", "frac": round(ach(alg_b) / peak, 4)},
        "staged": {"bytes_per_read": staged_b, "achieved": round(ach(staged_b), 1), "peak": peak, "unit": "GB/s",
                   "frac": round(ach(staged_b) / peak, 4)},
    }
    line = {
        "metric": "reads/s UMI group_by + k-mer spectra (C3 front end), 150 bp reads, 12 bp UMI, 1 MI355X",
        "value": round(n * args.steps / el, 1), "unit": "reads/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * el / args.steps, 3),
        "config": {"workload": "C3: H3 exact UMI ids -> group_by -> k-mer spectra per group",
                   "staging": "ASCII rows" if args.ascii else "2-bit block column (rogtk_pack_reads, once per step)",
                   "reads": n, "read_len": RL, "umi_len": L, "k": args.k, "k_eff": int(st[:, 0].max()),
                   "min_coverage": args.min_coverage, "groups": G, "lds_groups": paths[0],
                   "global_groups": paths[1], "valid_kmers": out["valid"], "spectrum_calls": out["n_calls"],
                   "sequences": int(st[:, 1].sum())},
        "phases_ms": {k: round(v / args.steps, 3) for k, v in phases.items()},
        "observations_per_s": round(obs_per_s, 1),
        "roofline": roofline,
        "data": f"synthetic (synth-v1 reads + UMIs, {n // 10} molecules), generated in {gen_s:.1f} s, resident in HBM",
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
