#!/usr/bin/env python3
"""bench.py — UMI score + cluster throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch of synthetic reads already
resident in HBM as the packed 2-bit SoA (BASELINE config C2: 10M reads per GPU,
12-bp UMI, Hamming<=1), through rogtk_amd.pipeline (three HIP streams, --depth
batches in flight; the timed region ends after every submitted batch is done):
  main     k_score_packed: H1 all 7 complexity fields + H2 Hamming-within bits;
           k_mark_xcd: H3 presence mark; presence -> bitmap
  resolve  [all-gather over ranks, RCCL] -> scan -> rank tables -> LDS-local CC ->
           global hook/jump rounds -> labels
  assign   cluster ids per read (waits for the next batch's score kernel, so the
           HBM-bound score overlaps only the latency-bound resolve; --overlap-score
           lifts that: ~4% faster steps, score kernel shares HBM with the gathers)
Weak scaling: every rank owns reads_per_gpu records of one global dataset
(shard by record); value = all ranks' reads / max-over-ranks wall time.

Workloads (--workload): C2 (default; BASELINE configs[1]) = 10M reads per GPU, weak
scaling; C4 (configs[3]) = 500M reads in all, 500M/N per GPU, strong scaling.

Usage: python bench.py [--gpus N --steps K --warmup W] [--workload C2|C4]
       torchrun --nproc-per-node N bench.py --gpus N ...
With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N ranks itself
(rogtk_amd.launch: spawned processes, one per GPU, before anything touches the GPU).
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from rogtk_amd import device as D  # noqa: E402
from rogtk_amd import dist as RD  # noqa: E402
from rogtk_amd import synth  # noqa: E402
from rogtk_amd.pipeline import UmiPipeline  # noqa: E402

METRIC = "reads/s UMI score+cluster, 150 bp/12 bp UMI, 1→8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
TARGET = b"ACGTACGTACGT"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20,
                    help="timed steps (the driver's 20: the pipeline fills and drains once per timed region, ~5%% "
                         "of 20 steps; 'sustained' reports the steady state)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=("C2", "C4"), default="C2",
                    help="C2: 10M reads per GPU (weak scaling); C4: 500M reads over all GPUs (strong scaling)")
    ap.add_argument("--reads-per-gpu", type=int, default=None,
                    help="override the workload's reads per GPU (C2 default 10M)")
    ap.add_argument("--total-reads", type=int, default=500_000_000, help="C4: reads over all GPUs")
    ap.add_argument("--umi-len", type=int, default=12)
    ap.add_argument("--max-distance", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip in-run HIP-event kernel timing")
    ap.add_argument("--profile-every", type=int, default=4,
                    help="in the timed region, time the score / assign launches of every Nth step")
    ap.add_argument("--sustain-seconds", type=float, default=4.0,
                    help="after the timed region, run the same pipelined steps for this long (untimed by the "
                         "contract; reported as 'sustained') so the GPU stays busy long enough for external "
                         "utilisation sampling; 0 = skip")
    ap.add_argument("--settle-seconds", type=float, default=1.0,
                    help="after the W warmup steps, more untimed steps until this many seconds have passed "
                         "(GPU clocks at steady state before the timed region); 0 = none")
    ap.add_argument("--no-end-to-end", action="store_true",
                    help="skip the host Arrow in -> host Arrow out measurement (level-2 entry points)")
    ap.add_argument("--iso-launches", type=int, default=10, help="isolated score-kernel launches after timing")
    ap.add_argument("--depth", type=int, default=2, help="batches in flight (1 = no cross-batch overlap)")
    ap.add_argument("--mark", choices=("auto", "xcd", "sort", "slices"), default="auto",
                    help="H3 presence bitmap: auto (LDS code slices for umi_len 7..12, partition sort for 13), "
                         "partition sort + LDS bitmap, LDS code slices, or the XCD-partitioned mark kernel")
    ap.add_argument("--overlap-score", action="store_true",
                    help="let assign of the previous batch overlap the score kernel (default: score overlaps "
                         "only the latency-bound resolve kernels)")
    ap.add_argument("--emulate-ranks", type=int, default=1,
                    help="(tools) on ONE GPU, act as rank 0 of W: the other W-1 shards' bitmaps are built once "
                         "before timing and the all-gather is replaced by a device copy; predicts per-rank "
                         "step time at N=W minus RCCL time. Never used by the driver.")
    ap.add_argument("--assign-on", choices=("resolve", "separate", "main"), default="main",
                    help="assign of batch k on its own stream one batch later (default), on the main stream "
                         "behind batch k+1's score kernel, or behind its resolve on the resolve stream")
    ap.add_argument("--resolve-streams", type=int, default=1,
                    help="resolve streams: consecutive batches resolve concurrently (needs depth > streams)")
    ap.add_argument("--spec-rounds", type=int, default=0,
                    help="H3 speculative global rounds per resolve (0 = the library default)")
    ap.add_argument("--reuse-gate", choices=("auto", "score", "resolve"), default="auto",
                    help="slot reuse: the main stream (score) or only the resolve waits for the slot's last assign")
    ap.add_argument("--prio", type=str, default="0,0,0", help="stream priorities main,resolve,assign (-1 = high)")
    ap.add_argument("--score-first", action="store_true",
                    help="main stream order score -> mark (round-2 order; default: mark -> score, so the "
                         "resolve overlaps the score kernel)")
    ap.add_argument("--fused-assign", action="store_true",
                    help="score kernel after the batch's resolve, writing the cluster ids too (one pass over the "
                         "codes; main stream: mark(k), score+assign(k-depth+1))")
    ap.add_argument("--mark-stream", action="store_true",
                    help="presence-bitmap mark on a stream of its own (overlaps score + assign)")
    ap.add_argument("--torch-events", action="store_true",
                    help="cross-stream hand-offs through torch events (system-scope release) instead of the "
                         "library's device-scope StreamEvents")
    ap.add_argument("--late-assign", action="store_true",
                    help="host order: enqueue batch k-1's assign after batch k's resolve (round-2 default)")
    ap.add_argument("--no-split-mark", action="store_true",
                    help="the whole presence mark on the main stream (round 4 order) instead of its slice mark + "
                         "merge at the head of the resolve stream")
    ap.add_argument("--assign-lag", type=int, default=0,
                    help="assign batch k-lag at batch k's submit (0: the pipeline's default, 1 per resolve stream)")
    ap.add_argument("--no-c3", action="store_true",
                    help="skip the C3 line part (BASELINE configs[2]: 100M reads, k-mer spectra per UMI group; "
                         "runs after C2 on rank 0 of a one-GPU run)")
    ap.add_argument("--c3-reads", type=int, default=100_000_000)
    ap.add_argument("--no-c3-k16", action="store_true",
                    help="skip the C3 block at the reference's default k (15 / 10: effective 16), min_coverage 5")
    ap.add_argument("--c3-steps", type=int, default=3)
    ap.add_argument("--no-h5", action="store_true",
                    help="skip the H5 block (every group of a 10M-read C3-style run assembled: GPU spectra + "
                         "host assembly threads, round 6)")
    ap.add_argument("--h5-reads", type=int, default=10_000_000)
    return ap.parse_args()


def emulated_shard_bitmap(n_total: int, r: int, W: int, L: int, dev) -> torch.Tensor:
    """The presence bitmap rank r of W would all-gather for its shard of n_total synth-v1
    reads (bench.py --emulate-ranks; tests/test_gpu_bench.py's emulated C4 rank)."""
    s0, c0 = RD.shard_range(n_total, r, W)
    eng = D.ClusterEngine(L, min(n_total, 4 ** L), dev)
    cr = torch.from_numpy(synth.umi_codes(n_total, L, start=s0, count=c0).view(np.int32)).to(dev)
    eng.mark(D.PackedBatch(cr, L))
    bm = eng.build_local_bitmap().clone()
    del cr, eng
    return bm


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    if world > 1:
        # ROGTK_DIST_BACKEND=gloo (tests only): several ranks may then share one GPU
        backend = os.environ.get("ROGTK_DIST_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: the process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    else:
        torch.cuda.set_device(0)
    return world, rank


def barrier(world):
    if world > 1:
        dist.barrier()


def cpu_baseline(codes_h: np.ndarray, L: int, md: int, budget_s: float):
    """Oracle (C++ restatement of the reference algorithm, 1 thread) on a bounded sample."""
    from oracle import pyoracle as P

    def run(k):
        col = P.StrCol.from_fixed(synth.codes_to_ascii(codes_h[:k], L))
        t0 = time.perf_counter()
        P.umi_complexity(col)
        P.hamming(col, TARGET, 1)
        P.umi_cluster(col, L, md)
        return time.perf_counter() - t0

    k = min(len(codes_h), 100_000)
    t = run(k)
    if t < budget_s / 4 and k < len(codes_h):
        k2 = int(min(len(codes_h), k * max(1.0, budget_s / max(t, 1e-6))))
        k2 = max(k2 // 1000 * 1000, k)
        t, k = run(k2), k2
    out = {"value": k / t, "unit": "reads/s", "cores": 1, "kind": "port",
           "sample": f"first {k} reads of the same C2 workload: oracle H1 (7 fields, per-UMI hash maps as "
                     f"umi_score.rs) + H2 hamming + H3 cluster (max_distance {md}), {t:.1f} s on 1 host core"}
    out["multi_thread"] = cpu_baseline_threads(codes_h[:k], L, md)
    return out


def end_to_end(codes_h: np.ndarray, L: int, md: int, iters: int = 3):
    """The drop-in boundary path on the same column: host Arrow LargeUtf8 buffers in ->
    rogtk_umi_complexity_host + rogtk_hamming_host + rogtk_umi_cluster_host (the three
    plugin calls a polars pipeline makes, expressions.rs:1234-1284, 1075-1101, and the
    caller's group_by) -> host Arrow arrays out. Every call uploads the column (the
    plugin ABI hands each expression its input); results land in pinned buffers
    (rogtk_host_alloc), so the D2H is direct DMA."""
    import pyarrow as pa

    import rogtk_amd as rg

    n = len(codes_h)
    asc = synth.codes_to_ascii(codes_h, L)
    offs = np.arange(0, (n + 1) * L, L, dtype=np.int64)
    col = pa.Array.from_buffers(pa.large_binary(), n, [None, pa.py_buffer(offs), pa.py_buffer(asc.reshape(-1))])
    calls = {"umi_complexity_host": lambda: rg.umi_complexity_scores(col),
             "hamming_host": lambda: rg.hamming_within(col, TARGET, 1),
             "umi_cluster_host": lambda: rg.umi_cluster(col, L, md)}
    for f in calls.values():  # warm: device buffers, pinned staging and result blocks
        f()
    ms = {k: [] for k in calls}
    for _ in range(iters):
        for k, f in calls.items():
            t0 = time.perf_counter()
            r = f()
            ms[k].append(1000 * (time.perf_counter() - t0))
            del r
    best = {k: min(v) for k, v in ms.items()}
    total = sum(best.values())
    pcie = 3 * (8 + L) + (48 + 4) + 1 / 8 + 4  # 3 uploads of the column; H1 + H2 bits + H3 ids back
    return {"value": round(n / (total / 1000), 1), "unit": "reads/s", "reads": n,
            "ms": {k: round(v, 2) for k, v in best.items()},
            "pcie_bytes_per_read": round(pcie, 3), "pcie_GBps": round(n * pcie / (total / 1000) / 1e9, 2),
            "path": "host Arrow LargeUtf8 -> rogtk_umi_complexity_host + rogtk_hamming_host + "
                    "rogtk_umi_cluster_host -> host Arrow (pinned result buffers); best of "
                    f"{iters} after a warm-up call"}


def host_threads() -> int:
    """Host threads this job may use: OMP_NUM_THREADS (the GPU box sets the job's CPU
    share there, 16 per GPU) or every core os.cpu_count() shows."""
    n = os.cpu_count() or 1
    try:
        return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))
    except ValueError:
        return n


def cpu_baseline_threads(codes_h: np.ndarray, L: int, md: int, threads: int = 0):
    """The same sample on `threads` host threads: H1 + H2 row-parallel (the oracle's C loops
    release the GIL; like a polars thread pool over chunks) and H3 through the oracle's
    threaded union-find (row passes + edge search split over the threads; identical ids)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import pyoracle as P

    threads = threads or host_threads()
    k = len(codes_h)
    asc = synth.codes_to_ascii(codes_h, L)
    cuts = np.linspace(0, k, threads + 1).astype(np.int64)
    parts = [P.StrCol.from_fixed(asc[a:b]) for a, b in zip(cuts, cuts[1:])]
    col = P.StrCol.from_fixed(asc)

    def h12(c):
        P.umi_complexity(c)
        P.hamming(c, TARGET, 1)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(h12, parts))
    t1 = time.perf_counter()
    P.umi_cluster(col, L, md, threads=threads)
    t2 = time.perf_counter()
    return {"value": k / (t2 - t0), "unit": "reads/s", "cores": threads, "kind": "port",
            "sample": f"same {k} reads, every stage on {threads} host threads (OMP_NUM_THREADS share of "
                      f"{os.cpu_count()} cores): H1+H2 {t1 - t0:.2f} s, H3 (threaded union-find) {t2 - t1:.2f} s"}


def c3_workload(n: int = 100_000_000, steps: int = 3, warmup: int = 1, k: int = 17, min_coverage: int = 20,
                read_len: int = 150, ascii: bool = False, global_only: bool = False,
                group_batch_rows: int = 100_000_000, profile: bool = True) -> dict:
    """BASELINE configs[2] (C3): n synthetic 150-bp reads with 12-bp UMIs resident in HBM;
    one step = H3 exact UMI ids (the caller's group_by('umi'), rogtk/__init__.py:206-214)
    -> rogtk_amd.device.group_spectra: stable group_by of the ids, then the k-mer spectra
    of every group (filter_kmers + CountFilter + censored exts, fracture.rs:105-116),
    k = 17 (effective 32, fracture.rs:246-256), min_coverage 20 (rogtk/__init__.py:212).
    The same path tests/test_gpu_c3.py checks against the oracle. Timed steps run without
    profiling; `profile` adds one untimed step with the pack / gather / k-mer kernels
    bracketed by events on their dispatch packets (kernel execution time)."""
    from rogtk_amd import _lib

    RL, L = read_len, 12
    dev = torch.device("cuda", torch.cuda.current_device())
    t0 = time.time()
    codes = torch.from_numpy(synth.umi_codes(n, L).view(np.int32)).to(dev)
    reads = torch.empty(n * RL, dtype=torch.uint8, device=dev)
    chunk = 2_000_000
    for a in range(0, n, chunk):  # host generator (OpenMP), streamed to HBM
        b = min(n, a + chunk)
        reads[a * RL:b * RL] = torch.from_numpy(synth.reads(n, RL, start=a, count=b - a).reshape(-1)).to(dev)
    offsets = torch.arange(0, (n + 1) * RL, RL, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    gen_s = time.time() - t0
    batch = D.PackedBatch(codes, L)
    eng = D.ClusterEngine(L, min(n, 4 ** L), dev)
    cid = torch.empty(n, dtype=torch.int32, device=dev)
    br = min(n, group_batch_rows)
    _lib.call("rogtk_kmer_set_path", 0 if global_only else 1)
    ev = lambda: torch.cuda.Event(enable_timing=True)
    phases = {"cluster": 0.0, "group_by+kmer": 0.0}
    acc = {}
    path_groups = [0, 0, 0, 0]

    def step(record):
        e0, e1, e3 = ev(), ev(), ev()
        e0.record()
        D.cluster_batch(eng, batch, cid, 0)
        e1.record()
        path_groups[:] = [0, 0, 0, 0]
        acc.update(valid=0, stats=[], calls=0)

        def consume(g0, g1, r):  # per spectrum call
            acc["valid"] += int(r["entry_offsets"][-1].item())
            acc["stats"].append(r["stats"].clone())
            acc["calls"] += 1
            ps = (ctypes.c_int64 * 2)()
            _lib.call("rogtk_kmer_path_stats", ps)
            path_groups[0] += ps[0]
            path_groups[1] += ps[1]
            try:  # groups the repeat certificate took off the LDS kernels (round 4)
                cg = ctypes.c_int64(0)
                _lib.call("rogtk_kmer_certified_groups", ctypes.byref(cg))
                path_groups[2] += cg.value
                _lib.call("rogtk_kmer_lds_rows", ctypes.byref(cg))  # rows the LDS kernels inserted
                path_groups[3] += cg.value
            except Exception:  # an older library (A/B)
                pass

        # max_len: the generator's read length (a bound the caller knows; the device still
        # rejects a longer row), so no reduction over the offsets runs in the step
        _, _, G, _ = D.group_spectra(offsets, reads, cid, k, min_coverage, batch_rows=br, consume=consume,
                                     packed=None if ascii else "auto", max_len=RL)
        e3.record()
        torch.cuda.synchronize()
        if record:
            phases["cluster"] += e0.elapsed_time(e1)
            phases["group_by+kmer"] += e1.elapsed_time(e3)
        return G

    for _ in range(warmup):
        step(False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        G = step(True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    st = (acc["stats"][0] if len(acc["stats"]) == 1 else torch.cat(acc["stats"])).cpu().numpy()
    k_eff = int(st[:, 0].max())
    step_s = el / steps
    obs = n * (RL - k_eff + 1)  # k-mer observations per step (every read is ACGT, full length)
    kernels = {}
    if profile:
        sel = ("pack_reads", "pack_gather", "row_gather", "kmer_wave", "kmer_lds", "kmer_minimizer")
        try:
            D.profile_select(",".join(sel))
        except Exception:  # a library without these kernel names (A/B of older builds)
            sel = ("pack_reads", "row_gather", "kmer_lds", "kmer_minimizer")
            try:
                D.profile_select(",".join(sel))
            except Exception:
                sel = ()
        D.profile_reset()
        D.profile_enable(True)
        step(False)
        torch.cuda.synchronize()
        D.profile_enable(False)
        for kname in sel:
            ms, launches = D.profile_read(kname)
            if launches:
                kernels[kname] = round(1000.0 * ms, 1)  # us per step (all launches of the step)
        D.profile_select(None)
    cu_clk = 256 * 2.4e9  # MI355X: 256 CUs at 2.4 GHz
    peak = HBM_PEAK_GBS
    # Algorithmic HBM bytes per read: the ASCII read once, its UMI code read and
    # its cluster id written (RL + 8). As built (round 5: fused pack + grouped staging): the
    # row and its index / offsets / group in, the packed words and row metadata out.
    alg_b, staged_b = RL + 8, RL + 8 + 16 + 4 + 8 * -(-RL // 32) + 8 + 4
    ach = lambda b: n * b / step_s / 1e9
    out = {
        "workload": f"C3: {n // 1_000_000}M reads x {RL} bp, 12-bp UMI; H3 exact ids -> group_by -> k-mer "
                    f"spectra per group, k={k} (effective {k_eff}), min_coverage {min_coverage}",
        "reads_per_s": round(n * steps / el, 1), "ms_per_step": round(1000 * step_s, 3), "steps": steps,
        "warmup": warmup, "groups": G, "lds_groups": path_groups[0], "global_groups": path_groups[1],
        "certified_empty_groups": path_groups[2],
        "valid_kmers": acc["valid"], "spectrum_calls": acc["calls"],
        "phases_ms": {kk: round(v / steps, 3) for kk, v in phases.items()},
        "kernels_us": kernels,
        "observations_per_s": round(obs / step_s, 1),
        "obs_per_cu_clock": round(obs / step_s / cu_clk, 3),
        "hbm_frac": round(ach(alg_b) / peak, 4),
        "roofline": {
            "step": {"bound": "hbm", "algorithmic_bytes_per_read": alg_b, "achieved": round(ach(alg_b), 1),
                     "peak": peak, "unit": "GB/s", "frac": round(ach(alg_b) / peak, 4)},
            "staged": {"bytes_per_read": staged_b, "achieved": round(ach(staged_b), 1), "peak": peak,
                       "unit": "GB/s", "frac": round(ach(staged_b) / peak, 4)},
        },
        "data": f"synthetic (synth-v1 reads + UMIs, {n // 10} molecules), generated in {gen_s:.1f} s, "
                "resident in HBM",
    }
    if "kmer_lds" in kernels or "kmer_wave" in kernels:
        # the insert kernels alone (the wave-per-group class 2 at k_eff <= 16, round 6, and the
        # workgroup classes 3 / 1 / 4): the observations THEY inserted per CU clock
        lds_obs = path_groups[3] * (RL - k_eff + 1)  # rows of the groups left on the LDS kernels
        us = kernels.get("kmer_wave", 0.0) + kernels.get("kmer_lds", 0.0)
        out["lds_rows"] = path_groups[3]
        out["roofline"]["kmer_lds"] = {"bound": "lds", "kernel": "k_kmer_wave + k_kmer_lds<1|3|4>"
                                       if "kmer_wave" in kernels else "k_kmer_lds<1|3|4>", "us": round(us, 1),
                                       "observations": lds_obs,
                                       "obs_per_cu_clock": round(lds_obs / (us * 1e-6) / cu_clk, 3)}
    if "pack_reads" in kernels:  # HBM stream: RL bytes in, one 64-B block out per read
        a = n * (RL + 64) / (kernels["pack_reads"] * 1e-6) / 1e9
        out["roofline"]["pack_reads"] = {"bound": "hbm", "kernel": "k_pack_reads", "us": kernels["pack_reads"],
                                         "bytes_per_read": RL + 64, "achieved": round(a, 1), "peak": peak,
                                         "unit": "GB/s", "frac": round(a / peak, 4)}
    if "pack_gather" in kernels:
        # k_pack_gather (round 5; its own profile name in round 6): per grouped row, in: the
        # RL-byte ASCII row, its row index (8 B), offsets (16 B) and group id (4 B); out: S
        # packed words (8 B each), observation count (8 B) and length (4 B). DESIGN §3b
        S = -(-RL // 32)
        bpr = RL + 8 + 16 + 4 + 8 * S + 8 + 4
        a = n * bpr / (kernels["pack_gather"] * 1e-6) / 1e9
        out["roofline"]["pack_gather"] = {"bound": "hbm", "kernel": "k_pack_gather", "us": kernels["pack_gather"],
                                          "bytes_per_read": bpr, "achieved": round(a, 1), "peak": peak,
                                          "unit": "GB/s", "frac": round(a / peak, 4)}
    if "row_gather" in kernels:  # 64-B block in, 40 B staged + 12 B of row metadata out
        a = n * (64 + 40 + 12) / (kernels["row_gather"] * 1e-6) / 1e9
        out["roofline"]["row_gather"] = {"bound": "hbm", "kernel": "k_row_gather", "us": kernels["row_gather"],
                                         "bytes_per_read": 116, "achieved": round(a, 1), "peak": peak,
                                         "unit": "GB/s", "frac": round(a / peak, 4)}
    del reads, codes, offsets, batch, eng, cid
    torch.cuda.empty_cache()
    return out


def h5_workload(n: int = 10_000_000, k: int = 10, min_coverage: int = 5, method: str = "compression",
                read_len: int = 150, steps: int = 2, cpu_groups: int = 200) -> dict:
    """H5 over a C3-style run (round 6): n synthetic 150-bp reads with 12-bp UMIs in HBM,
    exact H3 ids (the caller's group_by('umi')), then EVERY group assembled with
    assemble_sequences' defaults (k = 10, min_coverage 5, rogtk/__init__.py:104-116; method
    compression, largest contig as the expression asks, expressions.rs:751): the groups' k-mer
    spectra on the GPU at min_coverage (device.group_spectra: the preliminary graphs), the
    graphs assembled on host threads (rogtk_assemble_groups_host). Beside it, on samples of
    the same groups: the per-group C ABI call (rogtk_assemble_host, its own spectrum round
    trip per group) and the Python restatement (oracle/pyassembly.py, 1 core)."""
    from rogtk_amd import assembly as AS

    RL, L = read_len, 12
    dev = torch.device("cuda", torch.cuda.current_device())
    codes = torch.from_numpy(synth.umi_codes(n, L).view(np.int32)).to(dev)
    reads_h = synth.reads(n, RL)
    values = torch.from_numpy(reads_h.reshape(-1)).to(dev)
    offsets = torch.arange(0, (n + 1) * RL, RL, dtype=torch.int64, device=dev)
    eng = D.ClusterEngine(L, min(n, 4 ** L), dev)
    cid = torch.empty(n, dtype=torch.int32, device=dev)
    D.cluster_batch(eng, D.PackedBatch(codes, L), cid, 0)
    torch.cuda.synchronize()
    threads = host_threads()
    phase = {"spectra_s": 0.0, "assemble_s": 0.0}

    def step():
        outs = []

        def consume(g0, g1, r):
            t0 = time.perf_counter()
            outs.append(AS.assemble_groups(r, method, n_threads=threads))
            phase["assemble_s"] += time.perf_counter() - t0

        t0 = time.perf_counter()
        rows, go, G, _ = D.group_spectra(offsets, values, cid, k, min_coverage, batch_rows=n, consume=consume)
        torch.cuda.synchronize()
        phase["spectra_s"] += time.perf_counter() - t0
        return rows, go, G, outs

    step()  # warm-up: buffers, pinned staging
    phase.update(spectra_s=0.0, assemble_s=0.0)
    t0 = time.perf_counter()
    for _ in range(steps):
        rows, go, G, outs = step()
    el = (time.perf_counter() - t0) / steps
    arr = pa_concat([a for a, _ in outs])
    nc = np.concatenate([c for _, c in outs])
    rows_h, goh = rows.cpu().numpy(), go.cpu().numpy()
    rng = np.random.default_rng(5)
    pick = np.sort(rng.choice(G, size=min(G, cpu_groups), replace=False))
    groups = [[bytes(reads_h[r]) for r in rows_h[goh[g]:goh[g + 1]]] for g in pick]
    import pyarrow as pa
    import rogtk_amd as rg
    got = arr.to_pylist()
    t1 = time.perf_counter()
    per_group = [rg.assemble_sequences(pa.array(items, type=pa.large_binary()), k, min_coverage, method)
                 for items in groups]
    t_per = time.perf_counter() - t1
    from oracle import pyassembly as PA
    t2 = time.perf_counter()
    ref = ["\n".join(PA.assemble(items, k, min_coverage, method, None, None, True, None, False)) for items in groups]
    t_cpu = time.perf_counter() - t2
    same = sum(got[g] == a == b for g, a, b in zip(pick, per_group, ref))
    del values, codes, offsets, cid, eng
    torch.cuda.empty_cache()
    spec_s = phase["spectra_s"] / steps - phase["assemble_s"] / steps
    return {"workload": f"H5: {n // 1_000_000}M reads x {RL} bp, 12-bp UMI; H3 exact ids -> every group's de Bruijn "
                        f"assembly, k={k}, min_coverage {min_coverage}, method {method}, largest contig "
                        f"(assemble_sequences defaults)",
            "groups": int(G), "groups_per_s": round(G / el, 1), "ms_per_step": round(1000 * el, 2), "steps": steps,
            "contigs": int(nc.sum()), "groups_with_contig": int((nc > 0).sum()),
            "split_ms": {"gpu_spectra": round(1000 * spec_s, 2), "host_assembly": round(1000 * phase["assemble_s"] / steps, 2)},
            "host_threads": threads,
            "per_group_abi": {"groups_per_s": round(len(pick) / t_per, 1), "sample_groups": len(pick),
                              "path": "rogtk_assemble_host per group (one GPU spectrum round trip per group)"},
            "cpu_baseline": {"value": round(len(pick) / t_cpu, 1), "unit": "groups/s", "cores": 1, "kind": "port",
                             "sample": f"{len(pick)} random groups of the same run, oracle/pyassembly.py (pure "
                                       f"Python restatement of fracture.rs + djfind.rs), {t_cpu:.1f} s"},
            "sample_identical": f"{same} of {len(pick)} groups: batched == per-group ABI == Python restatement"}


def pa_concat(arrs):
    import pyarrow as pa
    return pa.concat_arrays(arrs) if arrs else pa.array([], type=pa.large_string())


# the single kernels of the C2 step profiled on their own (besides score / assign)
STEP_KERNELS = ("k_slice_bucket", "k_slice_mark", "k_or_partials", "k_scan_rt", "k_local_cc", "k_hook_g", "k_jump",
                "k_roots_check", "k_word_label")


def kernel_bytes(kernel: str, n: int, L: int, n_distinct: int, score_bpr: float) -> float:
    """Algorithmic HBM bytes of one launch (SURVEY §8(d) per-unit figures): n rows, the 4^L
    code space (bitmap 4^L / 8 B, rank table 16 B per 64 codes, word labels 4 + 8 B per 64
    codes), n_distinct present codes (4 B of f each). Rows: score 56.125 B, assign 8 B (code
    in, id out), slice bucket 8 B (code in, segment out), slice mark 4 B + 8 chunk partial
    bitmaps; resolve kernels: the tables they must read or write once."""
    words = 4 ** L // 64
    bm = 4 ** L // 8
    return {"k_score_packed": n * score_bpr, "k_assign": n * 8.0, "k_slice_bucket": n * 8.0,
            "k_slice_mark": n * 4.0 + 8 * bm, "k_or_partials": 9.0 * bm, "k_scan_rt": bm + words * 16.0,
            "k_local_cc": words * 20.0 + n_distinct * 4.125, "k_hook_g": words * 20.0,
            "k_jump": n_distinct * 8.0, "k_roots_check": n_distinct * 4.125,
            "k_word_label": words * 32.0 + n_distinct * 4.0}.get(kernel, 0.0)


def kernel_traffic(kernel: str, reads_per_launch: int):
    """Corrected PMC HBM bytes per launch of `kernel` from the latest committed summary made
    at the same reads per launch (its most-launched instance), or None."""
    for path in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")))):
        try:
            with open(path) as f:
                j = json.load(f)
        except Exception:
            continue
        if j.get("reads_per_launch", 10_000_000) != reads_per_launch:
            continue
        hits = [v for k, v in j.get("kernels", {}).items() if k == kernel or k.startswith(kernel + "<")]
        if hits:
            return max(hits, key=lambda v: v.get("launches_counted", 0)).get("hbm_bytes")
    return None


def load_traffic(reads_per_launch: int, fused: bool = False, key: str = None):
    """Per-launch HBM bytes of k_score_packed (its fused score + assign instance when
    `fused`; another kernel's by `key`) from the latest committed PMC summary made at the
    same reads per launch, if any."""
    key = key or ("score_assign_hbm_bytes_per_launch" if fused else "score_packed_hbm_bytes_per_launch")
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")))
    for path in reversed(files):
        try:
            with open(path) as f:
                j = json.load(f)
        except Exception:
            continue
        if j.get("reads_per_launch", 10_000_000) == reads_per_launch and j.get(key):
            return j[key], os.path.relpath(path, ROOT)
    return None, None


def main():
    args = parse()
    world, rank = setup_dist(args)
    L, md = args.umi_len, args.max_distance
    if args.workload == "C4":  # strong scaling: a fixed total split over the ranks
        n_total = args.total_reads if args.reads_per_gpu is None else args.reads_per_gpu * world
    else:  # C2, weak scaling: a fixed shard per rank
        n_total = (args.reads_per_gpu or 10_000_000) * world
    n = -(-n_total // world)
    start, count = RD.shard_range(n_total, rank, world)
    codes_h = synth.umi_codes(n_total, L, start=start, count=count)
    dev = torch.device("cuda", torch.cuda.current_device())
    codes = torch.from_numpy(codes_h.view(np.int32)).to(dev)
    batch = D.PackedBatch(codes, L)
    exchange = None
    if args.emulate_ranks > 1:
        if world > 1:
            raise SystemExit("--emulate-ranks is a single-process tool")
        W = args.emulate_ranks
        # C2: reads_per_gpu per emulated rank; C4: the fixed total split over the W ranks
        n_total = (args.total_reads if args.reads_per_gpu is None else args.reads_per_gpu * W) \
            if args.workload == "C4" else n * W
        n = count = RD.shard_range(n_total, 0, W)[1]
        others = [emulated_shard_bitmap(n_total, r, W, L, dev) for r in range(1, W)]
        codes_h = synth.umi_codes(n_total, L, start=0, count=n)  # rank 0's shard of the W-rank dataset
        codes = torch.from_numpy(codes_h.view(np.int32)).to(dev)
        batch = D.PackedBatch(codes, L)
        gathered = torch.cat([torch.zeros_like(others[0])] + others)

        def exchange(bm):
            gathered[: bm.numel()].copy_(bm)
            return gathered, W

    D.set_mark_method({"sort": D.MARK_SORT, "slices": D.MARK_SLICES}.get(args.mark, D.MARK_AUTO))
    D.set_spec_rounds(args.spec_rounds)
    pipe = UmiPipeline(L, min(n_total, 4 ** L), count, dev, depth=args.depth, target=TARGET,
                       max_distance=md, group=None,
                       priorities=tuple(int(x) for x in args.prio.split(",")), mark=args.mark,
                       score_alone=not args.overlap_score, exchange=exchange,
                       resolve_streams=args.resolve_streams, assign_on=args.assign_on,
                       reuse_gate=args.reuse_gate, assign_early=not args.late_assign,
                       mark_first=not args.score_first, device_events=not args.torch_events,
                       mark_stream=args.mark_stream, fused_assign=args.fused_assign, assign_lag=args.assign_lag,
                       split_mark=not args.no_split_mark)

    def step():
        pipe.submit(batch)

    for _ in range(args.warmup):
        step()
    pipe.drain()
    torch.cuda.synchronize()
    # untimed settle: more of the same steps until --settle-seconds have passed since the
    # warmup began, so the timed region starts at the GPU's steady-state clocks (a 20-step
    # region is ~8 ms; the first milliseconds of activity run slower)
    settle_steps = 0
    if args.settle_seconds > 0:
        t_s = time.perf_counter()
        while time.perf_counter() - t_s < args.settle_seconds:
            for _ in range(25):
                step()
            settle_steps += 25
            torch.cuda.synchronize()
        pipe.drain()
        torch.cuda.synchronize()
    if not args.no_profile:
        # only the two row-streaming kernels are timed inside the timed region, both by
        # events on their dispatch packets (no packets of their own: the score kernel also
        # by its in-kernel span); the other kernels' bracketing events would add packets
        # to their streams (measured: +0.055 ms/step when all kernels are bracketed)
        try:
            D.profile_select("score_packed,cluster_assign")
        except Exception:  # a library without kernel lists (A/B of older builds)
            D.profile_select("score_packed")
        D.profile_reset()
        D.profile_enable(True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if not args.no_profile and args.profile_every > 1:
            # the timed launches of every profile_every-th step only (their events and the
            # score kernel's in-kernel clocks cost ~10-15 us per step when every step has them)
            D.profile_enable(i % args.profile_every == 0)
        step()
    pipe.drain()
    torch.cuda.synchronize()
    barrier(world)
    el = time.perf_counter() - t0
    kernels = {}
    if not args.no_profile:
        D.profile_enable(False)
        ms, launches = D.profile_read("score_packed")
        sms, slaunches = D.profile_read_span("score_packed")
        if slaunches:
            # the kernel's own execution span (in-kernel device clock: first workgroup in ->
            # last out, what rocprofv3's kernel trace reports); the bracketing stream events
            # also time their own fences (~15 us more per launch)
            kernels["score_packed"] = {"avg_us": 1000.0 * sms / slaunches, "launches": slaunches,
                                       "event_avg_us": 1000.0 * ms / launches if launches else None}
        ams, alaunches = D.profile_read("cluster_assign")
        if alaunches:
            kernels["cluster_assign"] = {"avg_us": 1000.0 * ams / alaunches, "launches": alaunches}
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    stats = pipe.slots[0].eng.stats()
    h3_rounds = pipe.slots[0].eng.rounds()  # global hook rounds the last resolve needed
    # Sustained run (outside the timed region): the same steps back to back for a few
    # seconds, all ranks together; reported beside `value` as a steady-state check
    sustained = None
    if args.sustain_seconds > 0:
        barrier(world)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        k_sus = 0
        while time.perf_counter() - t1 < args.sustain_seconds:
            for _ in range(50):
                step()
            k_sus += 50
            torch.cuda.synchronize()  # bounds the queue; a drain per 50 steps
        pipe.drain()
        torch.cuda.synchronize()
        el_sus = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([el_sus], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_sus = float(t.item())
        sustained = {"value": round(n_total * k_sus / el_sus, 1), "steps": k_sus, "seconds": round(el_sus, 2),
                     "ms_per_step": round(1000 * el_sus / k_sus, 4)}

    # Outside the timed region: a few more pipelined steps with every kernel bracketed,
    # for the per-phase breakdown (kernels_us; these steps are not timed).
    breakdown = {}
    per_kernel = {}
    if not args.no_profile:
        pipe.drain()  # the window then holds exactly w batches' kernels
        torch.cuda.synchronize()
        D.profile_select(None)
        D.profile_reset()
        D.profile_enable(True)
        w = min(args.steps, 5)
        for _ in range(w):
            step()
        pipe.drain()
        torch.cuda.synchronize()
        D.profile_enable(False)
        for k in ("score_packed", "cluster_mark", "cluster_bitmap", "cluster_scan", "cluster_compact", "cluster_union",
                  "cluster_flatten", "cluster_label", "cluster_assign", "cluster_resolve"):
            ms, launches = D.profile_read(k)
            if launches:
                breakdown[k] = round(1000.0 * ms / launches, 2)
        # every kernel of the step on its own dispatch-packet events (as rocprofv3's kernel
        # trace: from the packet's start, so a kernel whose workgroups wait for CU room counts
        # that wait), per launch and per step (all launches of one batch)
        for name, k in (("k_score_packed", "score_packed"), ("k_assign", "cluster_assign")) + tuple(
                (x, x) for x in STEP_KERNELS):
            ms, launches = D.profile_read(k)
            if launches:
                per_kernel[name] = {"avg_us": round(1000.0 * ms / launches, 2), "launches_per_step": launches / w,
                                    "per_step_us": round(1000.0 * ms / w, 2)}
    # Outside the timed region: the same score kernel launched alone (nothing else on
    # the GPU), so its duration is the kernel's own, not the pipeline-shared one.
    iso = None
    if not args.no_profile:
        slot = pipe.slots[0]
        torch.cuda.synchronize()
        D.profile_reset()
        D.profile_enable(True)
        for _ in range(args.iso_launches):
            if args.fused_assign:
                D.score_assign_packed(batch, slot.eng, slot.cid, slot.scores, TARGET, 1, None, slot.within)
            else:
                D.score_packed(batch, slot.scores, TARGET, 1, None, slot.within)
        torch.cuda.synchronize()
        D.profile_enable(False)
        ms, launches = D.profile_read_span("score_packed")
        if launches:
            iso = 1000.0 * ms / launches

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    ms_per_step = 1000.0 * el / args.steps
    value = n_total * args.steps / el if args.emulate_ranks == 1 else n * args.emulate_ranks * args.steps / el
    # roofline of the dominant kernel: algorithmic bytes per read of k_score_packed
    #   in: 4 B packed code; out: 6 x 8 B f64 fields + 4 B longest run + 1/8 B within bit
    # + the u32 cluster id when the score kernel assigns its own batch (--fused-assign)
    bpr = 4 + 48 + 4 + 0.125 + (4 if args.fused_assign else 0)
    roof = None
    if "score_packed" in kernels:
        avg_s = kernels["score_packed"]["avg_us"] * 1e-6
        achieved = count * bpr / avg_s / 1e9
        traffic, src = load_traffic(count, fused=args.fused_assign)
        roof = {"kernel": "k_score_packed", "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": src,
                "algorithmic_bytes_per_launch": int(count * bpr), "bytes_per_read": bpr,
                "avg_us": round(kernels["score_packed"]["avg_us"], 2),
                "timing": "in-kernel span (device wall clock, first workgroup entry to last exit) of "
                          + ("every launch" if args.profile_every <= 1 else f"launches of every {args.profile_every}th step")
                          + " in the timed region",
                "launches_timed": kernels["score_packed"]["launches"],
                "event_avg_us": (round(kernels["score_packed"]["event_avg_us"], 2)
                                 if kernels["score_packed"]["event_avg_us"] else None),
                "measured_over": f"timed region, {args.depth} batches in flight (kernel overlaps the resolve "
                                 f"of the previous batch" + (" and assign" if args.overlap_score else "") + ")"}
        # the whole step against the same roofline: SURVEY §8d's 60 B/read (4 B code in;
        # 48 + 4 B of H1 fields, 4 B cluster id out) + the within bit + the 4^L tables once
        # per batch (presence bitmap 4^L / 8 B + labels 4^L x 4 B read and written)
        step_bytes = count * (60 + 0.125) + (4 ** L) // 8 + 2 * 4 * (4 ** L)
        roof["step"] = {"algorithmic_bytes": int(step_bytes), "achieved": round(step_bytes / (el / args.steps) / 1e9, 1),
                        "frac": round(step_bytes / (el / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                        "note": "whole pipelined step (all kernels, ms_per_step) vs SURVEY §8d's algorithmic bytes"}
        # the kernel with the largest share of the step's device time among ALL kernels of the
        # step (per_kernel: dispatch-packet events, untimed steps), against its §8(d) bytes
        # (kernel_bytes) and its corrected PMC traffic from the latest committed summary
        if per_kernel:
            dk = max(per_kernel, key=lambda k: per_kernel[k]["per_step_us"])
            d = per_kernel[dk]
            d_bytes = kernel_bytes(dk, count, L, stats["n_distinct"], bpr)
            d_ach = d_bytes / (d["avg_us"] * 1e-6) / 1e9
            d_traffic = (traffic if dk == "k_score_packed" else kernel_traffic(dk, count))
            roof["dominant"] = {"kernel": dk, "avg_us": d["avg_us"], "per_step_us": d["per_step_us"],
                                "launches_per_step": d["launches_per_step"],
                                "algorithmic_bytes_per_launch": int(d_bytes), "achieved": round(d_ach, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(d_ach / HBM_PEAK_GBS, 4),
                                "traffic": d_traffic,
                                "traffic_ratio": round(d_traffic / d_bytes, 3) if d_traffic else None,
                                "per_step_us_all": {k: v["per_step_us"] for k, v in
                                                    sorted(per_kernel.items(), key=lambda kv: -kv[1]["per_step_us"])},
                                "timing": "HIP events on each kernel's dispatch packet, 5 untimed pipelined steps "
                                          "after the timed region"}
        if iso:
            a_iso = count * bpr / (iso * 1e-6) / 1e9
            roof["isolated"] = {"avg_us": round(iso, 2), "achieved": round(a_iso, 1),
                                "frac": round(a_iso / HBM_PEAK_GBS, 4), "launches": args.iso_launches,
                                "note": "same kernel, same batch, launched alone after the timed region"}
    sort_mark = pipe.sort_mark
    c3 = c3_k16 = None
    if world == 1 and not args.no_c3 and args.emulate_ranks == 1:
        del pipe, batch, codes
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        c3 = c3_workload(args.c3_reads, steps=args.c3_steps, warmup=1)
        if not args.no_c3_k16:
            # the reference's own operating point: assemble_sequences defaults k = 10 and the
            # docstring's k = 15 (rogtk/__init__.py:106-107, 211-212), both effective 16
            # (fracture.rs:246-256), min_coverage 5
            c3_k16 = c3_workload(args.c3_reads, steps=args.c3_steps, warmup=1, k=15, min_coverage=5)
    h5 = None
    if world == 1 and not args.no_h5 and args.emulate_ranks == 1:
        h5 = h5_workload(args.h5_reads)
    e2e = None
    if not args.no_end_to_end and args.emulate_ranks == 1:
        e2e = end_to_end(codes_h[: min(count, 10_000_000)], L, md)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(codes_h, L, md, args.cpu_seconds)
        cpu["cores_available"] = os.cpu_count()
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "reads/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.workload == "C4" else "weak",
        "vs_baseline": None,
        "dtype": "u32/f64",
        "data": "synthetic (synth-v1: seeded 12-bp UMIs, N/10 molecules, 0.001/base UMI errors), packed 2-bit SoA resident in HBM",
        "config": {"workload": (f"C4: {n_total // 1_000_000}M reads over {world} GPU(s), " if args.workload == "C4"
                                else f"C2: {count // 1_000_000}M reads per GPU, ")
                               + f"{L}-bp UMI, H1 complexity (7 fields) + H2 Hamming-within + H3 Hamming<=1 "
                                 "cluster ids",
                   "total_reads": n_total,
                   "reads_per_gpu": count, "umi_len": L, "max_distance": md,
                   "n_distinct": stats["n_distinct"], "n_clusters": stats["n_clusters"],
                   "h3_rounds": h3_rounds,
                   "h3_global": "hook+jump rounds",
                   "h3_bitmap": ("LDS code slices" if args.mark in ("auto", "slices") and 7 <= L <= 12 else
                                 "partition sort + LDS bitmap") if sort_mark else "XCD-partitioned mark",
                   "parallelism": f"dp{world} shard-by-record + presence-bitmap all-gather"
                                  + (f" (rank 0 of {args.emulate_ranks} EMULATED on one GPU, no RCCL)"
                                     if args.emulate_ranks > 1 else "")},
        "roofline": roof,
        "sustained": sustained,
        "settle": {"seconds": args.settle_seconds, "steps": settle_steps} if settle_steps else None,
        "end_to_end": e2e,
        "c3": c3,
        "c3_k16": c3_k16,
        "h5": h5,
        "cpu_baseline": cpu,
        "kernels_us": breakdown,
        "kernels_per_step": per_kernel,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _rank_main(argv):
    sys.argv = [sys.argv[0]] + list(argv)
    main()


if __name__ == "__main__":
    _args = parse()
    if _args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started before anything touches the GPU
        from rogtk_amd.launch import run_local_ranks

        from rogtk_amd.launch import visible_gpus

        # (ROGTK_DIST_BACKEND=gloo, tests only: ranks may share a GPU). The count comes from
        # the KFD topology in sysfs: no HIP call in this parent, whose children are spawned
        n_vis = visible_gpus()
        if os.environ.get("ROGTK_DIST_BACKEND", "nccl") == "nccl" and n_vis is not None and n_vis < _args.gpus:
            raise SystemExit(f"bench.py: --gpus {_args.gpus} but {n_vis} GPU(s) visible")
        sys.exit(run_local_ranks(_args.gpus, _rank_main, (sys.argv[1:],)))
    main()
