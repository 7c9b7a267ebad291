#!/usr/bin/env python3
"""C3 measurement (BASELINE.json configs[2]): UMI grouping + k-mer front end on 1 MI355X.

A command-line front end of bench.c3_workload (the C3 part of bench.py's line, which
the driver's bench run reports as "c3"): one step = H3 exact UMI ids -> group_by ->
k-mer spectra per group over synthetic 150-bp reads resident in HBM. Prints one JSON
line (value = reads/s over the timed steps).

Usage: python tools/bench_kmer.py [--reads 10000000 --steps 5 --warmup 1]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


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
                    help="k-mer spectra run over consecutive groups of at most this many rows per call")
    ap.add_argument("--no-profile", action="store_true", help="skip the untimed kernel-bracketed step")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    c3 = bench.c3_workload(args.reads, steps=args.steps, warmup=args.warmup, k=args.k,
                           min_coverage=args.min_coverage, read_len=args.read_len, ascii=args.ascii,
                           global_only=args.global_only, group_batch_rows=args.group_batch_rows,
                           profile=not args.no_profile)
    line = {"metric": "reads/s UMI group_by + k-mer spectra (C3 front end), 150 bp reads, 12 bp UMI, 1 MI355X",
            "value": c3["reads_per_s"], "unit": "reads/s", "n_gpus": 1, **c3}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
