#!/usr/bin/env python3
"""Sum rocprofv3 PMC counters per kernel (template instance) over the dispatches of a run.

Usage: pmc_kernels.py <out_dir> [substring ...]  (prints "kernel counter total dispatches";
only kernels whose name contains one of the substrings; deletes the per-dispatch CSVs)
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"(k_\w+(<[^()]*>)?)", name)
    return m.group(1) if m else name[:60]


def main():
    d, subs = sys.argv[1], sys.argv[2:]
    agg, cnt = collections.defaultdict(float), collections.Counter()
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if subs and not any(s in k for s in subs):
                continue
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            cnt[(k, r["Counter_Name"])] += 1
    for (k, c), v in sorted(agg.items()):
        print(k, c, int(v), cnt[(k, c)])
    for f in fs:
        os.remove(f)


if __name__ == "__main__":
    main()
