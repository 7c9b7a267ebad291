"""Digest of rocprofv3 --pmc runs (one directory per run under a root): per run, per
kernel, per counter: launches and mean value per launch. Usage: pmc_digest.py <root> <out.json>"""
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"\b(k_\w+|gather4)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    root, out = sys.argv[1], sys.argv[2]
    res = {}
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        acc = {}
        for r in csv.DictReader(open(f[0])):
            k = (short(r["Kernel_Name"]), r["Counter_Name"])
            a = acc.setdefault(k, [0, 0.0, []])
            a[0] += 1
            a[1] += float(r["Counter_Value"])
            if len(a[2]) < 12:
                a[2].append(round(float(r["Counter_Value"])))
        run = {}
        for (kern, ctr), (n, tot, first) in acc.items():
            run.setdefault(kern, {})[ctr] = {"launches": n, "mean": round(tot / n, 1), "first": first}
        res[os.path.basename(d)] = run
    json.dump(res, open(out, "w"), indent=1)
    print(f"{len(res)} runs -> {out}")


if __name__ == "__main__":
    main()
