"""Turn a tools/profile_bench.sh run (gpurun_out/prof_bench) into committed files:

profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (bench.py)
profiles/<tag>_pmc.json           per-kernel HBM traffic from separate FETCH_SIZE /
                                  WRITE_SIZE passes, corrected as MI355X_MICROARCH.md
                                  prescribes (units KB; gfx950 FETCH_SIZE x2 for wide
                                  streaming reads), per launch
profiles/<tag>_score_split.json   k_score_packed dispatch durations from the trace, split into
                                  the bench's phases (warmup+timed pipeline vs the isolated
                                  launches after the timed region) so they can be compared with
                                  the bench line's roofline.avg and roofline.isolated
Usage: python tools/summarize_profiles.py <tag> [reads_per_launch] [isolated_launches]
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "prof_bench")
# PROFILES_OUT: where the summaries go (default profiles/; on the GPU box a directory under
# gpurun_out/, which is what comes back)
OUT = os.environ.get("PROFILES_OUT", os.path.join(ROOT, "profiles"))


def short(name):
    n = name.replace("void ", "").replace("rogtk::(anonymous namespace)::", "")
    return n.split("(")[0]


def counters(kind, counter):
    rows = list(csv.DictReader(open(os.path.join(SRC, kind, "run_counter_collection.csv"))))
    by = {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        by.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in by.items()}, {k: len(v) for k, v in by.items()}


def main():
    tag = sys.argv[1]
    reads = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
    n_iso = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    os.makedirs(OUT, exist_ok=True)
    shutil.copy(os.path.join(SRC, "trace", "run_kernel_stats.csv"), os.path.join(OUT, f"{tag}_kernel_stats.csv"))
    stats = {short(r["Name"]): r for r in csv.DictReader(open(os.path.join(SRC, "trace", "run_kernel_stats.csv")))}
    fetch, nf = counters("fetch", "FETCH_SIZE")
    write, nw = counters("write", "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if "rocclr" in k:
            continue
        fb = 2 * fetch.get(k, 0.0) * 1024  # gfx950: FETCH_SIZE reads half the streamed bytes
        wb = write.get(k, 0.0) * 1024
        e = {"fetch_bytes_corrected": round(fb), "write_bytes": round(wb), "hbm_bytes": round(fb + wb),
             "launches_counted": max(nf.get(k, 0), nw.get(k, 0))}
        if k in stats:
            e["avg_us"] = round(float(stats[k]["AverageNs"]) / 1000, 2)
            e["hbm_GBps"] = round((fb + wb) / (float(stats[k]["AverageNs"]) * 1e-9) / 1e9, 1)
        kernels[k] = e
    sp = [k for k in kernels if k.startswith("k_score_packed")]
    out = {"tag": tag, "reads_per_launch": reads,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (with --kernel-trace); "
                     "KB*1024; FETCH_SIZE doubled (gfx950 reports half of wide streaming reads, "
                     "MI355X_MICROARCH.md HBM section); WRITE_SIZE exact for 16-B/lane streaming stores",
           "kernels": kernels}
    asg = [k for k in kernels if k.startswith("k_assign")]
    if asg:  # bench.py's roofline.dominant reads this when k_assign takes the most time
        out["assign_hbm_bytes_per_launch"] = kernels[asg[0]]["hbm_bytes"]
        out["assign_bytes_per_read"] = round(kernels[asg[0]]["hbm_bytes"] / reads, 2)
    if sp:
        out["score_packed_hbm_bytes_per_launch"] = kernels[sp[0]]["hbm_bytes"]
        out["score_packed_bytes_per_read"] = round(kernels[sp[0]]["hbm_bytes"] / reads, 2)
    tr = [r for r in csv.DictReader(open(os.path.join(SRC, "trace", "run_kernel_trace.csv")))
          if short(r["Kernel_Name"]).startswith("k_score_packed")]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in tr]
    if d:
        pipe, iso = d[:-n_iso] if len(d) > n_iso else d, d[-n_iso:] if len(d) > n_iso else []
        split = {"kernel": short(tr[0]["Kernel_Name"]), "dispatches": len(d),
                 "pipeline_avg_us": round(sum(pipe) / len(pipe), 2), "pipeline_dispatches": len(pipe),
                 "isolated_avg_us": round(sum(iso) / len(iso), 2) if iso else None, "isolated_dispatches": len(iso),
                 "all_avg_us": round(sum(d) / len(d), 2)}
        with open(os.path.join(OUT, f"{tag}_score_split.json"), "w") as f:
            json.dump(split, f, indent=1)
        print(json.dumps(split))
    with open(os.path.join(OUT, f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main()
