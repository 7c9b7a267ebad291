#!/usr/bin/env python3
"""Experiment: per-phase clocks of k_kmer_lds (needs the ROGTK_KMER_TIMING build of the
library in place of rogtk_amd/librogtk_hip.so; see tools/kmer_timing.sh). Runs
tools/bench_kmer.py's step once more after its own run (extra arguments are passed to it)
and prints the phase split."""
import ctypes
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rogtk_amd import _lib  # noqa: E402

buf = (ctypes.c_ulonglong * 8)()
sys.argv = [os.path.join(ROOT, "tools", "bench_kmer.py"), "--steps", "1", "--warmup", "1"] + sys.argv[1:]
_lib.call("rogtk_kmer_timing", buf)
runpy.run_path(sys.argv[0], run_name="__main__")
_lib.call("rogtk_kmer_timing", buf)
names = ["skip", "load", "insert", "count+scan", "compact", "small-sort+out", "big-sort+out", "tail"]
tot = sum(buf)
for n, v in zip(names, buf):
    print(f"{n:16s} {v / 100.0:14.1f} us(WG-summed) {100.0 * v / max(tot, 1):6.1f} %")
