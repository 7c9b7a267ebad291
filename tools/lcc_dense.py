#!/usr/bin/env python3
"""Experiment (round 6): per-phase clocks of k_local_cc on the DENSE union of 8 ranks (80M
synth-v1 reads at L = 12: 6.94M distinct codes, 41% of the space; the 7-position tiling),
resolve alone. Needs the -DROGTK_LCC_TIMING build installed as rogtk_amd/librogtk_hip.so."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rogtk_amd import _lib, synth  # noqa: E402
from rogtk_amd import device as D  # noqa: E402

n, L = int(os.environ.get("N", "80000000")), 12
codes = torch.from_numpy(synth.umi_codes(n, L).view(np.int32)).cuda()
eng = D.ClusterEngine(L, min(n, 4 ** L), "cuda")
bm = eng.mark_bitmap(D.PackedBatch(codes, L)).clone()
for _ in range(2):
    eng.resolve(bm, 1, 1)
eng.sync()
torch.cuda.synchronize()
out = (ctypes.c_ulonglong * 8)()
_lib.hip().rogtk_debug_lcc_clock(out)  # zero
D.profile_reset()
D.profile_enable(True)
for _ in range(5):
    eng.resolve(bm, 1, 1)
eng.sync()
torch.cuda.synchronize()
D.profile_enable(False)
_lib.hip().rogtk_debug_lcc_clock(out)
v = list(out)
wg = max(v[5], 1)
print({"n": n, "stats": eng.stats(), "workgroups": v[5], "phase_us": [round(x / wg * 0.01, 2) for x in v[:4]],
       "wg_us": round(v[4] / wg * 0.01, 2)})
for k in ("k_local_cc", "k_hook_g", "k_jump", "k_scan_rt", "k_roots_check", "k_word_label"):
    ms, c = D.profile_read(k)
    if c:
        print(k, round(1000 * ms / 5, 1), "us per resolve,", c // 5, "launches")
