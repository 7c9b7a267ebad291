"""Per-phase clocks of k_local_cc (experiment build with -DROGTK_LCC_TIMING, installed as
rogtk_amd/librogtk_hip.so by the caller): the resolve alone on a C2 batch's bitmap, then
the bench's pipelined steps. Prints the mean per-workgroup duration of each phase (us)
and of the whole workgroup, so a kernel that takes twice as long in the pipeline shows
whether its workgroups run slower or start later."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rogtk_amd import _lib, synth  # noqa: E402
from rogtk_amd import device as D  # noqa: E402
from rogtk_amd.pipeline import UmiPipeline  # noqa: E402

TICK_US = 0.01  # wall_clock64: 100 MHz


def read_clk():
    out = (ctypes.c_ulonglong * 8)()
    assert _lib.hip().rogtk_debug_lcc_clock(out) == 0
    v = list(out)
    wg = max(v[5], 1)
    return {"workgroups": v[5], "phase_us": [round(x / wg * TICK_US, 2) for x in v[:4]],
            "wg_us": round(v[4] / wg * TICK_US, 2),
            "unites_per_wg": round(v[6] / wg, 1), "cas_retries_per_wg": round(v[7] / wg, 1)}


def main():
    n, L = 10_000_000, 12
    codes = torch.from_numpy(synth.umi_codes(n, L).view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    eng = D.ClusterEngine(L, n, "cuda")
    bm = eng.mark_bitmap(batch).clone()
    for _ in range(3):
        eng.resolve(bm, 1, 1)
    eng.sync()
    torch.cuda.synchronize()
    read_clk()
    reps = 20
    for _ in range(reps):
        eng.resolve(bm, 1, 1)
        eng.sync()
    torch.cuda.synchronize()
    alone = read_clk()
    pipe = UmiPipeline(L, n, n, "cuda", depth=2, target=b"ACGTACGTACGT", max_distance=1, score_alone=True)
    for _ in range(10):
        pipe.submit(batch)
    pipe.drain()
    torch.cuda.synchronize()
    read_clk()
    for _ in range(40):
        pipe.submit(batch)
    pipe.drain()
    torch.cuda.synchronize()
    piped = read_clk()
    print(json.dumps({"alone": alone, "pipeline": piped}))


if __name__ == "__main__":
    main()
