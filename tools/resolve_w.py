"""Times H3 resolve + assign in isolation (one stream) on the W-shard global bitmap that
rank 0 sees at N=W (bench.py --emulate-ranks data). Run under rocprofv3 for kernel stats."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rogtk_amd import device as D, synth  # noqa: E402
from rogtk_amd import dist as RD  # noqa: E402

L, n = 12, 10_000_000
for W in [int(x) for x in os.environ.get("WS", "1,8").split(",")]:
    n_total = n * W
    eng = D.ClusterEngine(L, min(n_total, 4 ** L), "cuda")
    bms = []
    for r in range(W):
        s0, c0 = RD.shard_range(n_total, r, W)
        cr = torch.from_numpy(synth.umi_codes(n_total, L, start=s0, count=c0).view(np.int32)).cuda()
        eng.mark(D.PackedBatch(cr, L))
        bms.append(eng.build_local_bitmap().clone())
        if r == 0:
            batch = D.PackedBatch(cr, L)
        else:
            del cr
    gathered = torch.cat(bms)
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(3):
        eng.resolve(gathered, W, 1)
        eng.assign(batch, cid)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        eng.resolve(gathered, W, 1)
        eng.assign(batch, cid)
    b.record()
    torch.cuda.synchronize()
    st = eng.stats()
    print(f"W={W} resolve+assign {a.elapsed_time(b) / 10 * 1000:.1f} us  distinct={st['n_distinct']} "
          f"clusters={st['n_clusters']} rounds={eng.rounds()}", flush=True)
    del eng, gathered, bms, batch, cid
    torch.cuda.empty_cache()
