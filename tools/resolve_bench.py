"""Times the H3 resolve phases at sparse (10M reads) and dense (80M reads) UMI-space occupancy."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rogtk_amd import device as D, synth

for n in [int(x) for x in os.environ.get("NS", "10000000,80000000").split(",")]:
    L = 12
    codes = torch.from_numpy(synth.umi_codes(n, L).view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    eng = D.ClusterEngine(L, min(n, 4**L), "cuda")
    eng.mark(batch); bm = eng.build_local_bitmap().clone()
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    for md in [int(x) for x in os.environ.get("MDS", "1,0").split(",")]:
        eng.resolve(bm, 1, md); torch.cuda.synchronize()
        D.profile_reset(); D.profile_enable(True)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5): eng.resolve(bm, 1, md)
        b.record(); torch.cuda.synchronize(); D.profile_enable(False)
        r = {"resolve_wall_us": round(a.elapsed_time(b) / 5 * 1000, 1)}
        for k in ("cluster_scan", "cluster_compact", "cluster_union", "cluster_flatten", "cluster_label"):
            ms, c = D.profile_read(k)
            if c: r[k] = round(1000 * ms / c, 1)
        st = eng.ws[:64].view(torch.int64).cpu().numpy()
        flags = eng.ws[64:64 + 4 * 16].view(torch.int32).cpu().numpy()
        ecnt = eng.ws[320:320 + 4 * 8].view(torch.int32).cpu().numpy()
        r["edge_counts"] = ecnt.tolist()
        print(f"n={n} md={md} distinct={st[0]} clusters={st[1]} rounds_flags={flags.tolist()}", r, flush=True)
    eng.assign(batch, cid); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5): eng.assign(batch, cid)
    b.record(); torch.cuda.synchronize()
    print(f"  assign_us={a.elapsed_time(b)/5*1000:.1f}", flush=True)
    del eng, codes, batch, bm, cid
    torch.cuda.empty_cache()
