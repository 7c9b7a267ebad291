"""Host-side cost of UmiPipeline.submit (Python + ctypes + HIP enqueue) vs the step time,
with per-call host times of one submit (assign_on from argv[1], default "resolve")."""
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rogtk_amd import device as D, synth
from rogtk_amd import pipeline as PL
from rogtk_amd.pipeline import UmiPipeline
assign_on = sys.argv[1] if len(sys.argv) > 1 else "resolve"
n, L = 10_000_000, 12
codes = torch.from_numpy(synth.umi_codes(n, L).view(np.int32)).cuda()
batch = D.PackedBatch(codes, L)
pipe = UmiPipeline(L, min(n, 4 ** L), n, torch.device("cuda", 0), depth=2, score_alone=True, assign_on=assign_on)
for _ in range(5):
    pipe.submit(batch)
pipe.drain(); torch.cuda.synchronize()
# wrap the engine / device calls to time them on the host
acc = {}
def wrap(obj, name, key):
    f = getattr(obj, name)
    def g(*a, **k):
        t = time.perf_counter(); r = f(*a, **k); acc[key] = acc.get(key, 0.0) + time.perf_counter() - t; return r
    setattr(obj, name, g)
for sl in pipe.slots:
    for nm in ("sync", "mark_bitmap", "resolve", "assign"):
        wrap(sl.eng, nm, nm)
wrap(PL.D, "score_packed", "score")
ts = []
t0 = time.perf_counter()
K = 40
for _ in range(K):
    a = time.perf_counter(); pipe.submit(batch); ts.append(time.perf_counter() - a)
pipe.drain(); torch.cuda.synchronize()
el = time.perf_counter() - t0
print(f"assign_on={assign_on} step {el / K * 1e3:.3f} ms; submit host median {np.median(ts) * 1e3:.3f} ms, "
      f"min {min(ts) * 1e3:.3f}; per-call host ms/step: " +
      ", ".join(f"{k} {1e3 * v / K:.3f}" for k, v in acc.items()))
