"""Device-side phase timeline of the default bench pipeline without a profiler: HIP events
recorded on each phase's stream right before and after its enqueue (after the stream's
cross-stream waits), so 'start' = when the stream reached the phase. Prints, per batch,
start/end (us, relative) of score, mark, resolve and assign, and the mean step.
Usage: python tools/phase_events.py [n_reads] [steps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rogtk_amd import device as D  # noqa: E402
from rogtk_amd import pipeline as PL  # noqa: E402
from rogtk_amd import synth  # noqa: E402
from rogtk_amd.pipeline import UmiPipeline  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 12
L = 12
codes = torch.from_numpy(synth.umi_codes(n, L).view(np.int32)).cuda()
batch = D.PackedBatch(codes, L)
pipe = UmiPipeline(L, min(n, 4 ** L), n, torch.device("cuda", 0), depth=2, score_alone=True,
                   target=b"ACGTACGTACGT")
for _ in range(4):
    pipe.submit(batch)
pipe.drain()
torch.cuda.synchronize()

recs = []  # (phase, batch index, ev_start, ev_end)
cur = {"k": 0}


def wrap(obj, name, phase, k_of):
    f = getattr(obj, name)

    def g(*a, **kw):
        s = kw.get("stream") or torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r = f(*a, **kw)
        e1.record(s)
        recs.append((phase, k_of(), e0, e1))
        return r
    setattr(obj, name, g)


wrap(PL.D, "score_packed", "score", lambda: cur["k"])
for sl in pipe.slots:
    wrap(sl.eng, "mark_bitmap", "mark", lambda: cur["k"])
    wrap(sl.eng, "resolve", "resolve", lambda: cur["k"])
    wrap(sl.eng, "assign", "assign", lambda: cur["k"] - 1)
ref = torch.cuda.Event(enable_timing=True)
ref.record(torch.cuda.current_stream())
for k in range(K):
    cur["k"] = k
    pipe.submit(batch)
pipe.drain()
end = torch.cuda.Event(enable_timing=True)
end.record(torch.cuda.current_stream())
torch.cuda.synchronize()
rows = {}
for ph, k, e0, e1 in recs:
    rows.setdefault(k, {})[ph] = (ref.elapsed_time(e0) * 1e3, ref.elapsed_time(e1) * 1e3)
print("batch " + "".join(f"{p:>22s}" for p in ("score", "mark", "resolve", "assign")))
for k in sorted(rows):
    print(f"{k:5d} " + "".join(f"{rows[k][p][0]:10.1f}-{rows[k][p][1]:9.1f}  " if p in rows[k] else " " * 22
                               for p in ("score", "mark", "resolve", "assign")))
print(f"mean step {ref.elapsed_time(end) * 1e3 / K:.1f} us over {K} batches")
