"""GPU: every A/B environment knob of the H1-H3 device path gives the oracle's outputs.

The knobs (DESIGN.md §7 "A/B switches") are read once per process, so each setting runs
in a child process (one at a time; a few seconds each) over the same synthetic batch; the
parent compares the child's cluster ids, H1 fields and within bits with the oracle.
"""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, L = 1_100_007, 12  # >= 2^20 rows: the slice mark runs its segment (bucket) pass

CHILD = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, {root!r})
from rogtk_amd import device as D
from rogtk_amd import synth
from rogtk_amd.pipeline import UmiPipeline
n, L = {n}, {L}
codes_h = synth.umi_codes(n, L)
codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
batch = D.PackedBatch(codes, L)
out = {{}}
def grab(slot, b):
    out["cid"] = slot.cid[:n].clone()
    out["within"] = slot.within.clone()
    out["comb"] = slot.scores["combined_score"][:n].clone()
    out["run"] = slot.scores["longest_homopolymer_run"][:n].clone()
pipe = UmiPipeline(L, n, n, "cuda", depth=2, target=b"ACGTACGTACGT", max_distance=1, on_assigned=grab,
                   score_alone=True, assign_on={assign_on!r})
pipe.submit(batch)
pipe.drain()
torch.cuda.synchronize()
np.savez({path!r}, **{{k: v.cpu().numpy() for k, v in out.items()}})
"""

KNOBS = [
    ({"ROGTK_LOCAL8": "0"}, "separate"),
    ({"ROGTK_SLICE_BUCKETS": "0"}, "separate"),
    ({"ROGTK_LOCAL8_BIG": "0"}, "main"),
    ({"ROGTK_FUSED_SCAN": "0"}, "main"),
    ({"ROGTK_FUSED_SCAN": "0", "ROGTK_LOCAL8": "0"}, "separate"),
    ({"ROGTK_WORD_EXC1": "0"}, "main"),
    ({"ROGTK_LCC_PREDICT": "0"}, "separate"),
]


@pytest.fixture(scope="module")
def reference():
    from oracle import pyoracle as P
    from rogtk_amd import synth

    codes_h = synth.umi_codes(N, L)
    col = P.StrCol.from_fixed(synth.codes_to_ascii(codes_h, L))
    ref = P.umi_complexity(col)
    _, rw, _ = P.hamming(col, b"ACGTACGTACGT", 1)
    rc, _, _, _ = P.umi_cluster(col, L, 1)
    return ref, rw, rc


@pytest.mark.parametrize("knobs,assign_on", KNOBS, ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items())
                         if isinstance(v, dict) else v)
def test_knob_matches_oracle(reference, tmp_path, knobs, assign_on):
    ref, rw, rc = reference
    path = str(tmp_path / "out.npz")
    env = dict(os.environ, **knobs)
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, n=N, L=L, path=path, assign_on=assign_on)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    z = np.load(path)
    assert np.array_equal(z["cid"].view(np.uint32), rc)
    assert np.array_equal(z["comb"].view(np.uint64), ref["combined_score"].view(np.uint64))
    assert np.array_equal(z["run"].view(np.uint32), ref["longest_homopolymer_run"])
    bits = np.unpackbits(z["within"].view(np.uint8), bitorder="little")[:N].astype(bool)
    assert np.array_equal(bits, rw)


KMER_CHILD = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, {root!r})
from rogtk_amd import device as D
z = np.load({src!r})
offs = torch.from_numpy(z["offsets"]).cuda()
vals = torch.from_numpy(z["values"]).cuda()
keys = torch.from_numpy(z["keys"]).cuda()
out = {{}}
for mc in (1, 3, 30):
    rows, go, G, calls = D.group_spectra(offs, vals, keys, 17, mc)
    out[f"rows{{mc}}"] = rows.cpu().numpy()
    for ci, (g0, g1, r) in enumerate(calls):
        for name, t in r.items():
            if isinstance(t, torch.Tensor):
                out[f"{{mc}}_{{ci}}_{{name}}"] = t.cpu().numpy()
np.savez({path!r}, **out)
"""


def _kmer_column(tmp_path):
    """Families of a few template reads with substitutions (counts reach min_coverage in the
    bigger ones), ragged lengths, and groups of many rows (every LDS class and the global
    path)."""
    rng = np.random.default_rng(11)
    fam = rng.integers(1, 40, 6000)
    fam[::500] = 300  # class 1 / 4 / global-path groups
    n = int(fam.sum())
    keys = np.repeat(np.arange(len(fam), dtype=np.int32), fam)
    rng.shuffle(keys)
    lens = np.where(rng.random(n) < 0.9, 150, rng.integers(20, 300, n))
    tmpl = rng.integers(0, 4, (len(fam), 300))
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    vals = np.empty(int(offs[-1]), np.uint8)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    for i in range(n):
        b = tmpl[keys[i], :lens[i]].copy()
        m = rng.random(lens[i]) < 0.01
        b[m] = rng.integers(0, 4, int(m.sum()))
        vals[offs[i]:offs[i + 1]] = acgt[b]
    src = str(tmp_path / "kcol.npz")
    np.savez(src, offsets=offs, values=vals, keys=keys)
    return src


def test_kmer_prune_knobs_identical(tmp_path):
    """The spectra without the repeat certificate (ROGTK_KMER_CERT=0), without the minimizer
    filter (ROGTK_KMER_MZ=0) or without both are the default's bit for bit, over
    min_coverage 1, 3 and 30."""
    src = _kmer_column(tmp_path)
    outs = []
    for i, knobs in enumerate(({}, {"ROGTK_KMER_CERT": "0"}, {"ROGTK_KMER_MZ": "0"},
                               {"ROGTK_KMER_CERT": "0", "ROGTK_KMER_MZ": "0"})):
        path = str(tmp_path / f"k{i}.npz")
        env = dict(os.environ, **knobs)
        r = subprocess.run([sys.executable, "-c", KMER_CHILD.format(root=ROOT, src=src, path=path)], env=env,
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(dict(np.load(path)))
    a = outs[0]
    for b in outs[1:]:
        assert sorted(a) == sorted(b)
        for name in a:
            assert np.array_equal(a[name], b[name]), name
