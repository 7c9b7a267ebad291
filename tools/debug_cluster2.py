import sys, numpy as np, pyarrow as pa
sys.path.insert(0, '.')
import torch
import rogtk_amd as rg
z = np.load('tests/golden/c1_stress.npz')
offs, vals, valid = z['offsets'], z['values'], z['valid']
rows = [vals[offs[i]:offs[i+1]].tobytes() if valid[i] else None for i in range(len(valid))]
reg = lambda r: len(r) == 12 and all(c in b'ACGT' for c in r)
irr = [r for r in rows if r is not None and not reg(r)]
def check(name, items, L=12):
    got, k, _ = rg.umi_cluster(pa.array(items, type=pa.large_binary()), L, 0)
    g = np.asarray(got.fill_null(0).to_numpy(zero_copy_only=False)).astype(np.int64)
    regs = sorted({r for r in items if r is not None and reg(r)})
    irs = sorted({r for r in items if r is not None and not reg(r)})
    ids = {s: i for i, s in enumerate(regs)}; ids.update({s: len(regs) + i for i, s in enumerate(irs)})
    exp = np.array([ids[r] if r is not None else 0 for r in items])
    bad = np.nonzero(g != exp)[0]
    print(f"{name}: n={len(items)} k={k} want_k={len(ids)} bad={len(bad)}", [(items[i][:14], g[i], exp[i]) for i in bad[:4]])
check('irregular only', irr)
check('irregular only again', irr)
short = [r for r in irr if len(r) <= 16]
check('irregular short only', short)
check('irregular <=64', [r for r in irr if len(r) <= 64])
check('irregular <=300', [r for r in irr if len(r) <= 300])
check('full', rows)
check('full again', rows)
