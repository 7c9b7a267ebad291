import sys, numpy as np, pyarrow as pa
sys.path.insert(0, '.')
import torch
import rogtk_amd as rg
from oracle import pyoracle as P
z = np.load('tests/golden/c1_stress.npz')
offs, vals, valid = z['offsets'], z['values'], z['valid']
rows = [vals[offs[i]:offs[i+1]].tobytes() if valid[i] else None for i in range(len(valid))]
col = pa.array(rows, type=pa.large_binary())
got, k, L = rg.umi_cluster(col, 12, 0)
g = np.asarray(got.fill_null(0).to_numpy(zero_copy_only=False)).astype(np.int64)
r = z['cluster_0'].astype(np.int64)
bad = np.nonzero((g != r) & valid)[0]
print('k', k, 'bad', len(bad))
for i in bad:
    print(i, rows[i][:24], len(rows[i]), 'got', g[i], 'want', r[i])
