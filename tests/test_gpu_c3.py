"""GPU: BASELINE config C3's path — the one tools/bench_kmer.py measures — under the oracle.

Pipeline (rogtk_amd.device): synth-v1 150-bp reads + 12-bp UMIs in HBM -> H3 exact UMI ids
(cluster_batch, max_distance 0: the caller's group_by('umi'), rogtk/__init__.py:206-214)
-> group_spectra (rogtk_group_by_key + rogtk_kmer_spectrum_dev over runs of consecutive
groups, k = 17 -> effective 32, min_coverage 20 as rogtk/__init__.py:212) -> every group's
(k-mer, censored exts, count) list and stats vs oracle/kmer_oracle.cpp (fracture.rs:105-146,
217-256 + debruijn filter_kmers, restated).

* 1M reads (~111k groups) plus injected groups that force every size class and hand-off:
  15 / 40 / 100 unrelated reads (distinct k-mers past class 3's and class 1's tables),
  250 and 700 reads of one template (class 4 and the global radix path), 3 / 4 clean
  templates (the wave class's sort bound), compared in full; k_eff 8 / 16 / 32.
* 100M reads at k = 15, min_coverage 5 (the reference's default, round 6): properties,
  2,600 groups vs the oracle, digest against the path without the wave class.
* 100M reads (the C3 configuration, 1 and 11 spectrum calls): size-independent properties
  over every group (n_sequences, node/terminal/isolated counts recomputed from the returned
  exts, counts >= min_coverage, ascending k-mers), the groups the minimizer filter decided
  (emptied and kept) and 300 random groups compared in full with the oracle, and one digest
  of every output for one call, 10M-row calls and the path without the repeat certificate
  and the minimizer filter (round 5).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
RL, UL, K, MINCOV = 150, 12, 17, 20
THREADS = min(16, os.cpu_count() or 1)


INJECT = ((15, "random"), (40, "random"), (100, "random"), (250, "template"), (700, "template"),
          (18, "multi3"), (24, "multi4"), (64, "multi4"), (65, "template"), (20, "polyT"))


def _inject(reads, codes, rng):
    """Overwrite rows with groups of chosen shapes (fresh UMI codes): random rows (distinct
    k-mers past the wave class's and class 3's / class 1's tables), one template (class 4, the
    global radix path, and 65 rows: one past the wave class), and 3 / 4 templates of 6 clean
    copies each (k_eff 16, min_coverage <= 6: ~405 / ~540 valid k-mers, the latter past the
    wave class's 512-entry sort; 64 rows: the wave class's row bound), and one template with
    a 90-base run of T (the all-T 16-mer, whose key is the wave table's empty mark)."""
    n = len(codes)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    rows = rng.choice(n, size=sum(sz for sz, _ in INJECT), replace=False)
    at = 0
    used = set(np.unique(codes).tolist())
    for size, kind in INJECT:
        sel = rows[at:at + size]
        at += size
        c = int(rng.integers(0, 4 ** UL))
        while c in used:
            c = int(rng.integers(0, 4 ** UL))
        used.add(c)
        codes[sel] = c
        if kind == "random":
            reads[sel] = acgt[rng.integers(0, 4, size=(size, RL))]
        elif kind.startswith("multi"):
            tpls = acgt[rng.integers(0, 4, size=(int(kind[5:]), RL))]
            for j, r in enumerate(sel):
                reads[r] = tpls[j % len(tpls)]
        else:
            tpl = acgt[rng.integers(0, 4, size=RL + 60)]
            if kind == "polyT":
                tpl[40:130] = ord("T")
            for j, r in enumerate(sel):
                a = int(rng.integers(0, 60))
                reads[r] = tpl[a:a + RL]
                if rng.random() < 0.2:
                    reads[r, int(rng.integers(RL))] = acgt[int(rng.integers(4))]


def _run_c3(codes_h, reads_h, min_cov=MINCOV, batch_rows=10_000_000, packed="auto", k=K):
    import torch

    from rogtk_amd import device as D

    n = len(codes_h)
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    values = torch.from_numpy(reads_h.reshape(-1)).cuda()
    offsets = torch.arange(0, (n + 1) * RL, RL, dtype=torch.int64, device="cuda")
    eng = D.ClusterEngine(UL, min(n, 4 ** UL), "cuda")
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    D.cluster_batch(eng, D.PackedBatch(codes, UL), cid, 0)
    rows, go, G, calls = D.group_spectra(offsets, values, cid, k, min_cov, batch_rows=batch_rows, packed=packed)
    torch.cuda.synchronize()
    return rows, go, G, calls


def _concat(calls, G):
    km, ex, cn, st = [], [], [], []
    eo = [np.zeros(1, np.int64)]
    base = 0
    for g0, g1, r in calls:
        k = r["kmers"].cpu().numpy().view(np.uint64)
        km.append(k)
        ex.append(r["exts"].cpu().numpy())
        cn.append(r["counts"].cpu().numpy().view(np.uint16))
        st.append(r["stats"].cpu().numpy())
        e = r["entry_offsets"].cpu().numpy()
        eo.append(e[1:] + base)
        base += int(e[-1])
    km = np.concatenate(km) if km else np.zeros((0, 2), np.uint64)
    return {"kmer_hi": km[:, 0], "kmer_lo": km[:, 1], "exts": np.concatenate(ex), "counts": np.concatenate(cn),
            "group_offsets": np.concatenate(eo), "stats": np.concatenate(st)}


@pytest.mark.parametrize("k,min_cov,batch_rows,packed,filt,path", [
    (K, MINCOV, 10_000_000, "auto", 0, 1), (K, 2, 200_000, "auto", 0, 1), (K, MINCOV, 10_000_000, None, 0, 1),
    (K, 3, 200_000, "auto", 1, 1), (K, MINCOV, 10_000_000, "blocks", 1, 1),
    # the reference's defaults: k = 15 (docstring) and 10 (assemble_sequences), effective 16,
    # min_coverage 5 (rogtk/__init__.py:106-107, 211-212): the wave-per-group class (round 6),
    # and the same without it (path 2: the workgroup kernels take those groups)
    (15, 5, 10_000_000, "auto", 1, 1), (10, 5, 200_000, "blocks", 1, 1), (15, 5, 10_000_000, "auto", 1, 2),
    (15, 3, 10_000_000, None, 1, 1), (7, 6, 10_000_000, "auto", 1, 1)])
def test_c3_path_1m_vs_oracle(k, min_cov, batch_rows, packed, filt, path):
    """packed "auto" (150-bp rows: "fused"): rows packed from their ASCII bytes in group
    order with the certificate (rogtk_kmer_spectrum_fused); "blocks": staged from the 2-bit
    block column (rogtk_pack_reads); None: from the ASCII bytes without a certificate.
    filt: with the minimizer filter (rogtk_kmer_set_filter). path: rogtk_kmer_set_path."""
    from oracle import pyoracle as P
    from rogtk_amd import _lib
    from rogtk_amd import synth
    import ctypes

    n = 1_000_000
    rng = np.random.default_rng(17 + min_cov)
    codes_h = synth.umi_codes(n, UL).copy()
    reads_h = synth.reads(n, RL).copy()
    _inject(reads_h, codes_h, rng)
    _lib.call("rogtk_kmer_set_path", path)
    _lib.call("rogtk_kmer_set_filter", filt)
    try:
        rows, go, G, calls = _run_c3(codes_h, reads_h, min_cov, batch_rows, packed, k)
    finally:
        _lib.call("rogtk_kmer_set_filter", 1)
        _lib.call("rogtk_kmer_set_path", 1)
    ps = (ctypes.c_int64 * 2)()
    _lib.call("rogtk_kmer_path_stats", ps)
    order = np.argsort(codes_h, kind="stable")
    assert np.array_equal(rows.cpu().numpy(), order)  # group_by: ids in code order, rows stable
    _, starts = np.unique(codes_h[order], return_index=True)
    goh = np.concatenate([starts, [n]]).astype(np.int64)
    assert G == len(starts) and np.array_equal(go.cpu().numpy(), goh)
    got = _concat(calls, G)
    ref = P.kmer_spectrum(P.StrCol.from_fixed(reads_h[order]), k, min_cov, False, goh, threads=THREADS)
    assert np.array_equal(got["group_offsets"], ref["group_offsets"])
    assert np.array_equal(got["stats"], ref["stats"])
    for f in ("kmer_hi", "kmer_lo", "exts", "counts"):
        assert np.array_equal(got[f], ref[f]), f
    assert G > 100_000 and len(calls) >= (1 if batch_rows >= n else 5)
    assert (got["stats"][:, 0] == (8 if k <= 8 else 16 if k <= 16 else 32)).all()


def _props(calls, min_cov, k_eff=32):
    """Size-independent properties of one run, checked on the device (1.28G entries at k_eff
    16); returns (sum n_sequences, groups, a digest)."""
    import torch

    nseq, groups = 0, 0
    digest = torch.zeros((), dtype=torch.int64, device="cuda")
    offs = [0, 0, 0, 0]  # positions run on across calls: the digest does not depend on the split
    sign = torch.tensor(-(2 ** 63), dtype=torch.int64, device="cuda")
    for g0, g1, r in calls:
        st = r["stats"].reshape(-1, 5)
        eo = r["entry_offsets"]
        G = st.shape[0]
        cnt = eo[1:] - eo[:-1]
        assert bool((st[:, 0] == k_eff).all())
        assert torch.equal(st[:, 2], cnt)  # node_count = entries
        ex = r["exts"].to(torch.int32)
        gid = torch.repeat_interleave(torch.arange(G, dtype=torch.int32, device="cuda"), cnt)
        l0, r0 = (ex & 0xF) == 0, (ex >> 4) == 0
        del ex
        for col, m in ((3, l0 | r0), (4, l0 & r0)):
            acc = torch.zeros(G, dtype=torch.int32, device="cuda").index_add_(0, gid, m.to(torch.int32))
            assert torch.equal(acc.to(torch.int64), st[:, col])
        del l0, r0
        assert bool(((r["counts"].to(torch.int32) & 0xFFFF) >= min_cov).all())
        lo = r["kmers"].reshape(-1, 2)[:, 1] ^ sign  # unsigned order as signed
        if lo.numel() > 1:  # ascending k-mers within a group (k_eff <= 32: the lo word)
            assert bool(((lo[1:] > lo[:-1]) | (gid[1:] != gid[:-1])).all())
        del lo, gid
        nseq += int(st[:, 1].sum())
        groups += G
        for i, t in enumerate((r["kmers"], r["exts"].to(torch.int64), r["counts"].to(torch.int64), r["stats"])):
            v = t.reshape(-1).to(torch.int64)
            w = torch.arange(offs[i] + 1, offs[i] + v.numel() + 1, device=v.device, dtype=torch.int64) * 0x9E3779B1
            digest += (v * w).sum()
            offs[i] += v.numel()
    return nseq, groups, int(digest.item())


def _c3_100m_inputs():
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    n = 100_000_000
    codes_h = synth.umi_codes(n, UL)
    values = torch.empty(n * RL, dtype=torch.uint8, device="cuda")
    chunk = 5_000_000
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        values[a * RL:b * RL] = torch.from_numpy(synth.reads(n, RL, start=a, count=b - a).reshape(-1)).cuda()
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    offsets = torch.arange(0, (n + 1) * RL, RL, dtype=torch.int64, device="cuda")
    eng = D.ClusterEngine(UL, min(n, 4 ** UL), "cuda")
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    D.cluster_batch(eng, D.PackedBatch(codes, UL), cid, 0)
    return n, values, offsets, cid


def c3_100m_digest():
    """(properties + digest, groups, calls) of the default C3 path at 100M reads, one spectrum
    call; the knob child below runs it under other environments."""
    import torch

    from rogtk_amd import device as D

    n, values, offsets, cid = _c3_100m_inputs()
    rows, go, G, calls = D.group_spectra(offsets, values, cid, K, MINCOV, batch_rows=100_000_000)
    torch.cuda.synchronize()
    return _props(calls, MINCOV) + (G, len(calls))


KNOB_CHILD = r"""
import importlib.util, json, sys
sys.path.insert(0, {root!r})
spec = importlib.util.spec_from_file_location("c3t", {path!r})
m = importlib.util.module_from_spec(spec)
spec.loader.exec_module(m)
print("DIGEST " + json.dumps(list(m.c3_100m_digest())), flush=True)
"""


def _oracle_groups(pick, rows_h, goh, values, n, calls, k=K, min_cov=MINCOV):
    """Groups `pick` (indices of one run's groups) in full against the oracle."""
    from oracle import pyoracle as P
    import torch

    sub_rows, sub_go = [], [0]
    for g in pick:
        rr = rows_h[goh[g]:goh[g + 1]]
        sub_rows.append(rr)
        sub_go.append(sub_go[-1] + len(rr))
    sub_rows = np.concatenate(sub_rows)
    reads_sub = values.view(n, RL)[torch.from_numpy(sub_rows).cuda()].cpu().numpy()
    ref = P.kmer_spectrum(P.StrCol.from_fixed(reads_sub), k, min_cov, False, np.array(sub_go), threads=THREADS)
    starts = np.concatenate([[0], np.cumsum([len(c[2]["stats"]) for c in calls])])
    nonempty = 0
    for j, g in enumerate(pick):
        ci = int(np.searchsorted(starts, g, side="right")) - 1
        r = calls[ci][2]
        lg = g - starts[ci]
        eo = r["entry_offsets"][lg:lg + 2].cpu().numpy()
        a, b = int(eo[0]), int(eo[1])
        ra, rb = int(ref["group_offsets"][j]), int(ref["group_offsets"][j + 1])
        assert np.array_equal(r["stats"][lg].cpu().numpy(), ref["stats"][j]), g
        km = r["kmers"][a:b].cpu().numpy().view(np.uint64)
        assert np.array_equal(km[:, 0], ref["kmer_hi"][ra:rb]) and np.array_equal(km[:, 1], ref["kmer_lo"][ra:rb]), g
        assert np.array_equal(r["exts"][a:b].cpu().numpy(), ref["exts"][ra:rb]), g
        assert np.array_equal(r["counts"][a:b].cpu().numpy().view(np.uint16), ref["counts"][ra:rb]), g
        nonempty += rb > ra
    return nonempty


def test_c3_full_size_100m_properties():
    """C3 at full size (100M reads): properties of every group, the groups the minimizer
    filter decided (>= 1000 it emptied and every one / >= 1000 it kept) plus 300 random
    groups in full against the oracle, a digest of every output identical for one call and
    10M-row calls, and identical to the path without the repeat certificate and the
    minimizer filter (ROGTK_KMER_CERT=0 ROGTK_KMER_MZ=0, a child process)."""
    import json
    import subprocess
    import sys

    import torch

    from rogtk_amd import _lib
    from rogtk_amd import device as D

    n, values, offsets, cid = _c3_100m_inputs()
    print("C3 100M: reads in HBM", flush=True)
    results = []
    for run in range(2):  # one spectrum call (the default), then calls of 10M rows
        dec = None
        if run == 0:  # the minimizer filter's decision per group (tests-only hook)
            dec = torch.zeros(n + 1, dtype=torch.uint8, device="cuda")
            _lib.call("rogtk_kmer_debug_filter", D._p(dec), n + 1)
        try:
            # run 0: the default (fused staging), one call; run 1: the block column, 10M-row calls
            rows, go, G, calls = D.group_spectra(offsets, values, cid, K, MINCOV,
                                                 batch_rows=100_000_000 if run == 0 else 10_000_000,
                                                 packed="auto" if run == 0 else "blocks")
            torch.cuda.synchronize()
        finally:
            _lib.call("rogtk_kmer_debug_filter", None, 0)
        results.append(_props(calls, MINCOV) + (G, len(calls)))
        print(f"C3 100M run {run}: {results[-1]}", flush=True)
        if run == 0:
            rng = np.random.default_rng(3)
            goh = go.cpu().numpy()
            rows_h = rows.cpu().numpy()
            d = dec[:G].cpu().numpy()
            emptied, kept = np.flatnonzero(d == 1), np.flatnonzero(d >= 2)
            print(f"filter: {len(emptied)} emptied, {len(kept)} kept", flush=True)
            assert len(emptied) >= 1000 and len(kept) >= 1
            pick_k = np.sort(rng.choice(kept, size=min(len(kept), 1500), replace=False))
            ne = min(len(emptied), max(1500, 2000 - len(pick_k)))
            pick_e = np.sort(rng.choice(emptied, size=ne, replace=False))
            assert len(pick_e) + len(pick_k) >= 2000
            # every emptied group's output is empty (stats say node_count 0); checked in full
            # against the oracle for the sample
            assert _oracle_groups(pick_e, rows_h, goh, values, n, calls) == 0
            nk = _oracle_groups(pick_k, rows_h, goh, values, n, calls)
            print(f"kept groups with valid k-mers: {nk} of {len(pick_k)}", flush=True)
            _oracle_groups(np.sort(rng.choice(G, size=300, replace=False)), rows_h, goh, values, n, calls)
        del calls, rows, go
    # bitwise deterministic and independent of the call split (digest of every output array)
    assert results[0][:4] == results[1][:4]
    nseq, groups, _, G, ncalls = results[0]
    assert nseq == n and groups == G and ncalls == 1 and results[1][4] >= 10
    del values, offsets, cid
    torch.cuda.empty_cache()
    # the same outputs without the certificate and the filter (every group through the LDS /
    # global kernels): a child process, the knobs being read once per process
    env = dict(os.environ, ROGTK_KMER_CERT="0", ROGTK_KMER_MZ="0")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-u", "-c", KNOB_CHILD.format(root=root, path=os.path.abspath(__file__))],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    child = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("DIGEST ")][-1][7:])
    assert tuple(child) == results[0], (child, results[0])


def test_c3_full_size_100m_k15():
    """C3 at the reference's default operating point at full size: 100M reads, k = 15
    (effective 16, rogtk/__init__.py:211-212, fracture.rs:246-256), min_coverage 5 - nearly
    every group has valid k-mers and runs the wave-per-group kernel (round 6). Properties of
    every group; 2,000 random groups plus the 300 with the most rows and the 300 with the
    most valid k-mers in full against the oracle; one digest of every output identical for
    one call on the default path and for 10M-row calls without the wave class
    (rogtk_kmer_set_path(2): the workgroup kernels take every LDS group)."""
    import torch

    from rogtk_amd import _lib
    from rogtk_amd import device as D

    k, mc = 15, 5
    n, values, offsets, cid = _c3_100m_inputs()
    print("C3 100M k=15: reads in HBM", flush=True)
    results = []
    for run in range(2):
        _lib.call("rogtk_kmer_set_path", 1 if run == 0 else 2)
        try:
            rows, go, G, calls = D.group_spectra(offsets, values, cid, k, mc,
                                                 batch_rows=100_000_000 if run == 0 else 10_000_000)
            torch.cuda.synchronize()
        finally:
            _lib.call("rogtk_kmer_set_path", 1)
        results.append(_props(calls, mc, 16) + (G, len(calls)))
        print(f"C3 100M k=15 run {run}: {results[-1]}", flush=True)
        if run == 0:
            rng = np.random.default_rng(15)
            goh = go.cpu().numpy()
            rows_h = rows.cpu().numpy()
            sizes = np.diff(goh)
            eo = calls[0][2]["entry_offsets"].cpu().numpy()
            nvalid = np.diff(eo)
            assert (nvalid > 0).mean() > 0.75  # the operating point: most groups have valid k-mers (UMI-error
            # singletons and families below 5 reads have none)
            big = np.argsort(sizes, kind="stable")[-300:]
            rich = np.argsort(nvalid, kind="stable")[-300:]
            pick = np.unique(np.concatenate([rng.choice(G, size=2000, replace=False), big, rich]))
            assert len(pick) >= 2000 and nvalid[rich].min() > 200
            ne = _oracle_groups(pick, rows_h, goh, values, n, calls, k, mc)
            print(f"C3 100M k=15: {len(pick)} groups vs oracle, {ne} with valid k-mers; "
                  f"largest group {sizes.max()} rows, most valid {nvalid.max()}", flush=True)
            assert ne >= 1500
        del calls, rows, go
    assert results[0][:4] == results[1][:4]
    nseq, groups, _, G, ncalls = results[0]
    assert nseq == n and groups == G and ncalls == 1 and results[1][4] >= 10
    del values, offsets, cid
    torch.cuda.empty_cache()


@pytest.mark.parametrize("lo,hi,bw", [(0, 150, 8), (100, 420, 16), (300, 990, 32)])
def test_packed_blocks_match_oracle(lo, hi, bw):
    """rogtk_pack_reads + rogtk_kmer_spectrum_blocks on ragged reads (empty rows, nulls, N,
    lowercase, every block size) vs the oracle, for several k and both LDS and radix paths."""
    import torch

    from oracle import pyoracle as P
    from rogtk_amd import _lib
    from rogtk_amd import device as D

    rng = np.random.default_rng(lo + hi)
    groups, items, go = 400, [], [0]
    acgt = np.frombuffer(b"ACGT", np.uint8)
    for g in range(groups):
        tpl = acgt[rng.integers(0, 4, size=hi + 50)]
        for _ in range(int(rng.integers(1, 40 if g % 50 else 600))):
            r = rng.random()
            if r < 0.03:
                items.append(None)
                continue
            L = int(rng.integers(lo, hi + 1))
            a = int(rng.integers(0, 50))
            x = bytearray(tpl[a:a + L].tobytes())
            if r < 0.06 and L:
                x[int(rng.integers(L))] = ord("N")
            elif r < 0.09:
                x = x.lower()
            items.append(bytes(x))
        go.append(len(items))
    n = len(items)
    lens = np.array([0 if x is None else len(x) for x in items], np.int64)
    off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)])).cuda()
    vals = torch.from_numpy(np.frombuffer(b"".join(x for x in items if x is not None) or b"\0", np.uint8).copy()).cuda()
    valid = np.array([x is not None for x in items])
    vbits = torch.from_numpy(np.packbits(np.concatenate([valid, np.zeros(7, bool)]), bitorder="little")).cuda()
    pk = D.PackedReads(off, vals, validity=vbits)
    # the longest row from the pack kernel's own reduction (rows past the guessed 224-base
    # blocks packed again at their size)
    assert pk.block_words == bw and pk.max_len == int(lens.max())
    gsel = torch.tensor(go, dtype=torch.int64).cuda()
    col = P.StrCol.from_list(items)
    fused = hi <= 224  # the fused staging (rogtk_kmer_spectrum_fused) takes rows up to 224 bases
    if not fused:
        with pytest.raises(_lib.RogtkError, match="224"):
            D.kmer_spectrum_fused(off, vals, gsel, 17, 1, 1, -1, validity=vbits)
    for k, mc in ((13, 2), (17, 1), (33, 2)):
        ref = P.kmer_spectrum(col, k, mc, False, np.array(go), threads=THREADS)
        for path, fz in ((1, False), (0, False), (1, True), (0, True)):
            if fz and not fused:
                continue
            _lib.call("rogtk_kmer_set_path", path)
            cap = int(np.clip(lens - 3, 0, None).sum())
            if fz:
                got = D.kmer_spectrum_fused(off, vals, gsel, k, mc, cap, -1, validity=vbits)
            else:
                got = D.kmer_spectrum_blocks(pk, off, vals, gsel, k, mc, cap, validity=vbits)
            torch.cuda.synchronize()
            km = got["kmers"].cpu().numpy().view(np.uint64)
            assert np.array_equal(got["entry_offsets"].cpu().numpy(), ref["group_offsets"]), (k, path)
            assert np.array_equal(got["stats"].cpu().numpy(), ref["stats"]), (k, path)
            assert np.array_equal(km[:, 0], ref["kmer_hi"]) and np.array_equal(km[:, 1], ref["kmer_lo"]), (k, path)
            assert np.array_equal(got["exts"].cpu().numpy(), ref["exts"]), (k, path)
            assert np.array_equal(got["counts"].cpu().numpy().view(np.uint16), ref["counts"]), (k, path)
    _lib.call("rogtk_kmer_set_path", 1)


def test_packed_reads_max_len_too_small_fails_loudly():
    """a PackedReads built with a max_len below the real row lengths used to
    stage truncated rows at a stride the k-mer kernels overran; the spectrum call now
    fails (rows longer than the stride are counted on the device)."""
    import torch

    from rogtk_amd import _lib
    from rogtk_amd import device as D

    rng = np.random.default_rng(5)
    items = [bytes(rng.choice(list(b"ACGT"), size=150).astype(np.uint8)) for _ in range(40)]
    lens = np.array([len(x) for x in items], np.int64)
    off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)])).cuda()
    vals = torch.from_numpy(np.frombuffer(b"".join(items), np.uint8).copy()).cuda()
    go = torch.tensor([0, 20, 40], dtype=torch.int64).cuda()
    ok = D.PackedReads(off, vals)
    D.kmer_spectrum_blocks(ok, off, vals, go, 17, 1, int((lens - 3).sum()))
    short = D.PackedReads(off, vals, max_len=100)  # 150-bp rows packed with a 100-base bound
    with pytest.raises(_lib.RogtkError, match="longer than max_len"):
        D.kmer_spectrum_blocks(short, off, vals, go, 17, 1, int((lens - 3).sum()))


def _py_norep(row: bytes) -> bool:
    """Python restatement of the repeat certificate (kmer_kernels.hip may_repeat16): no
    aligned 16-mer [16j, 16j + 16) of the row occurs again at a later position."""
    L = len(row)
    for a in range(0, L - 15, 16):
        s = row[a:a + 16]
        for i in range(a + 1, L - 15):
            if row[i:i + 16] == s:
                return False
    return True


def _cert_rows(rng, n, lo=20, hi=224):
    """Rows of random ACGT with planted repeats: tandem copies of a 20-60-base unit, a
    16-mer repeated once (certificate withheld, no 32-mer repeat), poly-A tails, N rows."""
    acgt = np.frombuffer(b"ACGT", np.uint8)
    out = []
    for _ in range(n):
        L = int(rng.integers(lo, hi + 1))
        x = bytearray(acgt[rng.integers(0, 4, L)].tobytes())
        r = rng.random()
        if r < 0.15:  # tandem repeat: 32-mers repeat
            u = int(rng.integers(20, 61))
            unit = x[:u]
            x = bytearray((bytes(unit) * (L // u + 1))[:L])
        elif r < 0.30 and L >= 48:  # one 16-mer twice (a 32-mer does not repeat)
            a = 16 * int(rng.integers(0, (L - 16) // 16 + 1))
            i = int(rng.integers(0, L - 15))
            x[i:i + 16] = x[a:a + 16]
        elif r < 0.35:
            x[-min(L, 20):] = b"A" * min(L, 20)
        elif r < 0.38 and L:
            x[int(rng.integers(L))] = ord("N")
        out.append(bytes(x))
    return out


def test_repeat_certificate_bit():
    """Block meta bit 33 (the repeat certificate of rogtk_pack_reads) is sound against the
    Python restatement (set => no aligned 16-mer repeats), and withheld only rarely
    beyond it (the kernel also compares windows that run into the row's end padding)."""
    import torch

    from rogtk_amd import device as D

    rng = np.random.default_rng(33)
    items = _cert_rows(rng, 4000)
    lens = np.array([len(x) for x in items], np.int64)
    off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)])).cuda()
    vals = torch.from_numpy(np.frombuffer(b"".join(items), np.uint8).copy()).cuda()
    pk = D.PackedReads(off, vals)
    assert pk.block_words == 8
    meta = pk.blocks.view(-1, 8)[:, 0].cpu().numpy().view(np.uint64)
    got = ((meta >> np.uint64(33)) & np.uint64(1)).astype(bool)
    clean = np.array([all(c in b"ACGT" for c in x) for x in items])
    want = np.array([c and _py_norep(x) for x, c in zip(items, clean)])
    assert not np.any(got & ~want), np.nonzero(got & ~want)[0][:10]  # sound
    assert np.all(~got[~clean])
    assert (want & ~got).sum() <= 0.02 * want.sum()
    assert want.sum() > 1000  # the random rows are certified


@pytest.mark.parametrize("mc", [2, 3, 8, 20])
def test_repeat_certificate_spectra(mc):
    """Groups around the certificate's bound (rows with observations vs min_coverage),
    with tandem repeats that reach min_coverage inside few rows, k = 17 and 31 (k_eff
    32): spectra and stats identical to the oracle on the block path."""
    import torch

    from oracle import pyoracle as P
    from rogtk_amd import _lib
    from rogtk_amd import device as D

    rng = np.random.default_rng(100 + mc)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    items, go = [], [0]
    for g in range(600):
        nrows = int(rng.integers(1, 2 * mc + 3))
        tpl = bytearray(acgt[rng.integers(0, 4, 224)].tobytes())
        if g % 5 == 0:  # tandem template: its 32-mers repeat inside every row
            u = int(rng.integers(20, 61))
            tpl = bytearray((bytes(tpl[:u]) * 12)[:224])
        for _ in range(nrows):
            L = int(rng.integers(100, 151)) if g % 3 else 150
            x = bytearray(tpl[:L])
            for _ in range(int(rng.integers(0, 3))):
                x[int(rng.integers(L))] = int(acgt[rng.integers(0, 4)])
            items.append(bytes(x))
        go.append(len(items))
    lens = np.array([len(x) for x in items], np.int64)
    off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)])).cuda()
    vals = torch.from_numpy(np.frombuffer(b"".join(items), np.uint8).copy()).cuda()
    pk = D.PackedReads(off, vals)
    gsel = torch.tensor(go, dtype=torch.int64).cuda()
    col = P.StrCol.from_list(items)
    _lib.call("rogtk_kmer_set_path", 1)
    for k, fz in ((17, False), (31, False), (17, True), (31, True)):
        ref = P.kmer_spectrum(col, k, mc, False, np.array(go), threads=THREADS)
        cap = int(np.clip(lens - 3, 0, None).sum())
        # the block path, and the fused staging (certificate computed in k_pack_gather)
        got = (D.kmer_spectrum_fused(off, vals, gsel, k, mc, cap, -1) if fz else
               D.kmer_spectrum_blocks(pk, off, vals, gsel, k, mc, cap))
        torch.cuda.synchronize()
        km = got["kmers"].cpu().numpy().view(np.uint64)
        assert np.array_equal(got["entry_offsets"].cpu().numpy(), ref["group_offsets"]), k
        assert np.array_equal(got["stats"].cpu().numpy(), ref["stats"]), k
        assert np.array_equal(km[:, 0], ref["kmer_hi"]) and np.array_equal(km[:, 1], ref["kmer_lo"]), k
        assert np.array_equal(got["exts"].cpu().numpy(), ref["exts"]), k
        assert np.array_equal(got["counts"].cpu().numpy().view(np.uint16), ref["counts"]), k
        # the tandem groups have valid k-mers below min_coverage rows
        if mc >= 3:
            tandem = [g for g in range(0, 600, 5) if go[g + 1] - go[g] < mc]
            assert sum(int(ref["group_offsets"][g + 1] - ref["group_offsets"][g]) > 0 for g in tandem) > 0


@pytest.mark.parametrize("mc", [2, 5, 20])
def test_minimizer_filter_spectra(mc):
    """The minimizer filter (kmer_kernels.hip k_minimizer_filter, rogtk_kmer_set_filter) on groups with min_coverage
    rows or more, all certified: mixtures of templates each below min_coverage copies
    (nothing valid: the filter empties them), one template at min_coverage copies or more
    read at shifted offsets with errors (valid k-mers: kept), and uncertified tandem /
    poly-A rows (left alone); k = 17 and 31 (k_eff 32). Spectra and stats identical to the
    oracle; the certified-empty count covers the mixtures."""
    import ctypes

    import torch

    from oracle import pyoracle as P
    from rogtk_amd import _lib
    from rogtk_amd import device as D

    rng = np.random.default_rng(300 + mc)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    rand = lambda n: bytearray(acgt[rng.integers(0, 4, n)].tobytes())
    items, go, mixtures, kept = [], [0], [], []

    def read(tpl, L, errs):
        o = int(rng.integers(0, len(tpl) - L + 1))
        x = bytearray(tpl[o:o + L])
        for _ in range(errs):
            x[int(rng.integers(L))] = int(acgt[rng.integers(0, 4)])
        return bytes(x)

    for g in range(400):
        kind = g % 4
        rows = []
        if kind == 0:  # mixture: every template below min_coverage copies, mc rows or more
            per = max(1, mc - 1)
            while len(rows) < mc + int(rng.integers(0, 2 * mc + 2)):
                tpl = rand(180)
                rows += [read(tpl, int(rng.integers(90, 151)), int(rng.integers(0, 2)))
                         for _ in range(int(rng.integers(1, per + 1)))]
            mixtures.append(g)
        elif kind == 1:  # one template at min_coverage copies or more, shifted, with errors
            tpl = rand(200)
            rows = [read(tpl, 150, int(rng.integers(0, 3))) for _ in range(mc + int(rng.integers(0, 6)))]
            rows += [read(rand(160), 150, 0) for _ in range(int(rng.integers(0, 4)))]
            kept.append(g)
        elif kind == 2:  # uncertified rows: a tandem template
            u = int(rng.integers(20, 50))
            tpl = bytearray((bytes(rand(u)) * 10)[:200])
            rows = [read(tpl, 150, 0) for _ in range(mc + int(rng.integers(0, 3)))]
        else:  # a poly-A tail in one row of a mixture
            rows = [read(rand(170), 150, 0) for _ in range(mc + 1)]
            rows[0] = rows[0][:110] + b"A" * 40
        items += rows
        go.append(len(items))
    lens = np.array([len(x) for x in items], np.int64)
    off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)])).cuda()
    vals = torch.from_numpy(np.frombuffer(b"".join(items), np.uint8).copy()).cuda()
    pk = D.PackedReads(off, vals)
    gsel = torch.tensor(go, dtype=torch.int64).cuda()
    col = P.StrCol.from_list(items)
    _lib.call("rogtk_kmer_set_path", 1)
    for k, filt, fz in ((17, 1, False), (31, 1, False), (17, 0, False), (17, 1, True), (31, 1, True)):
        ref = P.kmer_spectrum(col, k, mc, False, np.array(go), threads=THREADS)
        _lib.call("rogtk_kmer_set_filter", filt)
        try:
            cap = int(np.clip(lens - 3, 0, None).sum())
            if fz:  # the fused staging: the certificate computed in k_pack_gather
                got = D.kmer_spectrum_fused(off, vals, gsel, k, mc, cap, -1)
            else:
                got = D.kmer_spectrum_blocks(pk, off, vals, gsel, k, mc, cap)
            torch.cuda.synchronize()
        finally:
            _lib.call("rogtk_kmer_set_filter", 1)
        cg = ctypes.c_int64(0)
        _lib.call("rogtk_kmer_certified_groups", ctypes.byref(cg))
        km = got["kmers"].cpu().numpy().view(np.uint64)
        assert np.array_equal(got["entry_offsets"].cpu().numpy(), ref["group_offsets"]), k
        assert np.array_equal(got["stats"].cpu().numpy(), ref["stats"]), k
        assert np.array_equal(km[:, 0], ref["kmer_hi"]) and np.array_equal(km[:, 1], ref["kmer_lo"]), k
        assert np.array_equal(got["exts"].cpu().numpy(), ref["exts"]), k
        assert np.array_equal(got["counts"].cpu().numpy().view(np.uint16), ref["counts"]), k
        eo = ref["group_offsets"]
        assert all(eo[g + 1] == eo[g] for g in mixtures)  # nothing valid in a mixture
        assert sum(eo[g + 1] > eo[g] for g in kept) > len(kept) // 2  # the kept groups do have output
        if filt:
            assert cg.value >= len(mixtures), (cg.value, len(mixtures))  # the filter emptied them
        else:
            assert cg.value < len(mixtures) // 2, cg.value  # (the row certificate alone cannot)
