"""GPU parity: librogtk_hip (through the C ABI) vs the CPU oracle, bit-exact.

f64 fields are compared as raw 64-bit patterns (including the x86 default NaN the
reference produces for an empty UMI); integers/booleans/cluster ids exactly.
Sizes the oracle finishes in seconds are compared row by row; BASELINE's full
10M-read configuration is checked through size-independent properties plus a
distinct-UMI oracle check (H1 of a regular row depends only on its code).
"""
from __future__ import annotations

import os

import numpy as np
import pyarrow as pa
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rg():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import rogtk_amd

    assert rogtk_amd.device_count() >= 1
    return rogtk_amd


def P():
    from oracle import pyoracle

    return pyoracle


def _col_from_npz(z):
    offs, vals, valid = z["offsets"], z["values"], z["valid"]
    n = len(valid)
    vbuf = None if valid.all() else pa.py_buffer(np.packbits(valid, bitorder="little"))
    return pa.Array.from_buffers(pa.large_binary(), n, [vbuf, pa.py_buffer(offs), pa.py_buffer(vals)])


def _np(a):
    """Arrow array -> numpy with nulls filled (callers compare valid rows only)."""
    if isinstance(a, (pa.Array, pa.ChunkedArray)):
        fill = False if pa.types.is_boolean(a.type) else 0
        return np.asarray(a.fill_null(fill).to_numpy(zero_copy_only=False))
    return np.asarray(a)


def _assert_scores_equal(got, ref: dict, valid):
    for name in P().FIELDS:
        r = np.asarray(ref[name])
        g = _np(got.field(name)) if hasattr(got, "field") else np.asarray(got[name])
        if r.dtype == np.float64:
            gb = g.astype(np.float64).view(np.uint64)[valid]
            rb = r.view(np.uint64)[valid]
        else:
            gb, rb = g[valid].astype(np.uint64), r[valid].astype(np.uint64)
        bad = np.nonzero(gb != rb)[0]
        assert bad.size == 0, f"{name}: {bad.size} rows differ, first at {bad[:5]}"


@pytest.mark.parametrize("fixture", ["c1_clean", "c1_stress"])
def test_golden_complexity(rg, fixture):
    z = np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False)
    col = _col_from_npz(z)
    got = rg.umi_complexity_scores(col)
    valid = z["valid"]
    assert got.null_count == 0  # df.into_struct: rows valid, fields null (expressions.rs:1258-1283)
    for f in P().FIELDS:
        assert got.field(f).null_count == (~valid).sum()
    ref = {f: (z["f_" + f].view(np.float64) if z["f_" + f].dtype == np.uint64 else z["f_" + f])
           for f in P().FIELDS}
    _assert_scores_equal(got, ref, valid)


@pytest.mark.parametrize("fixture", ["c1_clean", "c1_stress"])
def test_golden_single_fields(rg, fixture):
    """The seven single-field exprs (expressions.rs:1286-1410) equal the struct fields."""
    z = np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False)
    col = _col_from_npz(z)
    c = rg.col(col)
    valid = z["valid"]
    for name in P().FIELDS:
        meth = {"longest_homopolymer_run": "longest_homopolymer_run"}.get(name, name)
        arr = getattr(c.umi, meth)()
        assert arr.null_count == (~valid).sum()
        r = z["f_" + name]
        g = _np(arr)
        if r.dtype == np.uint64:
            assert np.array_equal(g.astype(np.float64).view(np.uint64)[valid], r[valid]), name
        else:
            assert np.array_equal(g[valid].astype(np.uint32), r[valid]), name


@pytest.mark.parametrize("fixture", ["c1_clean", "c1_stress"])
def test_golden_hamming(rg, fixture):
    z = np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False)
    col = _col_from_npz(z)
    valid = z["valid"]
    k = 0
    while f"ham_target_{k}" in z:
        t = z[f"ham_target_{k}"].tobytes()
        d = _np(rg.hamming_distance(col, t))
        w = _np(rg.hamming_within(col, t, 1))
        assert np.array_equal(d[valid].astype(np.uint32), z[f"ham_dist_{k}"][valid]), t
        assert np.array_equal(w[valid].astype(bool), z[f"ham_within_{k}"][valid]), t
        k += 1
    assert k >= 5


@pytest.mark.parametrize("fixture", ["c1_clean", "c1_stress"])
@pytest.mark.parametrize("md", [0, 1])
def test_golden_cluster(rg, fixture, md):
    z = np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False)
    col = _col_from_npz(z)
    got, k, L = rg.umi_cluster(col, 12, md)
    assert L == 12
    assert k == int(z[f"n_clusters_{md}"][0])
    v = z[f"cluster_valid_{md}"]
    assert got.null_count == (~v).sum()
    g = _np(got)
    assert np.array_equal(g[v].astype(np.uint32), z[f"cluster_{md}"][v])


def _random_strings(rng, n, lengths, alphabet=b"ACGT"):
    out = []
    for _ in range(n):
        L = int(rng.choice(lengths))
        out.append(rng.choice(list(alphabet), size=L).astype(np.uint8).tobytes())
    return out


@pytest.mark.parametrize("L", list(range(1, 17)))
def test_packed_every_length(rg, L):
    """Packed path for every supported UMI length (all rows regular)."""
    rng = np.random.default_rng(L)
    umis = _random_strings(rng, 3000, [L])
    umis += [b"A" * L, b"C" * L, (b"ACGT" * 5)[:L], (b"AAAT" * 5)[:L]]
    ref = P().umi_complexity(P().StrCol.from_list(umis))
    got = rg.umi_complexity_scores(pa.array(umis, type=pa.large_binary()))
    _assert_scores_equal(got, ref, ref["valid"])


def test_byte_path_edge_cases(rg):
    rng = np.random.default_rng(3)
    umis = [b"", b"A", b"N", b"NN", b"NNN", b"acgt", "é".encode(), "éé".encode(), b"\x00\x00\x00",
            b"ACGT\x00ACGT", b"A" * 64, b"A" * 65, b"AC" * 40, b"ACGTTTTTTTTGCA" * 10]
    umis += _random_strings(rng, 400, list(range(0, 40)), alphabet=b"ACGTNacgtX")
    umis += _random_strings(rng, 60, [64, 70, 100, 150, 200], alphabet=b"ACGTN")
    umis += _random_strings(rng, 20, [300, 500], alphabet=b"AC")
    ref = P().umi_complexity(P().StrCol.from_list(umis))
    got = rg.umi_complexity_scores(pa.array(umis, type=pa.large_binary()))
    _assert_scores_equal(got, ref, ref["valid"])


def test_nulls_and_chunks(rg):
    umis = ["ACGTACGTACGT", None, "AAAAAAAAAAAA", None, "ACGTNACGTACG", ""]
    ch = pa.chunked_array([pa.array(umis[:3]), pa.array(umis[3:])])
    got = rg.umi_complexity_scores(ch)
    assert got.null_count == 0 and sum(c.field(0).null_count for c in got.chunks) == 2
    ref = P().umi_complexity(P().StrCol.from_list(umis))
    flat = pa.concat_arrays(got.chunks)
    _assert_scores_equal(flat, ref, ref["valid"])
    # sliced array (non-zero Arrow offset on values + validity)
    arr = pa.array(umis * 50)[7:251]
    got2 = rg.umi_complexity_scores(arr)
    ref2 = P().umi_complexity(P().StrCol.from_list(arr.to_pylist()))
    _assert_scores_equal(got2, ref2, ref2["valid"])


@pytest.mark.parametrize("target", [b"ACGTACGTACGT", b"ACGTACGTACG", b"NNNNNNNNNNNN", b"acgtacgtacgt",
                                    "ACGTACGTACé".encode(), b"", b"A"])
@pytest.mark.parametrize("maxd", [0, 1, 3])
def test_hamming_targets(rg, target, maxd):
    rng = np.random.default_rng(5)
    umis = _random_strings(rng, 2000, [11, 12, 13], alphabet=b"ACGT")
    umis += _random_strings(rng, 200, [12], alphabet=b"ACGTNa")
    umis += ["ACGTACGTACé".encode(), "ééééééACGTAC".encode(), b"", b"A", None]
    col = P().StrCol.from_list(umis)
    rd, rw, valid = P().hamming(col, target, maxd)
    arr = pa.array(umis, type=pa.large_binary())
    gd = _np(rg.hamming_distance(arr, target))
    gw = _np(rg.hamming_within(arr, target, maxd))
    assert np.array_equal(gd[valid].astype(np.uint32), rd[valid])
    assert np.array_equal(gw[valid].astype(bool), rw[valid])


@pytest.mark.parametrize("L", [1, 2, 3, 5, 8, 12, 13, 14, 16, 17, 20, 24, 31, 32])
@pytest.mark.parametrize("md", [0, 1])
def test_cluster_lengths(rg, L, md):
    """Dense-table sizes from 4 codes up to 4^16 (label-by-code for L<=13, by index above);
    17..32: the sort-based long-UMI engine (long_cluster.hip)."""
    rng = np.random.default_rng(100 + L)
    n = 20000
    if L <= 6:
        umis = _random_strings(rng, n, [L])
    else:
        parents = _random_strings(rng, n // 10, [L])
        umis = []
        for _ in range(n):
            p = bytearray(parents[int(rng.integers(len(parents)))])
            if rng.random() < 0.3:
                j = int(rng.integers(L))
                p[j] = b"ACGT"[int(rng.integers(4))]
            umis.append(bytes(p))
    umis += [None, b"N" * L, b"acgt"[: min(L, 4)], b"ACGT" * 5]
    col = P().StrCol.from_list(umis)
    rc, rv, rk, _ = P().umi_cluster(col, L, md)
    got, k, rl = rg.umi_cluster(pa.array(umis, type=pa.large_binary()), L, md)
    assert rl == L and k == rk
    g = _np(got)
    assert np.array_equal(g[rv].astype(np.uint32), rc[rv])


@pytest.mark.parametrize("L,n,want_p0,want_lcap", [(9, 20_000, 8, 0), (9, 120_000, 8, 1), (9, 300_000, 7, 1),
                                                    (8, 6_000, 8, 0), (8, 30_000, 8, 1), (8, 60_000, 7, 1),
                                                    (10, 150_000, 8, 0), (10, 600_000, 7, 1), (12, 200_000, 8, 0)])
def test_local_tiling_both_paths(rg, L, n, want_p0, want_lcap):
    """The local phase covers positions 0..7 (4^8-code tiles) when every tile holds at most
    16384 distinct codes (the 8192-code instance, S_LCAP 0, or the 16384-code one, S_LCAP 1)
    and 0..6 otherwise (decided on the device, stats[S_P0]): random codes of a few densities
    take each path (the wanted values follow from the densest tile, checked below), and the
    ids equal the oracle."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    rng = np.random.default_rng(L * 1000 + n)
    parents = rng.integers(0, 4 ** L, size=max(n // 4, 1), dtype=np.uint64)
    codes_h = parents[rng.integers(0, len(parents), size=n)]
    flip = rng.random(n) < 0.3
    pos = rng.integers(0, L, size=n).astype(np.uint64)
    codes_h = np.where(flip, codes_h ^ (rng.integers(1, 4, size=n).astype(np.uint64) << (2 * pos)), codes_h)
    codes_h = codes_h.astype(np.uint32)
    densest = int(np.bincount(np.unique(codes_h) >> 16).max())
    assert (8 if densest <= 16384 else 7) == want_p0 and (1 if densest > 8192 else 0) == want_lcap
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    eng = D.ClusterEngine(L, min(n, 4 ** L), "cuda")
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    D.cluster_batch(eng, batch, cid, 1)
    torch.cuda.synchronize()
    st = eng.ws[:64].view(torch.int64)
    assert int(st[6].item()) == want_p0
    if want_p0 == 8:
        assert int(st[7].item()) == want_lcap
    rc, _, rk, _ = P().umi_cluster(P().StrCol.from_fixed(synth.codes_to_ascii(codes_h, L)), L, 1)
    assert eng.stats()["n_clusters"] == rk
    assert np.array_equal(cid.cpu().numpy().view(np.uint32), rc)


@pytest.mark.parametrize("L", [18, 32])
def test_long_cluster_bruteforce_and_chains(rg, L):
    """Long UMIs vs the O(d^2) brute force, with Hamming-1 chains that cross every
    position (many union rounds) and irregular / null rows mixed in."""
    rng = np.random.default_rng(L)
    umis = []
    for c in range(30):  # chains: each step changes one random position
        u = bytearray(_random_strings(rng, 1, [L])[0])
        for _ in range(int(rng.integers(2, 40))):
            j = int(rng.integers(L))
            u[j] = b"ACGT"[(b"ACGT".index(u[j]) + int(rng.integers(1, 4))) % 4]
            umis.append(bytes(u))
    umis += _random_strings(rng, 800, [L])
    umis += [None, b"N" * L, b"ACGT", b"acgt" * (L // 4), b"A" * (L + 1)]
    order = rng.permutation(len(umis))
    umis = [umis[i] for i in order]
    ref, rk = P().py_cluster_bruteforce(umis, L, 1)
    got, k, _ = rg.umi_cluster(pa.array(umis, type=pa.large_binary()), L, 1)
    assert k == rk
    assert got.to_pylist() == ref


def test_long_cluster_position_batches(rg, monkeypatch):
    """The long engine finds its edges in batches of positions when nd * L passes the
    record budget (ROGTK_LONG_REC_BATCH lowered): ids equal the one-batch run."""
    rng = np.random.default_rng(5)
    L = 24
    umis = []
    for _ in range(3000):
        u = bytearray(_random_strings(rng, 1, [L])[0])
        for _ in range(int(rng.integers(1, 6))):
            j = int(rng.integers(L))
            u[j] = b"ACGT"[int(rng.integers(4))]
            umis.append(bytes(u))
    col = pa.array(umis, type=pa.large_binary())
    ref, rk = rg.umi_cluster(col, L, 1)[:2]
    for batch in ("1", "5000", "40000"):
        monkeypatch.setenv("ROGTK_LONG_REC_BATCH", batch)
        got, k, _ = rg.umi_cluster(col, L, 1)
        assert k == rk and got.to_pylist() == ref.to_pylist(), batch
    rc, _, ok, _ = P().umi_cluster(P().StrCol.from_list(umis), L, 1)
    assert ok == rk and np.array_equal(_np(ref).astype(np.uint32), rc)


def test_cluster_dev_matches_host_long_and_short(rg):
    """rogtk_umi_cluster_dev (device column) == rogtk_umi_cluster_host, both engines."""
    import ctypes
    import torch
    from rogtk_amd import _lib
    rng = np.random.default_rng(77)
    for L in (12, 20):
        umis = _random_strings(rng, 5000, [L]) + [b"N" * L, b"ACG", b""]
        host, k, _ = rg.umi_cluster(pa.array(umis, type=pa.large_binary()), L, 1)
        off = torch.tensor(np.concatenate([[0], np.cumsum([len(u) for u in umis])]), dtype=torch.int64).cuda()
        val = torch.tensor(np.frombuffer(b"".join(umis), np.uint8).copy()).cuda()
        cid = torch.empty(len(umis), dtype=torch.int32, device="cuda")
        nk = ctypes.c_int64(0)
        _lib.call("rogtk_umi_cluster_dev", ctypes.c_void_p(off.data_ptr()), ctypes.c_void_p(val.data_ptr()), None,
                  len(umis), L, 1, ctypes.c_void_p(cid.data_ptr()), ctypes.byref(nk),
                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert nk.value == k
        assert np.array_equal(cid.cpu().numpy().view(np.uint32), _np(host).astype(np.uint32))


@pytest.mark.parametrize("L,utf8", [(4, 0), (6, 0), (8, 0), (12, 0), (13, 0), (16, 0), (20, 0), (32, 0), (33, 0),
                                    (6, 0.1), (12, 0.1), (24, 0.1)])
def test_cluster_irregular_families(rg, L, utf8):
    """SURVEY §8a H3.2 for every engine: strings with N, lowercase bytes and other lengths
    get Hamming-1 edges to each other and to regular codes (and bridge regular clusters);
    host and device-column paths vs the oracle and the O(d^2) brute force. utf8 > 0 adds
    multi-byte UTF-8 members: H3 compares bytes, so the appended pin pair
    A^(L-2)+U+00E9 / A^L (H2.1 distance 1: chars zipped) stays in two clusters."""
    import ctypes
    import torch
    from conftest import irregular_families
    from rogtk_amd import _lib

    umis = irregular_families(L + int(utf8 * 1000), 400 if L <= 8 else 700, L, p_utf8=utf8)
    if utf8:
        assert any(0xC3 in u for u in umis if u)
        pin = pa.array(umis[-2:], type=pa.large_binary())
        assert _np(rg.hamming_distance(pin, b"A" * L)).tolist() == [1, 0]  # H2.1: chars zipped
    col = P().StrCol.from_list(umis)
    for md in (0, 1):
        rc, rv, rk, _ = P().umi_cluster(col, L, md)
        ref, bk = P().py_cluster_bruteforce(umis, L, md)
        assert rk == bk
        got, k, rl = rg.umi_cluster(pa.array(umis, type=pa.large_binary()), L, md)
        assert rl == L and k == rk, (md, k, rk)
        assert got.to_pylist() == ref
        # device column (rogtk_umi_cluster_dev, nulls as empty strings -> compare valid rows)
        dense = [u if u is not None else b"" for u in umis]
        off = torch.tensor(np.concatenate([[0], np.cumsum([len(u) for u in dense])]), dtype=torch.int64).cuda()
        val = torch.tensor(np.frombuffer(b"".join(dense) or b"\0", np.uint8).copy()).cuda()
        vbits = torch.from_numpy(np.packbits(np.array([u is not None for u in umis] + [False] * 7),
                                             bitorder="little")).cuda()
        cid = torch.empty(len(umis), dtype=torch.int32, device="cuda")
        nk = ctypes.c_int64(0)
        _lib.call("rogtk_umi_cluster_dev", ctypes.c_void_p(off.data_ptr()), ctypes.c_void_p(val.data_ptr()),
                  ctypes.c_void_p(vbits.data_ptr()), len(umis), L, md, ctypes.c_void_p(cid.data_ptr()),
                  ctypes.byref(nk), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert nk.value == rk
        assert np.array_equal(cid.cpu().numpy().view(np.uint32)[rv], rc[rv])
        if utf8 and md == 1:
            assert ref[-2] != ref[-1]  # byte-wise: 2 mismatches, no edge


@pytest.mark.parametrize("L", [12, 24])
def test_cluster_n_stress_large(rg, L):
    """200k synth reads with N at 1e-3/base and lowercase at 5e-4/base (SURVEY §8d's
    N-stress variant): ids equal the oracle."""
    from rogtk_amd import synth

    umis = [bytes(r) for r in synth.umi_ascii(200_000, L, p_n=1e-3, p_lower=5e-4)]
    col = P().StrCol.from_list(umis)
    rc, rv, rk, _ = P().umi_cluster(col, L, 1)
    got, k, _ = rg.umi_cluster(pa.array(umis, type=pa.large_binary()), L, 1)
    assert k == rk
    assert np.array_equal(_np(got).astype(np.uint32), rc)
    n_irr = sum(1 for u in umis if any(c not in b"ACGT" for c in u))
    assert n_irr > 1000


def test_cluster_bruteforce_small(rg):
    """H3 spec vs the O(d^2) brute force on the H2 distance (independent of the oracle)."""
    rng = np.random.default_rng(9)
    umis = _random_strings(rng, 3000, [6])
    umis += [None, b"NNNNNN", b"ACGTN", b"acgtac"]
    ref, rk = P().py_cluster_bruteforce(umis, 6, 1)
    got, k, _ = rg.umi_cluster(pa.array(umis, type=pa.large_binary()), 6, 1)
    assert k == rk
    assert got.to_pylist() == ref


# ----------------------------------------------------------------------------
# Device-level pipeline (the bench path) and size-independent properties
# ----------------------------------------------------------------------------
def _device_run(n, L=12, md=1, target=b"ACGTACGTACGT", seed=None, shards=1):
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    seed = synth.DEFAULT_SEED if seed is None else seed
    codes_h = synth.umi_codes(n, L, seed=seed)
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    scores = D.alloc_scores(n, codes.device)
    hd = torch.empty(n, dtype=torch.int32, device="cuda")
    hw = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    if shards == 1:
        eng = D.ClusterEngine(L, min(n, 4 ** L), "cuda")
        D.score_packed(batch, scores, target, 1, hd, hw)
        D.cluster_batch(eng, batch, cid, md)
        stats = eng.stats()
    else:
        # emulate `shards` ranks on one GPU: local bitmaps -> concatenation (= all-gather) -> resolve
        bounds = np.linspace(0, n, shards + 1).astype(np.int64)
        bounds = (bounds // 4) * 4
        bounds[-1] = n
        engs, bats = [], []
        for r in range(shards):
            a, b = int(bounds[r]), int(bounds[r + 1])
            e = D.ClusterEngine(L, min(n, 4 ** L), "cuda")
            bt = D.PackedBatch(codes[a:b], L)
            e.mark(bt)
            engs.append(e)
            bats.append((a, b, bt))
        gathered = torch.cat([e.build_local_bitmap().clone() for e in engs])
        D.score_packed(batch, scores, target, 1, hd, hw)
        for e, (a, b, bt) in zip(engs, bats):
            e.resolve(gathered, shards, md)
            e.assign(bt, cid[a:b])
        stats = engs[0].stats()
    torch.cuda.synchronize()
    return codes_h, scores, hd, hw, cid, stats


def test_device_pipeline_vs_oracle(rg):
    """1M reads through the fused device path, every output row vs the oracle."""
    from rogtk_amd import synth

    n = 1_000_000
    codes_h, scores, hd, hw, cid, stats = _device_run(n)
    umis = synth.codes_to_ascii(codes_h, 12)
    col = P().StrCol.from_fixed(umis)
    ref = P().umi_complexity(col)
    got = {f: scores[f][:n].cpu().numpy() for f in P().FIELDS}
    got["longest_homopolymer_run"] = got["longest_homopolymer_run"].view(np.uint32)
    _assert_scores_equal(got, ref, np.ones(n, bool))
    rd, rw, _ = P().hamming(col, b"ACGTACGTACGT", 1)
    assert np.array_equal(hd.cpu().numpy().view(np.uint32), rd)
    bits = np.unpackbits(hw.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(bits, rw)
    rc, _, rk, _ = P().umi_cluster(col, 12, 1)
    assert stats["n_clusters"] == rk and stats["overflow"] == 0
    assert np.array_equal(cid.cpu().numpy().view(np.uint32), rc)


@pytest.mark.parametrize("polls", [0, 1, 3])
@pytest.mark.parametrize("md", [0, 1])
def test_lookback_fallback_exact(rg, polls, md):
    """The single-pass scan's bounded look-back (k_scan_rt): a block whose wait gives up
    recounts its prefix from the bitmaps, so ids stay exact (a give-up used to
    leave a partial prefix behind an unread error flag). polls=0 forces the recount in
    every block, 1 / 3 mix it with published prefixes."""
    from rogtk_amd import device as D
    from rogtk_amd import synth

    n = 2_000_000
    try:
        D.set_lookback_polls(polls)
        codes_h, _, _, _, cid, stats = _device_run(n, md=md)
    finally:
        D.set_lookback_polls(-1)
    col = P().StrCol.from_fixed(synth.codes_to_ascii(codes_h, 12))
    rc, _, rk, _ = P().umi_cluster(col, 12, md)
    assert stats["n_clusters"] == rk and stats["overflow"] == 0 and stats["error"] == 0
    assert np.array_equal(cid.cpu().numpy().view(np.uint32), rc)


@pytest.mark.parametrize("L,fields,ham,deferred,spec", [(12, "all", "within", False, 0), (12, "all", "within", True, 1),
                                                        (12, None, "both", True, 0), (10, "all", "both", False, 0),
                                                        (9, "comb", None, True, 1)])
def test_score_assign_fused_vs_oracle(rg, L, fields, ham, deferred, spec):
    """rogtk_umi_score_assign_packed (score + H3 ids in one pass over the codes; the L=12
    instance and the generic one, deferred with 1 speculative round = the re-run path)
    equals the oracle row by row."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    n = 700_001
    codes_h = synth.umi_codes(n, L, seed=synth.DEFAULT_SEED + L)
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    scores = None
    if fields == "all":
        scores = D.alloc_scores(n, codes.device)
    elif fields == "comb":
        scores = {"combined_score": torch.empty(n, dtype=torch.float64, device="cuda")}
    hd = torch.empty(n, dtype=torch.int32, device="cuda") if ham == "both" else None
    hw = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda") if ham else None
    target = b"ACGTACGTACGTACGT"[:L] if ham else None
    cid = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    eng = D.ClusterEngine(L, min(n, 4 ** L), "cuda")
    try:
        D.set_spec_rounds(spec)
        eng.mark_bitmap(batch)
        eng.resolve(eng.local_bitmap, 1, 1)
        D.score_assign_packed(batch, eng, cid, scores, target, 1, hd, hw, deferred=deferred)
        eng.sync()
        torch.cuda.synchronize()
    finally:
        D.set_spec_rounds(0)
    col = P().StrCol.from_fixed(synth.codes_to_ascii(codes_h, L))
    rc, _, _, _ = P().umi_cluster(col, L, 1)
    assert np.array_equal(cid.cpu().numpy().view(np.uint32), rc)
    if scores is not None:
        ref = P().umi_complexity(col)
        for f, t in scores.items():
            g = t.cpu().numpy()
            r = ref[f]
            if r.dtype == np.float64:
                assert np.array_equal(g.view(np.uint64), r.view(np.uint64)), f
            else:
                assert np.array_equal(g.view(np.uint32), r), f
    if ham:
        rd, rw, _ = P().hamming(col, target, 1)
        if hd is not None:
            assert np.array_equal(hd.cpu().numpy().view(np.uint32), rd)
        bits = np.unpackbits(hw.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
        assert np.array_equal(bits, rw)


@pytest.mark.parametrize("n_codes,expect_p0", [(3_400_000, 8), (5_500_000, 7), (900_000, 8)])
def test_dense_space_local_tilings_vs_oracle(rg, n_codes, expect_p0):
    """Uniform random 12-bp codes at 19% / 28% / 5% density: the 8-position local CC for
    tiles of 8193..16384 codes (the union bitmap of 2-4 ranks), the 7-position one above
    that, the 8192-code instance below; ids equal the oracle's union-find."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    rng = np.random.default_rng(n_codes)
    codes_h = rng.integers(0, 4 ** 12, n_codes, dtype=np.uint32)
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    batch = D.PackedBatch(codes, 12)
    cid = torch.empty(n_codes, dtype=torch.int32, device="cuda")
    eng = D.ClusterEngine(12, n_codes, "cuda")
    eng.mark_bitmap(batch)
    eng.resolve(eng.local_bitmap, 1, 1)
    eng.assign(batch, cid)
    stats = eng.stats()
    torch.cuda.synchronize()
    rc, _, rk, _ = P().umi_cluster(P().StrCol.from_fixed(synth.codes_to_ascii(codes_h, 12)), 12, 1)
    assert stats["n_clusters"] == rk
    assert np.array_equal(cid.cpu().numpy().view(np.uint32), rc)
    # which tiling ran: the workspace's stats block (slot 6 = first global position)
    p0 = int(eng.ws[48:56].cpu().numpy().view(np.int64)[0])
    assert p0 == expect_p0


@pytest.mark.parametrize("poison", [False, True])
@pytest.mark.parametrize("deferred", [False, True])
def test_local_cc_prediction_redo(rg, deferred, poison):
    """One workspace, batches whose tilings change: sparse (8 positions, <= 8192 codes per
    tile), 19% dense (8 positions, <= 16384), 28% dense (7 positions), sparse again. Each
    resolve launches only the local-CC instance of the workspace's previous resolve; a
    mismatch flags S_REDO and cluster_finish redoes the local and global phases (and the
    deferred assign). Ids equal the oracle's every time. poison: the workspace is filled
    with 0xFF bytes before every batch after the first, so the speculative kernels that
    run behind a mismatched instance would read out-of-range parents if they did not stop
    at S_REDO."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    sizes = [900_000, 3_400_000, 5_500_000, 900_000, 900_000]
    eng = D.ClusterEngine(12, max(sizes), "cuda")
    for i, n_codes in enumerate(sizes):
        codes_h, rc, rk = _redo_batch(i, n_codes)
        codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
        batch = D.PackedBatch(codes, 12)
        cid = torch.empty(n_codes, dtype=torch.int32, device="cuda")
        if poison and i:
            eng.ws.fill_(0xFF)
        eng.mark_bitmap(batch)
        eng.resolve(eng.local_bitmap, 1, 1)
        eng.assign(batch, cid, deferred=deferred)
        eng.sync()
        stats = eng.stats()
        torch.cuda.synchronize()
        assert stats["n_clusters"] == rk and stats["error"] == 0, i
        assert np.array_equal(cid.cpu().numpy().view(np.uint32), rc), i


_REDO_CACHE = {}


def _redo_batch(i, n_codes):
    """Batch i of the redo test and its oracle ids (the same for every parametrisation)."""
    if i not in _REDO_CACHE:
        from rogtk_amd import synth

        codes_h = np.random.default_rng(1000 + i).integers(0, 4 ** 12, n_codes, dtype=np.uint32)
        rc, _, rk, _ = P().umi_cluster(P().StrCol.from_fixed(synth.codes_to_ascii(codes_h, 12)), 12, 1,
                                       threads=min(16, os.cpu_count() or 1))
        _REDO_CACHE[i] = (codes_h, rc, rk)
    return _REDO_CACHE[i]


@pytest.mark.parametrize("shards", [2, 4, 8])
def test_sharded_resolve_matches_single(rg, shards):
    """N-rank exchange emulated on one GPU: ids identical to the single-batch run."""
    n = 400_003
    _, _, _, _, cid1, s1 = _device_run(n, shards=1)
    _, _, _, _, cidn, sn = _device_run(n, shards=shards)
    assert s1["n_clusters"] == sn["n_clusters"]
    assert np.array_equal(cid1.cpu().numpy(), cidn.cpu().numpy())


def test_full_size_c2_properties(rg):
    """BASELINE C2 (10M reads, L=12, Hamming<=1): full-size parity without a 10M-row H1 oracle run.

    H1/H2 of a regular row are functions of its code, so the oracle runs on the
    distinct codes and is broadcast back; H3 ids are checked against the oracle's
    union-find on the full 10M codes; the run is repeated for determinism.
    """
    from rogtk_amd import synth

    n = 10_000_000
    codes_h, scores, hd, hw, cid, stats = _device_run(n)
    uniq, inv = np.unique(codes_h, return_inverse=True)
    ucol = P().StrCol.from_fixed(synth.codes_to_ascii(uniq, 12))
    ref = P().umi_complexity(ucol)
    for f in P().FIELDS:
        g = scores[f][:n].cpu().numpy()
        r = ref[f][inv]
        if r.dtype == np.float64:
            assert np.array_equal(g.view(np.uint64), r.view(np.uint64)), f
        else:
            assert np.array_equal(g.view(np.uint32), r), f
    rd, _, _ = P().hamming(ucol, b"ACGTACGTACGT", 1)
    assert np.array_equal(hd.cpu().numpy().view(np.uint32), rd[inv])
    # H3: oracle on the full column of codes
    rc, _, rk, _ = P().umi_cluster(P().StrCol.from_fixed(synth.codes_to_ascii(codes_h, 12)), 12, 1)
    assert stats["n_distinct"] == len(uniq)
    assert stats["n_clusters"] == rk
    g = cid.cpu().numpy().view(np.uint32)
    assert np.array_equal(g, rc)
    # determinism: a second run is bitwise identical
    _, scores2, _, _, cid2, _ = _device_run(n)
    assert np.array_equal(cid2.cpu().numpy(), cid.cpu().numpy())
    assert np.array_equal(scores2["combined_score"][:n].cpu().numpy().view(np.uint64),
                          scores["combined_score"][:n].cpu().numpy().view(np.uint64))


def test_full_size_c2_bench_pipeline_all_outputs(rg):
    """BASELINE C2 through the bench's own path: 10M reads, UmiPipeline with bench.py's
    arguments (depth 2, slice-bucket mark, assign on the main stream, deferred assigns,
    device events), three submits of the batch as the bench's steps do; every output of
    both slots is compared: the 7 H1 fields, the H2 distance and within columns (distinct
    codes broadcast back) and the H3 ids (oracle union-find on the 10M codes)."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth
    from rogtk_amd.pipeline import UmiPipeline

    n, L = 10_000_000, 12
    codes_h = synth.umi_codes(n, L)
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    pipe = UmiPipeline(L, min(n, 4 ** L), n, "cuda", depth=2, target=b"ACGTACGTACGT", max_distance=1,
                       score_alone=True, with_distance=True)
    for _ in range(3):
        pipe.submit(batch)
    pipe.drain()
    torch.cuda.synchronize()
    uniq, inv = np.unique(codes_h, return_inverse=True)
    ucol = P().StrCol.from_fixed(synth.codes_to_ascii(uniq, L))
    ref = P().umi_complexity(ucol)
    rd, rw, _ = P().hamming(ucol, b"ACGTACGTACGT", 1)
    rc, _, rk, _ = P().umi_cluster(P().StrCol.from_fixed(synth.codes_to_ascii(codes_h, L)), L, 1)
    for slot in pipe.slots:
        for f in P().FIELDS:
            g = slot.scores[f][:n].cpu().numpy()
            r = ref[f][inv]
            if r.dtype == np.float64:
                assert np.array_equal(g.view(np.uint64), r.view(np.uint64)), f
            else:
                assert np.array_equal(g.view(np.uint32), r), f
        assert np.array_equal(slot.dist[:n].cpu().numpy().view(np.uint32), rd[inv])
        bits = np.unpackbits(slot.within.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
        assert np.array_equal(bits, rw[inv])
        st = slot.eng.stats()
        assert st["n_distinct"] == len(uniq) and st["n_clusters"] == rk
        assert np.array_equal(slot.cid[:n].cpu().numpy().view(np.uint32), rc)


@pytest.mark.parametrize("depth,nb,alone", [(4, 4, False), (2, 5, False), (1, 3, False), (3, 5, True)])
@pytest.mark.parametrize("mark", ["xcd", "sort"])
@pytest.mark.parametrize("assign_on", ["resolve", "separate", "main", "main_mark_stream", "main_fused"])
def test_streaming_pipeline_matches_sequential(rg, depth, nb, alone, mark, assign_on):
    """rogtk_amd.pipeline (3 streams, `depth` batches in flight) == the sequential device
    path for EVERY batch (outputs copied out by the on_assigned hook before slot reuse)."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth
    from rogtk_amd.pipeline import UmiPipeline

    n, L = 300_001, 12
    seeds = [synth.DEFAULT_SEED + 17 * k for k in range(nb)]
    outs = []
    mark_stream = assign_on == "main_mark_stream"
    fused = assign_on == "main_fused"
    if mark_stream or fused:
        if fused and depth < 2:
            pytest.skip("the fused score + assign needs depth >= 2")
        assign_on = "main"

    def grab(slot, batch):
        outs.append((slot.cid[:n].clone(), slot.within.clone(), slot.scores["combined_score"][:n].clone(),
                     slot.scores["longest_homopolymer_run"][:n].clone()))

    pipe = UmiPipeline(L, n, n, "cuda", depth=depth, target=b"ACGTACGTACGT", max_distance=1, mark=mark,
                       on_assigned=grab, score_alone=alone, assign_on=assign_on, mark_stream=mark_stream,
                       fused_assign=fused)
    keep = []
    for s in seeds:
        codes = torch.from_numpy(synth.umi_codes(n, L, seed=s).view(np.int32)).cuda()
        keep.append(D.PackedBatch(codes, L))
        pipe.submit(keep[-1])
    pipe.drain()
    torch.cuda.synchronize()
    assert len(outs) == nb
    for k in range(nb):
        _, scores, _, hw, cid, _ = _device_run(n, seed=seeds[k])
        g_cid, g_w, g_comb, g_long = (t.cpu().numpy() for t in outs[k])
        assert np.array_equal(g_cid, cid.cpu().numpy()), k
        assert np.array_equal(g_w, hw.cpu().numpy()), k
        assert np.array_equal(g_comb.view(np.uint64), scores["combined_score"][:n].cpu().numpy().view(np.uint64)), k
        assert np.array_equal(g_long, scores["longest_homopolymer_run"][:n].cpu().numpy()), k


@pytest.mark.parametrize("assign_on", ["main", "main_no_split", "separate", "main_mark_stream", "main_fused",
                                       "resolve"])
def test_pipeline_segment_mark(rg, assign_on):
    """>= 2^20 rows: the code-slice mark runs its segment (bucket) pass and merges one
    partial bitmap per row chunk. Every batch's ids, scores and Hamming bits equal the
    sequential device path."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth
    from rogtk_amd.pipeline import UmiPipeline

    n, L, nb = 1_100_009, 12, 4
    seeds = [synth.DEFAULT_SEED + 31 * k for k in range(nb)]
    outs = []

    def grab(slot, batch):
        outs.append((slot.cid[:n].clone(), slot.within.clone(), slot.scores["combined_score"][:n].clone()))

    mark_stream, fused = assign_on == "main_mark_stream", assign_on == "main_fused"
    split = assign_on != "main_no_split"  # round 5 default: the slice mark at the head of the resolve stream
    pipe = UmiPipeline(L, n, n, "cuda", depth=2, target=b"ACGTACGTACGT", max_distance=1, on_assigned=grab,
                       assign_on="main" if mark_stream or fused or not split else assign_on, mark_stream=mark_stream,
                       fused_assign=fused, split_mark=split)
    keep = []
    for s in seeds:
        keep.append(D.PackedBatch(torch.from_numpy(synth.umi_codes(n, L, seed=s).view(np.int32)).cuda(), L))
        pipe.submit(keep[-1])
    pipe.drain()
    torch.cuda.synchronize()
    assert len(outs) == nb
    for k in range(nb):
        _, scores, _, hw, cid, _ = _device_run(n, seed=seeds[k])
        g_cid, g_w, g_comb = (t.cpu().numpy() for t in outs[k])
        assert np.array_equal(g_cid, cid.cpu().numpy()), k
        assert np.array_equal(g_w, hw.cpu().numpy()), k
        assert np.array_equal(g_comb.view(np.uint64), scores["combined_score"][:n].cpu().numpy().view(np.uint64)), k


@pytest.mark.parametrize("spec", [1, 4])
@pytest.mark.parametrize("depth,nb", [(2, 5), (3, 3), (1, 2)])
@pytest.mark.parametrize("assign_on,gate,order", [("separate", "auto", "score_first"), ("separate", "resolve", "score_first"),
                                                  ("resolve", "auto", "score_first"), ("separate", "auto", "mark_first"),
                                                  ("separate", "auto", "late_assign"),
                                                  ("main", "auto", "mark_first"), ("main", "auto", "score_first"),
                                                  ("main", "auto", "mark_stream"), ("main", "auto", "fused")])
def test_pipeline_deferred_assign(rg, depth, nb, spec, assign_on, gate, order):
    """No on_assigned hook: assigns are enqueued before their resolve's flags are checked;
    with 1 speculative round every batch needs the deferred completion (rounds + labels +
    the assign again) when its slot comes round or at drain. With reuse_gate "resolve",
    score and mark of a slot's next batch do not wait for its assign.
    The slots' final outputs (ids, scores, Hamming bits) equal the sequential device path."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth
    from rogtk_amd.pipeline import UmiPipeline

    n, L = 200_003, 12
    seeds = [synth.DEFAULT_SEED + 29 * k for k in range(nb)]
    if order == "fused" and depth < 2:
        pytest.skip("the fused score + assign needs depth >= 2")
    try:
        D.set_spec_rounds(spec)
        pipe = UmiPipeline(L, n, n, "cuda", depth=depth, target=b"ACGTACGTACGT", max_distance=1,
                           assign_on=assign_on, reuse_gate=gate, score_alone=depth == 2,
                           mark_first=order != "score_first" and order != "late_assign",
                           assign_early=order != "late_assign", mark_stream=order == "mark_stream",
                           fused_assign=order == "fused")
        keep, last = [], {}
        for k, s in enumerate(seeds):
            codes = torch.from_numpy(synth.umi_codes(n, L, seed=s).view(np.int32)).cuda()
            keep.append(D.PackedBatch(codes, L))
            last[id(pipe.submit(keep[-1]))] = k
        pipe.drain()
        torch.cuda.synchronize()
    finally:
        D.set_spec_rounds(0)
    for slot in pipe.slots:
        if id(slot) not in last:
            continue
        k = last[id(slot)]
        _, scores, _, hw, cid, _ = _device_run(n, seed=seeds[k])
        assert np.array_equal(slot.cid[:n].cpu().numpy(), cid.cpu().numpy()), k
        assert np.array_equal(slot.scores["combined_score"][:n].cpu().numpy().view(np.uint64),
                              scores["combined_score"][:n].cpu().numpy().view(np.uint64)), k
        assert np.array_equal(slot.within.cpu().numpy()[:len(hw)], hw.cpu().numpy()), k


@pytest.mark.parametrize("assign_on,dev_ev", [("separate", True), ("main", True), ("separate", False)])
def test_pipeline_settle_gives_final_ids(rg, assign_on, dev_ev):
    """settle(slot) right after submit (1 speculative round: every batch needs the deferred
    completion) returns the final ids of that batch, mid-stream."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth
    from rogtk_amd.pipeline import UmiPipeline

    n, L = 150_001, 12
    seeds = [synth.DEFAULT_SEED + 31 * k for k in range(4)]
    try:
        D.set_spec_rounds(1)
        pipe = UmiPipeline(L, n, n, "cuda", depth=2, target=b"ACGTACGTACGT", max_distance=1, score_alone=True,
                           assign_on=assign_on, device_events=dev_ev)
        keep, got = [], []
        for s in seeds:
            codes = torch.from_numpy(synth.umi_codes(n, L, seed=s).view(np.int32)).cuda()
            keep.append(D.PackedBatch(codes, L))
            slot = pipe.submit(keep[-1])
            got.append(pipe.settle(slot)[:n].clone())
        pipe.drain()
        torch.cuda.synchronize()
    finally:
        D.set_spec_rounds(0)
    for k, s in enumerate(seeds):
        cid = _device_run(n, seed=s)[4]
        assert np.array_equal(got[k].cpu().numpy(), cid.cpu().numpy()), k


def _chain_codes(rng, L, length, high_bases):
    """Self-avoiding walk that changes one of the first `high_bases` bases per step (low bases
    fixed): every edge crosses LDS-local groups, so the global rounds carry the whole merge."""
    shift0 = 2 * (L - high_bases)
    low = int(rng.integers(1 << shift0))
    cur = int(rng.integers(4 ** high_bases))
    seen, path = {cur}, [cur]
    while len(path) < length:
        for _ in range(64):
            j = int(rng.integers(high_bases))
            b = int(rng.integers(1, 4))
            nxt = cur ^ (b << (2 * j))
            if nxt not in seen:
                break
        else:
            break
        seen.add(nxt)
        path.append(nxt)
        cur = nxt
    return np.array([(c << shift0) | low for c in path], dtype=np.uint32)


@pytest.mark.parametrize("spec", [1, 2])
@pytest.mark.parametrize("L", [12, 16])
def test_deferred_rounds_match(rg, L, spec):
    """With fewer speculative rounds than the data needs, the rounds that assign runs
    after the (speculative) labels must give the same clusters: labels never clobber
    the forest."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    n = 200_000
    codes_h = synth.umi_codes(n, L, seed=11)
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    eng = D.ClusterEngine(L, n, "cuda")
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    try:
        D.set_spec_rounds(spec)
        D.cluster_batch(eng, batch, cid, 1)
        rounds = eng.rounds()
    finally:
        D.set_spec_rounds(0)
    if spec == 1:
        assert rounds > spec  # the deferred path ran
    rc, _, rk, _ = P().umi_cluster(P().StrCol.from_fixed(synth.codes_to_ascii(codes_h, L)), L, 1)
    assert eng.stats()["n_clusters"] == rk
    assert np.array_equal(cid.cpu().numpy().view(np.uint32), rc)


@pytest.mark.parametrize("L", [12, 16])
def test_long_chains_need_extra_rounds(rg, L):
    """Long Hamming-1 paths (diameter >> speculative rounds) resolve exactly: the deferred
    completion in assign must finish them."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    rng = np.random.default_rng(L)
    parts = [_chain_codes(rng, L, 3000, min(L - 7, 8)) for _ in range(4)]
    codes_h = np.unique(np.concatenate(parts))
    codes_h = codes_h[rng.permutation(len(codes_h))]
    n = len(codes_h)
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    eng = D.ClusterEngine(L, n, "cuda")
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    D.cluster_batch(eng, batch, cid, 1)
    stats = eng.stats()
    rounds = eng.rounds()
    print(f"L={L} n={n} rounds={rounds}")
    rc, _, rk, _ = P().umi_cluster(P().StrCol.from_fixed(synth.codes_to_ascii(codes_h, L)), L, 1)
    assert stats["n_clusters"] == rk
    assert np.array_equal(cid.cpu().numpy().view(np.uint32), rc)
    assert rounds >= 1


@pytest.mark.parametrize("n", [1_000_000, 6_000_000])
@pytest.mark.parametrize("L", [10, 12, 14])
def test_dense_and_sparse_spaces(rg, L, n):
    """Dense (4^10 saturated at these sizes) and sparse (4^14) code spaces: ids equal the
    oracle's (1M) and are deterministic across two workspaces (6M)."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    codes_h = synth.umi_codes(n, L, seed=L + n)
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    batch = D.PackedBatch(codes, L)
    out = []
    for _ in range(2):
        eng = D.ClusterEngine(L, min(n, 4 ** L), "cuda")
        cid = torch.empty(n, dtype=torch.int32, device="cuda")
        D.cluster_batch(eng, batch, cid, 1)
        out.append((cid.cpu().numpy(), eng.stats()["n_clusters"]))
    assert out[0][1] == out[1][1] and np.array_equal(out[0][0], out[1][0])
    if n <= 1_000_000:
        rc, _, rk, _ = P().umi_cluster(P().StrCol.from_fixed(synth.codes_to_ascii(codes_h, L)), L, 1)
        assert out[0][1] == rk
        assert np.array_equal(out[0][0].view(np.uint32), rc)


@pytest.mark.parametrize("n", [0, 1, 5000, 300_000, 3_000_000, 1_048_579])
@pytest.mark.parametrize("L", [7, 8, 10, 11, 12, 13])
def test_mark_bitmap_sort_equals_presence_path(rg, L, n):
    """The partition-sort bitmap equals mark + local_bitmap bit for bit, with irregular
    rows (regular bit 0) mixed in, whose codes must not be marked."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    codes_h = synth.umi_codes(max(n, 1), L, seed=L * 7 + n)[:n] if n else np.zeros(0, np.uint32)
    codes = torch.from_numpy(codes_h.view(np.int32).copy()).cuda() if n else torch.zeros(4, dtype=torch.int32,
                                                                                          device="cuda")[:0]
    rng = np.random.default_rng(n)
    reg = rng.random(n) > 0.01
    if n:
        reg[-1] = False  # an irregular row in the last partition's bucket
        codes_h = codes_h.copy()
        codes_h[-1] = 4 ** L - 1
        codes = torch.from_numpy(codes_h.view(np.int32).copy()).cuda()
    bits = np.packbits(np.concatenate([reg, np.zeros((-n) % 64, bool)]), bitorder="little").view(np.int64)
    regbits = torch.from_numpy(bits.copy()).cuda() if n else torch.zeros(1, dtype=torch.int64, device="cuda")
    for rb in (regbits, None):
        batch = D.PackedBatch(codes, L, rb)
        a = D.ClusterEngine(L, max(min(n, 4 ** L), 1), "cuda")
        a.mark(batch)
        ref = a.build_local_bitmap().clone()
        for method in (D.MARK_SORT, D.MARK_SLICES):
            if method == D.MARK_SLICES and L > 12:
                continue
            try:
                D.set_mark_method(method)
                b = D.ClusterEngine(L, max(min(n, 4 ** L), 1), "cuda")
                got = b.mark_bitmap(batch).clone()
                torch.cuda.synchronize()
            finally:
                D.set_mark_method(D.MARK_AUTO)
            assert torch.equal(ref, got), (L, n, rb is None, method)


@pytest.mark.parametrize("L,skew", [(12, "one_slice"), (12, "two_slices"), (11, "one_slice"), (12, "uniform"),
                                    (12, "half")])
def test_slice_bucket_overflow_falls_back(rg, L, skew):
    """Slice mark with per-workgroup segments: rows concentrated in one or two code slices
    overflow their segments (4x the mean share), and the slice pass reads those rows
    instead, per chunk; every bitmap equals the presence path bit for bit."""
    import torch

    from rogtk_amd import device as D

    rng = np.random.default_rng(hash(skew) % 1000 + L)
    n = 2_100_000
    space = 4 ** L
    if skew == "one_slice":
        codes_h = rng.integers(0, 1 << 20, size=n, dtype=np.uint64).astype(np.uint32)
    elif skew == "two_slices":
        codes_h = (rng.integers(0, 1 << 20, size=n, dtype=np.uint64) + (rng.integers(0, 2, size=n) << 22).astype(np.uint64)).astype(np.uint32)
    else:
        codes_h = rng.integers(0, space, size=n, dtype=np.uint64).astype(np.uint32)
        if skew == "half":  # the second half in one slice: some chunks overflow, others not
            codes_h[n // 2:] = rng.integers(0, 1 << 20, size=n - n // 2, dtype=np.uint64).astype(np.uint32)
    codes = torch.from_numpy(codes_h.view(np.int32)).cuda()
    reg = rng.random(n) > 0.02
    bits = np.packbits(np.concatenate([reg, np.zeros((-n) % 64, bool)]), bitorder="little").view(np.int64)
    batch = D.PackedBatch(codes, L, torch.from_numpy(bits.copy()).cuda())
    a = D.ClusterEngine(L, min(n, space), "cuda")
    a.mark(batch)
    ref = a.build_local_bitmap().clone()
    try:
        D.set_mark_method(D.MARK_SLICES)
        b = D.ClusterEngine(L, min(n, space), "cuda")
        for _ in range(2):  # the bucket cursors are reset per call
            got = b.mark_bitmap(batch).clone()
            torch.cuda.synchronize()
            assert torch.equal(ref, got), skew
    finally:
        D.set_mark_method(D.MARK_AUTO)


def test_level2_transfers_pinned_and_pageable(rg):
    """The level-2 entry points move data by direct DMA for pinned buffers (rogtk_host_alloc:
    the Python API's results) and through the pinned staging chunks (32 MiB) for pageable
    ones: 6M rows (72 MB of values, 48 MB per f64 field) give the same bytes both ways and
    equal the oracle on a sample."""
    import ctypes

    from rogtk_amd import _lib
    from rogtk_amd import synth

    n, L = 6_000_000, 12
    asc = synth.umi_ascii(n, L, p_n=1e-4)
    offs = np.arange(0, (n + 1) * L, L, dtype=np.int64)
    vals = asc.reshape(-1)
    col = pa.Array.from_buffers(pa.large_binary(), n, [None, pa.py_buffer(offs), pa.py_buffer(vals)])
    pinned = rg.umi_complexity_scores(col)  # results in rogtk_host_alloc blocks
    out = {name: np.zeros(n, dtype=np.uint32 if name == "longest_homopolymer_run" else np.float64)
           for name, _ in rg.FIELDS}
    sc = _lib.UmiScores(*[ctypes.c_void_p(out[name].ctypes.data) for name, _ in rg.FIELDS])
    _lib.call("rogtk_umi_complexity_host", ctypes.c_void_p(offs.ctypes.data), 8, ctypes.c_void_p(vals.ctypes.data),
              vals.size, None, 0, n, ctypes.byref(sc))
    for name, _ in rg.FIELDS:
        a = _np(pinned.field(name))
        assert np.array_equal(a.view(np.uint64) if a.dtype == np.float64 else a,
                              out[name].view(np.uint64) if out[name].dtype == np.float64 else out[name]), name
    idx = np.random.default_rng(1).choice(n, size=20_000, replace=False)
    ref = P().umi_complexity(P().StrCol.from_fixed(asc[idx]))
    _assert_scores_equal({k: v[idx] for k, v in out.items()}, ref, np.ones(len(idx), bool))
    cid_p, k_p, _ = rg.umi_cluster(col, L, 1)
    cid = np.zeros(n, np.uint32)
    nk, rl = ctypes.c_int64(0), ctypes.c_int(0)
    _lib.call("rogtk_umi_cluster_host", ctypes.c_void_p(offs.ctypes.data), 8, ctypes.c_void_p(vals.ctypes.data),
              vals.size, None, 0, n, L, 1, ctypes.c_void_p(cid.ctypes.data), ctypes.byref(nk), ctypes.byref(rl))
    assert nk.value == k_p and np.array_equal(_np(cid_p).astype(np.uint32), cid)


@pytest.mark.parametrize("depth,rs,lag,assign_on", [(3, 2, 0, "main"), (4, 2, 3, "main"), (4, 3, 0, "main"),
                                                    (2, 1, 0, "separate"), (3, 2, 0, "separate")])
def test_pipeline_resolve_streams(rg, depth, rs, lag, assign_on):
    """resolve_streams > 1 (consecutive batches resolve on different streams) with the
    default schedule, with assign_lag, and with the assign on a stream of its own (the split
    mark then spans three streams): every batch's ids, scores and Hamming bits,
    taken at its on_assigned hook, equal the sequential device path."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth
    from rogtk_amd.pipeline import UmiPipeline

    n, L, nb = 600_011, 12, 6
    seeds = [synth.DEFAULT_SEED + 13 * k for k in range(nb)]
    outs = []

    def grab(slot, batch):
        outs.append((slot.cid[:n].clone(), slot.within.clone(), slot.scores["combined_score"][:n].clone()))

    pipe = UmiPipeline(L, n, n, "cuda", depth=depth, target=b"ACGTACGTACGT", max_distance=1, on_assigned=grab,
                       resolve_streams=rs, assign_lag=lag, assign_on=assign_on)
    assert pipe.split_mark
    keep = []
    for s in seeds:
        keep.append(D.PackedBatch(torch.from_numpy(synth.umi_codes(n, L, seed=s).view(np.int32)).cuda(), L))
        pipe.submit(keep[-1])
    pipe.drain()
    torch.cuda.synchronize()
    assert len(outs) == nb
    for k in range(nb):
        _, scores, _, hw, cid, _ = _device_run(n, seed=seeds[k])
        g_cid, g_w, g_comb = (t.cpu().numpy() for t in outs[k])
        assert np.array_equal(g_cid, cid.cpu().numpy()), k
        assert np.array_equal(g_w, hw.cpu().numpy()), k
        assert np.array_equal(g_comb.view(np.uint64), scores["combined_score"][:n].cpu().numpy().view(np.uint64)), k


def test_events_ride_on_dispatch_packets(rg):
    """rogtk_event_attach_next: the slice-bucket pass and the resolve's last kernel record
    the pipeline's hand-off events on their own dispatch packets. A second stream that waits
    only for those events sees the finished mark / resolve: its ids equal the plain path's."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    n, L = 2_000_003, 12
    batch = D.PackedBatch(torch.from_numpy(synth.umi_codes(n, L, seed=synth.DEFAULT_SEED + 5).view(np.int32)).cuda(), L)
    _, _, _, _, cid_ref, _ = _device_run(n, seed=synth.DEFAULT_SEED + 5)
    eng = D.ClusterEngine(L, n, "cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    marked = D.StreamEvent()
    marked.attach_next()
    eng.mark_bitmap(batch, stream=s1, phase=1)
    assert marked.attach_done()  # the bucket pass took it (10M-row segment mode applies at 2M)
    marked.wait(s2)
    eng.mark_bitmap(batch, stream=s2, phase=2)
    resolved = D.StreamEvent()
    resolved.attach_next()
    eng.resolve(eng.local_bitmap, 1, 1, stream=s2)
    assert resolved.attach_done()
    resolved.wait(s1)
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    eng.assign(batch, cid, stream=s1)
    torch.cuda.synchronize()
    assert np.array_equal(cid.cpu().numpy(), cid_ref.cpu().numpy())
