"""H4 k-mer spectra on the GPU vs the oracle (oracle/kmer_oracle.cpp), bit-exact.

Every output array (k-mer codes, censored exts, saturating counts, per-group entry
offsets and the 5 per-group stats) must equal the oracle's for the same column and
groups: effective k 4/8/16/32/64, auto_k, min_coverage, nulls, lowercase, N and
other bytes (row dropped), empty rows, rows shorter than k, k > 64, many groups.
"""
from __future__ import annotations

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu
_LAST_MODE = [1]


@pytest.fixture(scope="module", params=["lds", "global"])
def rg(request):
    """Every test runs twice: small groups in LDS (default) and all groups through
    the global radix-sort path (rogtk_kmer_set_path(0))."""
    import rogtk_amd
    from rogtk_amd import _lib

    _LAST_MODE[0] = 1 if request.param == "lds" else 0
    _lib.call("rogtk_kmer_set_path", _LAST_MODE[0])
    yield rogtk_amd
    _lib.call("rogtk_kmer_set_path", 1)


def P():
    from oracle import pyoracle
    return pyoracle


def _check(rg, items, k, min_cov, auto_k=False, group_offsets=None):
    col = P().StrCol.from_list(items)
    ref = P().kmer_spectrum(col, k, min_cov, auto_k, group_offsets)
    got = rg.kmer_spectrum(pa.array(items, type=pa.large_binary()), k, min_cov, auto_k, group_offsets)
    assert np.array_equal(got["entry_offsets"], ref["group_offsets"])
    assert np.array_equal(got["stats"], ref["stats"])
    for f in ("kmer_hi", "kmer_lo", "exts", "counts"):
        assert np.array_equal(got[f], ref[f]), f
    return got


def _reads(rng, n, lo, hi, alphabet=b"ACGT"):
    out = []
    for _ in range(n):
        L = int(rng.integers(lo, hi + 1))
        out.append(bytes(rng.choice(np.frombuffer(alphabet, np.uint8), L)))
    return out


def test_reference_fixture_sequences(rg):
    """fracture.rs:611-626 test sequences (their 44-bp assembly = 29 16-mers for k=13)."""
    seqs = [b"GAGACTGCATGGGCTGGTGGGCGTCCGTCTGC", b"GGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"]
    for k in (4, 13, 20, 33):
        _check(rg, seqs, k, 1)
    got = _check(rg, seqs, 13, 1)
    contig = b"GAGACTGCATGGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"
    want = sorted({contig[i:i + 16] for i in range(len(contig) - 15)})
    have = [P().kmer_to_str(h, l, 16).encode() for h, l in zip(got["kmer_hi"], got["kmer_lo"])]
    assert have == want


@pytest.mark.parametrize("k", [1, 4, 5, 8, 11, 16, 17, 31, 32, 33, 47, 64, 65, 100])
@pytest.mark.parametrize("min_cov", [1, 2, 5])
def test_single_group_all_k(rg, k, min_cov):
    rng = np.random.default_rng(k * 10 + min_cov)
    template = _reads(rng, 1, 200, 200)[0]
    items = []
    for _ in range(30):  # overlapping fragments of one template -> real coverage
        a = int(rng.integers(0, 120))
        items.append(template[a:a + int(rng.integers(20, 80))])
    items += [None, b"", b"ACGTNACGT" * 4, b"acgtacgtacgtacgtacgtACGTACGTAAACCC", b"AC"]
    _check(rg, items, k, min_cov)


def test_auto_k(rg):
    rng = np.random.default_rng(5)
    for lens in ((10, 20), (30, 40), (90, 150), (150, 150), (1, 3), (0, 0)):
        items = _reads(rng, 12, *lens) + [None]
        _check(rg, items, 0, 1, auto_k=True)
    _check(rg, [], 0, 1, auto_k=True)
    _check(rg, [None, None], 0, 1, auto_k=True)


def test_many_groups_mixed(rg):
    """Many groups, each one polars group: sizes 0..600 rows (small and medium ones take
    the LDS size classes 3, 1 and 4, groups of more than 512 rows the global path, all in
    the same call), mixed validity and bytes."""
    rng = np.random.default_rng(11)
    items, go = [], [0]
    for g in range(300):
        u = rng.random()  # LDS classes (<= 512 rows) and global-path groups (> 512 rows)
        m = int(rng.integers(0, 40)) if u < 0.8 else int(rng.integers(60, 200)) if u < 0.9 else int(rng.integers(513, 600))
        tpl = _reads(rng, 1, 150, 150)[0]
        for _ in range(m):
            r = rng.random()
            if r < 0.03:
                items.append(None)
            elif r < 0.06:
                items.append(b"ACGTN" + tpl[:40])
            elif r < 0.09:
                items.append(tpl[:60].lower())
            else:
                a = int(rng.integers(0, 60))
                items.append(tpl[a:a + int(rng.integers(30, 91))])
        go.append(len(items))
    import ctypes

    from rogtk_amd import _lib

    for k, mc in ((17, 3), (13, 1), (31, 2), (33, 2), (7, 4)):
        _check(rg, items, k, mc, group_offsets=go)
        paths = (ctypes.c_int64 * 2)()
        _lib.call("rogtk_kmer_path_stats", paths)
        if k > 32 or _LAST_MODE[0] == 0:
            assert paths[0] == 0 and paths[1] == 300
        else:
            assert paths[0] > 100 and paths[1] > 10 and paths[0] + paths[1] == 300, tuple(paths)
    _check(rg, items, 0, 2, auto_k=True, group_offsets=go)


def test_long_rows_and_chunk_edges(rg):
    """Rows of 193..700 bases (the staging kernel's 4th 64-base chunk and its tail loop
    past 256 bases, with a bad byte past 256 dropping a row), and group counts around
    the LDS path's 64-group chunks (63, 64, 65, 130 groups: partial last chunks, chunks
    whose groups are all of one class or of none)."""
    rng = np.random.default_rng(21)
    for n_groups in (63, 64, 65, 130):
        items, go = [], [0]
        for g in range(n_groups):
            tpl = _reads(rng, 1, 800, 800)[0]
            m = int(rng.integers(0, 12)) if g % 7 else int(rng.integers(25, 40))
            for _ in range(m):
                a = int(rng.integers(0, 90))
                r = bytearray(tpl[a:a + int(rng.integers(193, 701))])
                if len(r) > 258 and rng.random() < 0.05:
                    r[int(rng.integers(257, len(r)))] = ord("N")  # past the first 256 bases
                items.append(bytes(r))
            go.append(len(items))
        for k, mc in ((17, 2), (31, 1)):
            _check(rg, items, k, mc, group_offsets=go)


def test_lds_class4_overflow(rg):
    """Groups move along the LDS classes by their distinct and valid k-mers: class 3
    (<= 1472 distinct, <= 1024 valid) -> class 1 (<= 2048 distinct) -> class 4 (<= 6144
    distinct, <= 2048 valid) -> the global path. `mid_valid` (1190 valid k-mers at
    min_cov 1) leaves class 3 for class 1 (its bitonic sort pads to 2048 entries, more
    than class 3's buffer). Every case == the oracle."""
    import ctypes

    from rogtk_amd import _lib

    rng = np.random.default_rng(8)
    tpl = _reads(rng, 1, 400, 400)[0]
    fits = [tpl[int(a):int(a) + 150] for a in rng.integers(0, 250, 60)]  # ~7k obs, few distinct
    many_distinct = _reads(rng, 100, 150, 150)  # 11.9k distinct k-mers
    many_valid = _reads(rng, 40, 150, 150)  # 4.8k distinct, all valid at min_cov 1
    mid_valid = _reads(rng, 10, 150, 150)  # 1190 distinct k-mers, all valid at min_cov 1
    groups = [fits, many_distinct, many_valid, fits[:5], mid_valid]
    items = [x for grp in groups for x in grp]
    go = np.r_[0, np.cumsum([len(grp) for grp in groups])].tolist()
    for k, mc in ((17, 1), (31, 2), (21, 1)):
        _check(rg, items, k, mc, group_offsets=go)
        paths = (ctypes.c_int64 * 2)()
        _lib.call("rogtk_kmer_path_stats", paths)
        if _LAST_MODE[0] == 1:
            # the distinct-overflow group always leaves; the valid-overflow one at min_cov 1
            assert paths[1] == (2 if mc == 1 else 1) and paths[0] == 5 - paths[1], tuple(paths)


def test_saturating_count(rg):
    """> 65535 observations of one k-mer: the count saturates at u16::MAX (CountFilter)."""
    items = [b"A" * 80] * 1200  # 77 observations of AAAA..(k=4) per row -> 92,400
    got = _check(rg, items, 4, 1)
    assert int(got["counts"][0]) == 0xFFFF
    _check(rg, items, 4, 70000)  # saturated count never reaches min_cov > 65535


def test_large_group(rg):
    """One group of 20k reads (2.4M observations at k_eff 32)."""
    rng = np.random.default_rng(3)
    tpl = _reads(rng, 1, 2000, 2000)[0]
    items = []
    for _ in range(20000):
        a = int(rng.integers(0, 1850))
        items.append(tpl[a:a + 150])
    _check(rg, items, 17, 20)


def test_group_by_key_device(rg):
    """rogtk_group_by_key == numpy stable argsort + run boundaries."""
    import torch

    from rogtk_amd import device as D

    rng = np.random.default_rng(2)
    # key ranges: the sort covers only the largest key's significant bits (all-zero keys,
    # a power-of-two bound, the full 32 bits with the null id)
    for n, hi in ((1, 5), (1000, 7), (5000, 1), (200_003, 1 << 23), (100_003, 50_000), (300_000, 0xFFFFFFFF)):
        keys = rng.integers(0, hi, n, dtype=np.uint64).astype(np.uint32)
        if n > 10 and hi > 1 << 23:
            keys[:5] = 0xFFFFFFFF  # null ids group last
        rows, go, G = D.group_by_key(torch.from_numpy(keys.view(np.int32)).cuda())
        order = np.argsort(keys, kind="stable")
        sk = keys[order]
        heads = np.flatnonzero(np.r_[True, sk[1:] != sk[:-1]])
        assert G == len(heads)
        assert np.array_equal(rows.cpu().numpy(), order)
        assert np.array_equal(go.cpu().numpy(), np.r_[heads, n])


@pytest.mark.parametrize("k,min_cov", [(17, 3), (13, 1), (33, 2), (70, 1)])
def test_device_spectrum_with_grouping(rg, k, min_cov):
    """Level-1 path: device column + device group_by permutation == host path on the
    same column physically regrouped (and so == the oracle)."""
    import torch

    from rogtk_amd import device as D

    rng = np.random.default_rng(k)
    n_mol = 400
    tpls = _reads(rng, n_mol, 150, 150)
    mol = rng.integers(0, n_mol, 6000)
    items = []
    for m in mol:
        t = tpls[m]
        a = int(rng.integers(0, 40))
        r = bytearray(t[a:a + 110])
        if rng.random() < 0.02:
            r[5] = ord("N")
        items.append(bytes(r))
    lens = np.array([len(x) for x in items], dtype=np.int64)
    offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
    vals = np.frombuffer(b"".join(items), dtype=np.uint8)
    rows, go, G = D.group_by_key(torch.from_numpy(mol.astype(np.uint32).view(np.int32)).cuda())
    cap = int(sum(max(0, L - 3) for L in lens))
    out = D.kmer_spectrum_dev(torch.from_numpy(offs).cuda(), torch.from_numpy(vals.copy()).cuda(), go, k, min_cov,
                              cap, rows=rows)
    order = rows.cpu().numpy()
    grouped = [items[i] for i in order]
    ref = P().kmer_spectrum(P().StrCol.from_list(grouped), k, min_cov, False, go.cpu().numpy())
    assert np.array_equal(out["entry_offsets"].cpu().numpy(), ref["group_offsets"])
    assert np.array_equal(out["stats"].cpu().numpy(), ref["stats"])
    km = out["kmers"].cpu().numpy().view(np.uint64)
    assert np.array_equal(km[:, 0], ref["kmer_hi"]) and np.array_equal(km[:, 1], ref["kmer_lo"])
    assert np.array_equal(out["exts"].cpu().numpy(), ref["exts"])
    assert np.array_equal(out["counts"].cpu().numpy().view(np.uint16), ref["counts"])


@pytest.mark.parametrize("k", [4, 9, 17, 32])
def test_capacity_bound_tight(rg, k):
    """Output capacity is sum(len - 3) / min_coverage per group (every valid k-mer takes at
    least min_coverage observations). Groups of R identical reads at min_coverage R make
    every distinct k-mer valid, the tightest case; a poly-A group has one k-mer seen
    len - k + 1 times per read. Host path and the device block path (group_spectra, one
    call) both equal the oracle."""
    import torch

    from rogtk_amd import device as D

    rng = np.random.default_rng(100 + k)
    R = 3
    items, keys = [], []
    for g in range(60):
        r = _reads(rng, 1, 40, 220)[0]
        items += [r] * R
        keys += [g] * R
    items += [b"A" * 150] * 2
    keys += [60] * 2
    go = np.r_[0, np.cumsum(np.bincount(keys))].astype(np.int64)
    _check(rg, items, k, R, group_offsets=go)
    lens = np.array([len(x) for x in items], dtype=np.int64)
    offs = torch.from_numpy(np.r_[0, np.cumsum(lens)].astype(np.int64)).cuda()
    vals = torch.from_numpy(np.frombuffer(b"".join(items), dtype=np.uint8).copy()).cuda()
    kt = torch.from_numpy(np.array(keys, dtype=np.uint32).view(np.int32)).cuda()
    rows, dgo, G, calls = D.group_spectra(offs, vals, kt, k, R)
    assert G == 61 and len(calls) == 1
    ref = P().kmer_spectrum(P().StrCol.from_list(items), k, R, False, go)  # keys already grouped
    out = calls[0][2]
    assert np.array_equal(out["entry_offsets"].cpu().numpy(), ref["group_offsets"])
    assert np.array_equal(out["stats"].cpu().numpy(), ref["stats"])
    km = out["kmers"].cpu().numpy().view(np.uint64)
    assert np.array_equal(km[:, 0], ref["kmer_hi"]) and np.array_equal(km[:, 1], ref["kmer_lo"])
    assert np.array_equal(out["counts"].cpu().numpy().view(np.uint16), ref["counts"])
