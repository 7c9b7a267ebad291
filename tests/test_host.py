"""CPU: the C-ABI library loads and exports what include/rogtk_hip.h declares, fails
loudly without a GPU, and the host-side pieces (synthetic generator, Arrow column
adapter, sharding) behave as specified."""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np
import pyarrow as pa
import pytest

from conftest import ROOT


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "rogtk_hip.h")).read()
    return sorted(set(re.findall(r"\b(rogtk_[a-z0-9_]+)\s*\(", hdr)))


def test_header_declares_the_boundary():
    syms = _declared_symbols()
    for must in ("rogtk_umi_score_packed", "rogtk_umi_score_rows", "rogtk_stage_strings",
                 "rogtk_cluster_resolve", "rogtk_cluster_assign", "rogtk_umi_complexity_host",
                 "rogtk_hamming_host", "rogtk_umi_cluster_host", "rogtk_last_error"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    from rogtk_amd import _lib

    lib = ctypes.CDLL(_lib.HIP_LIB_PATH)
    missing = [s for s in _declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_every_symbol():
    from rogtk_amd import _lib

    bound = set(_lib.SIGNATURES) | set(_lib.VOID_SIGNATURES) | {"rogtk_version", "rogtk_last_error"}
    assert set(_declared_symbols()) <= bound


def test_no_device_fails_loudly():
    import torch

    import rogtk_amd as rg

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert rg.device_count() == 0
    with pytest.raises(rg.RogtkError) as e:
        rg.umi_complexity_scores(["ACGT"])
    assert e.value.code == 4 and "no HIP device" in str(e.value)


def test_argument_errors_cross_the_abi_as_status_codes():
    from rogtk_amd import _lib

    lib = _lib.hip()
    nbytes = ctypes.c_int64(0)
    assert lib.rogtk_cluster_workspace_size(17, 10, ctypes.byref(nbytes)) == _lib.ROGTK_E_UNSUPPORTED
    assert b"umi_len 17" in lib.rogtk_last_error()
    assert lib.rogtk_cluster_workspace_size(12, 0, ctypes.byref(nbytes)) == _lib.ROGTK_E_INVALID
    assert lib.rogtk_cluster_workspace_size(12, 10_000_000, ctypes.byref(nbytes)) == 0
    assert nbytes.value > 4 ** 12  # presence table + rank tables + labels
    words = ctypes.c_int64(0)
    assert lib.rogtk_cluster_bitmap_words(12, ctypes.byref(words)) == 0 and words.value == 4 ** 12 // 64
    assert lib.rogtk_cluster_bitmap_words(1, ctypes.byref(words)) == 0 and words.value == 1
    assert lib.rogtk_profile_read(b"nope", ctypes.byref(ctypes.c_double()), ctypes.byref(ctypes.c_int64())) == 1


def test_event_attach_disarms_without_a_launch():
    """rogtk_event_attach_next arms an event for the next library launch of this thread;
    with no launch in between, attach_done reports it untaken (the caller then records it)
    and disarms, so a later launch cannot pick up a stale event. No HIP call is made."""
    from rogtk_amd import _lib

    lib = _lib.hip()
    taken = ctypes.c_int32(7)
    assert lib.rogtk_event_attach_next(ctypes.c_void_p(0x1000)) == 0
    assert lib.rogtk_event_attach_done(ctypes.byref(taken)) == 0 and taken.value == 0
    assert lib.rogtk_event_attach_done(ctypes.byref(taken)) == 0 and taken.value == 0
    assert lib.rogtk_event_attach_done(None) == _lib.ROGTK_E_INVALID


def test_synth_is_deterministic_and_shardable():
    from rogtk_amd import synth

    n = 50_000
    full = synth.umi_codes(n, 12)
    parts = np.concatenate([synth.umi_codes(n, 12, start=s, count=c)
                            for s, c in ((0, 12_345), (12_345, 20_000), (32_345, n - 32_345))])
    assert np.array_equal(full, parts)
    assert np.array_equal(full, synth.umi_codes(n, 12))
    asc = synth.umi_ascii(n, 12)
    assert np.array_equal(synth.codes_to_ascii(full, 12), asc)
    # family structure: ~N/10 molecules, UMI errors ~0.001/base
    mol = synth.molecules(n)
    assert 0.8 * n / 10 < len(np.unique(mol)) <= n / 10
    assert 1_000 < len(np.unique(full)) < 1.3 * n / 10 * 1.1


def test_synth_stress_variants_have_irregular_bytes():
    from rogtk_amd import synth

    a = synth.umi_ascii(20_000, 12, p_n=5e-3, p_lower=5e-3)
    assert (a == ord("N")).any() and ((a >= ord("a")) & (a <= ord("z"))).any()
    r = synth.reads(1000, 150)
    assert r.shape == (1000, 150) and set(np.unique(r)) <= set(b"ACGT")


def test_arrow_column_adapter_rebases_slices():
    from rogtk_amd.columns import chunks

    arr = pa.array(["AC", None, "GGT", "", "TTTT"] * 3)[4:11]
    (ch,) = list(chunks(arr))
    assert ch.n == 7 and ch.offsets[0] == 0
    got = [None if not ((ch.validity[(ch.validity_offset + i) // 8] >> ((ch.validity_offset + i) % 8)) & 1)
           else ch.values[ch.offsets[i]:ch.offsets[i + 1]].tobytes().decode() for i in range(ch.n)]
    assert got == arr.to_pylist()
    big = pa.chunked_array([pa.array(["A", "C"]), pa.array(["G"], type=pa.string())])
    assert [c.n for c in chunks(big)] == [2, 1]
    (fx,) = list(chunks(np.array([b"ACGT", b"TTTT"], dtype="S4")))
    assert fx.values.tobytes() == b"ACGTTTTT" and fx.offset_width == 8


def test_shard_ranges_cover_exactly():
    from rogtk_amd.dist import shard_range

    for n, w in ((10, 3), (1_000_003, 8), (7, 8)):
        spans = [shard_range(n, r, w) for r in range(w)]
        assert spans[0][0] == 0
        for (s0, c0), (s1, _) in zip(spans, spans[1:]):
            assert s0 + c0 == s1
        assert sum(c for _, c in spans) == n
