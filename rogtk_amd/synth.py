"""Seeded synthetic UMIs / reads (spec "synth-v1", rogtk_amd/csrc/synth.cpp).

Every read is a pure function of (seed, read index): a rank generates its shard
[start, start+count) of one global dataset of n_total reads with O(count) work.
Defaults follow SURVEY.md §8d: 12-bp UMIs, M = N/10 molecules, UMI substitution
rate 0.001/base, read substitution rate 0.005/base, seed 0x524F47544B ("ROGTK").
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

DEFAULT_SEED = 0x524F47544B
P_UMI_SUB = 0.001
P_READ_SUB = 0.005


def umi_codes(n_total: int, umi_len: int = 12, seed: int = DEFAULT_SEED, p_sub: float = P_UMI_SUB,
              start: int = 0, count: int | None = None) -> np.ndarray:
    """Packed uint32 codes (first base most significant) of reads [start, start+count)."""
    count = n_total - start if count is None else count
    out = np.empty(max(count, 1), dtype=np.uint32)
    rc = _lib.synth().rogtk_synth_umis_codes(n_total, umi_len, seed, p_sub, start, count,
                                             ctypes.c_void_p(out.ctypes.data))
    if rc:
        raise ValueError("umi_len must be 1..16 for packed codes")
    return out[:count]


def umi_ascii(n_total: int, umi_len: int = 12, seed: int = DEFAULT_SEED, p_sub: float = P_UMI_SUB,
              p_n: float = 0.0, p_lower: float = 0.0, start: int = 0, count: int | None = None) -> np.ndarray:
    """Fixed-width ASCII UMIs as an (count, umi_len) uint8 array."""
    count = n_total - start if count is None else count
    out = np.empty((max(count, 1), umi_len), dtype=np.uint8)
    _lib.synth().rogtk_synth_umis_ascii(n_total, umi_len, seed, p_sub, p_n, p_lower, start, count,
                                        ctypes.c_void_p(out.ctypes.data))
    return out[:count]


def reads(n_total: int, read_len: int = 150, seed: int = DEFAULT_SEED, p_sub: float = P_READ_SUB,
          start: int = 0, count: int | None = None) -> np.ndarray:
    count = n_total - start if count is None else count
    out = np.empty((max(count, 1), read_len), dtype=np.uint8)
    _lib.synth().rogtk_synth_reads(n_total, read_len, seed, p_sub, start, count,
                                   ctypes.c_void_p(out.ctypes.data))
    return out[:count]


def molecules(n_total: int, seed: int = DEFAULT_SEED, start: int = 0, count: int | None = None) -> np.ndarray:
    count = n_total - start if count is None else count
    out = np.empty(max(count, 1), dtype=np.uint64)
    _lib.synth().rogtk_synth_molecules(n_total, seed, start, count, ctypes.c_void_p(out.ctypes.data))
    return out[:count]


def codes_to_ascii(codes: np.ndarray, umi_len: int) -> np.ndarray:
    """Unpack codes to an (n, L) uint8 ASCII array (numpy, host)."""
    shifts = np.arange(umi_len - 1, -1, -1, dtype=np.uint32) * 2
    idx = (codes[:, None] >> shifts[None, :]) & 3
    return np.frombuffer(b"ACGT", dtype=np.uint8)[idx]


def ascii_to_strings(arr: np.ndarray):
    return [bytes(r) for r in arr]
