"""TEST INFRASTRUCTURE ONLY — Python side of the CPU oracle.

Two things live here:

1. ctypes bindings of ``librogtk_oracle.so`` (the C++ restatement in
   ``rogtk_oracle.cpp``), used as the checker by tests/ and as the CPU baseline
   by bench.py.
2. An independent pure-Python restatement of the same reference functions,
   used only to cross-check the C++ oracle on small inputs:

   * ``py_umi_complexity``  — /root/reference/src/umi_score.rs:17-200
   * ``py_hamming``         — /root/reference/src/expressions.rs:1048-1101
   * ``py_cluster_bruteforce`` — the H3 spec by O(n^2) union-find
     over all pairs with the H2 distance, no neighbour enumeration.

Parity status: pinned by SURVEY.md Appendix A known answers (tests/test_oracle.py)
and by golden vectors committed under tests/golden/ (tests/make_golden.py).
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Iterable, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "librogtk_oracle.so")
_lib = None


def build() -> str:
    """Compile the oracle (g++) in-tree if it is missing or stale."""
    src = os.path.join(_HERE, "rogtk_oracle.cpp")
    if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, i32, u32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32
        L.oracle_umi_complexity.argtypes = [vp, i64, i32, vp, vp]
        L.oracle_umi_complexity.restype = None
        L.oracle_umi_complexity_batch.argtypes = [vp, i32, vp, vp, i64, i64, i32] + [vp] * 7
        L.oracle_umi_complexity_batch.restype = None
        L.oracle_hamming_batch.argtypes = [vp, i32, vp, vp, i64, i64, vp, i64, u32, vp, vp]
        L.oracle_hamming_batch.restype = None
        L.oracle_umi_cluster.argtypes = [vp, i32, vp, vp, i64, i64, i32, i32, vp, vp, vp]
        L.oracle_umi_cluster.restype = i64
        L.oracle_plogp.argtypes = [u32, u32]
        L.oracle_plogp.restype = ctypes.c_double
        L.oracle_version.restype = ctypes.c_char_p
        _lib = L
    return _lib


# --------------------------------------------------------------------------
# Arrow-style string column helpers (offsets int64, values u8, validity bitmap)
# --------------------------------------------------------------------------
class StrCol:
    """Minimal Arrow large_string layout held in numpy arrays."""

    def __init__(self, offsets: np.ndarray, values: np.ndarray, validity: Optional[np.ndarray], n: int):
        self.offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self.values = np.ascontiguousarray(values, dtype=np.uint8)
        self.validity = None if validity is None else np.ascontiguousarray(validity, dtype=np.uint8)
        self.n = int(n)

    @classmethod
    def from_list(cls, items: Sequence[Optional[object]]) -> "StrCol":
        n = len(items)
        offs = np.zeros(n + 1, dtype=np.int64)
        chunks = []
        valid = np.ones(n, dtype=bool)
        pos = 0
        for i, s in enumerate(items):
            if s is None:
                valid[i] = False
            else:
                b = s.encode("utf-8") if isinstance(s, str) else bytes(s)
                chunks.append(b)
                pos += len(b)
            offs[i + 1] = pos
        values = np.frombuffer(b"".join(chunks), dtype=np.uint8) if pos else np.zeros(1, np.uint8)
        validity = None if valid.all() else np.packbits(valid, bitorder="little")
        return cls(offs, values, validity, n)

    @classmethod
    def from_fixed(cls, arr: np.ndarray) -> "StrCol":
        """(n, L) uint8 array of equal-length, all-valid strings."""
        n, L = arr.shape
        offs = np.arange(n + 1, dtype=np.int64) * L
        return cls(offs, arr.reshape(-1).copy() if n * L else np.zeros(1, np.uint8), None, n)

    def valid_mask(self) -> np.ndarray:
        if self.validity is None:
            return np.ones(self.n, dtype=bool)
        return np.unpackbits(self.validity, bitorder="little")[: self.n].astype(bool)

    def get(self, i: int) -> Optional[bytes]:
        if not self.valid_mask()[i]:
            return None
        return self.values[self.offsets[i]: self.offsets[i + 1]].tobytes()

    def to_list(self):
        vm = self.valid_mask()
        return [self.values[self.offsets[i]: self.offsets[i + 1]].tobytes() if vm[i] else None
                for i in range(self.n)]

    def _ptrs(self):
        vp = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)
        return vp(self.offsets), vp(self.values), vp(self.validity)


FIELDS = ("shannon_entropy", "linguistic_complexity", "homopolymer_fraction",
          "dinucleotide_entropy", "longest_homopolymer_run", "dust_score", "combined_score")


def umi_complexity(col: StrCol, dinuc_order: int = 0) -> dict:
    """Oracle H1 over a column. Returns dict field -> numpy array (+ 'valid')."""
    L = lib()
    n = col.n
    out = {f: np.zeros(n, dtype=np.uint32 if f == "longest_homopolymer_run" else np.float64) for f in FIELDS}
    o, v, val = col._ptrs()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    L.oracle_umi_complexity_batch(o, 8, v, val, 0, n, dinuc_order,
                                  vp(out["shannon_entropy"]), vp(out["linguistic_complexity"]),
                                  vp(out["homopolymer_fraction"]), vp(out["dinucleotide_entropy"]),
                                  vp(out["longest_homopolymer_run"]), vp(out["dust_score"]),
                                  vp(out["combined_score"]))
    out["valid"] = col.valid_mask()
    return out


def hamming(col: StrCol, target: str | bytes, max_distance: int = 1):
    L = lib()
    t = target.encode() if isinstance(target, str) else bytes(target)
    tb = np.frombuffer(t, dtype=np.uint8) if t else np.zeros(1, np.uint8)
    dist = np.zeros(col.n, dtype=np.uint32)
    within = np.zeros(col.n, dtype=np.uint8)
    o, v, val = col._ptrs()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    L.oracle_hamming_batch(o, 8, v, val, 0, col.n, vp(tb), len(t), max_distance, vp(dist), vp(within))
    return dist, within.astype(bool), col.valid_mask()


def umi_cluster(col: StrCol, umi_len: int = 0, max_distance: int = 1):
    """Oracle H3. Returns (cluster_id u32, valid bool, n_clusters, resolved L)."""
    L = lib()
    cid = np.zeros(col.n, dtype=np.uint32)
    valid = np.zeros(col.n, dtype=np.uint8)
    rl = ctypes.c_int(0)
    o, v, val = col._ptrs()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    k = L.oracle_umi_cluster(o, 8, v, val, 0, col.n, umi_len, max_distance, vp(cid), vp(valid),
                             ctypes.byref(rl))
    if k < 0:
        raise ValueError("oracle_umi_cluster: bad arguments")
    return cid, valid.astype(bool), int(k), rl.value


def umi_complexity_one(s: bytes, dinuc_order: int = 0):
    L = lib()
    buf = np.frombuffer(s, dtype=np.uint8) if s else np.zeros(1, np.uint8)
    out6 = np.zeros(6, dtype=np.float64)
    lg = np.zeros(1, dtype=np.uint32)
    L.oracle_umi_complexity(buf.ctypes.data_as(ctypes.c_void_p), len(s), dinuc_order,
                            out6.ctypes.data_as(ctypes.c_void_p), lg.ctypes.data_as(ctypes.c_void_p))
    return {"shannon_entropy": out6[0], "linguistic_complexity": out6[1],
            "homopolymer_fraction": out6[2], "dinucleotide_entropy": out6[3],
            "longest_homopolymer_run": int(lg[0]), "dust_score": out6[4], "combined_score": out6[5]}


# --------------------------------------------------------------------------
# Independent pure-Python restatement (small inputs only)
# --------------------------------------------------------------------------
def py_umi_complexity(s: bytes, dinuc_order: int = 0) -> dict:
    n = len(s)
    # shannon_entropy umi_score.rs:45-73
    counts = [s.count(b) for b in b"ACGT"]
    if n == 0:
        sh = 0.0
    else:
        sh = 0.0
        for c in counts:
            if c > 0:
                p = c / n
                sh -= p * math.log2(p)
    # linguistic_complexity :77-93
    ling = 0.0 if n < 3 else len({s[i:i + 3] for i in range(n - 2)}) / min(n - 2, 64)
    # homopolymer_fraction :96-121
    if n == 0:
        homo = 0.0
    else:
        inh, i = 0, 0
        while i < n:
            r = 1
            while i + r < n and s[i + r] == s[i]:
                r += 1
            if r >= 3:
                inh += r
            i += r
        homo = inh / n
    # dinucleotide_entropy :124-146
    if n < 2:
        di = 0.0
    else:
        pairs = {}
        for i in range(n - 1):
            k = s[i:i + 2]
            pairs[k] = pairs.get(k, 0) + 1  # dict keeps first-occurrence order
        keys = sorted(pairs) if dinuc_order == 0 else list(pairs)
        e = 0.0
        for k in keys:
            p = pairs[k] / (n - 1)
            e -= p * math.log2(p)
        di = e / 4.0
    # longest_homopolymer_run :149-168
    if n == 0:
        lg = 0
    else:
        lg, cur = 1, 1
        for i in range(1, n):
            if s[i] == s[i - 1]:
                cur += 1
                lg = max(lg, cur)
            else:
                cur = 1
    # dust_score :171-200 (window 64)
    w = 64
    if n < w:
        dust = 0.0
    else:
        tot = 0.0
        for i in range(n - w + 1):
            win = s[i:i + w]
            tc = {}
            for j in range(w - 2):
                tc[win[j:j + 3]] = tc.get(win[j:j + 3], 0) + 1
            ws = 0.0
            for c in tc.values():
                if c > 1:
                    ws += (c * (c - 1)) / 2.0
            tot += ws
        dust = tot / (n - w + 1)
    if n == 0:
        comb = float("nan")
    else:
        comb = (0.25 * sh + 0.25 * ling + 0.15 * (1.0 - homo) + 0.15 * di
                + 0.10 * (1.0 - (lg / n)) + 0.10 * (1.0 - min(dust, 1.0)))
    return {"shannon_entropy": sh, "linguistic_complexity": ling, "homopolymer_fraction": homo,
            "dinucleotide_entropy": di, "longest_homopolymer_run": lg, "dust_score": dust,
            "combined_score": comb}


def py_hamming(s: bytes, target: bytes) -> int:
    """expressions.rs:1054-1069: byte-length check, then chars().zip()."""
    if len(s) != len(target):
        return 0xFFFFFFFF
    a = s.decode("utf-8")
    b = target.decode("utf-8")
    return sum(1 for x, y in zip(a, b) if x != y)


def py_cluster_bruteforce(items: Sequence[Optional[bytes]], umi_len: int = 0, max_distance: int = 1):
    """H3 spec by brute force: O(d^2) pairwise H2 distances between distinct UMIs."""
    L = umi_len
    if L <= 0:
        L = next((len(x) for x in items if x is not None), 0)
    regular = sorted({x for x in items if x is not None and len(x) == L and L >= 1
                      and all(c in b"ACGT" for c in x)})
    irregular = sorted({x for x in items if x is not None and x not in set(regular)})
    parent = list(range(len(regular)))

    def find(x):
        while parent[x] != x:
            x = parent[x]
        return x

    if max_distance == 1:
        for i in range(len(regular)):
            for j in range(i):
                if sum(1 for a, b in zip(regular[i], regular[j]) if a != b) <= 1:
                    ri, rj = find(i), find(j)
                    if ri != rj:
                        parent[max(ri, rj)] = min(ri, rj)
    roots = sorted({find(i) for i in range(len(regular))})
    rank = {r: k for k, r in enumerate(roots)}
    reg_id = {u: rank[find(i)] for i, u in enumerate(regular)}
    irr_id = {u: len(roots) + k for k, u in enumerate(irregular)}
    out = []
    for x in items:
        if x is None:
            out.append(None)
        elif x in reg_id:
            out.append(reg_id[x])
        else:
            out.append(irr_id[x])
    return out, len(roots) + len(irregular)
