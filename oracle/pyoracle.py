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
    srcs = [os.path.join(_HERE, f) for f in ("rogtk_oracle.cpp", "kmer_oracle.cpp")]
    if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < max(map(os.path.getmtime, srcs)):
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
        L.oracle_umi_cluster_mt.argtypes = [vp, i32, vp, vp, i64, i64, i32, i32, vp, vp, vp, i32]
        L.oracle_umi_cluster_mt.restype = i64
        L.oracle_plogp.argtypes = [u32, u32]
        L.oracle_plogp.restype = ctypes.c_double
        L.oracle_version.restype = ctypes.c_char_p
        L.oracle_kmer_spectrum.argtypes = [vp, i32, vp, vp, i64, i64, i64, i32, i32, i64, vp, vp, vp, i64, vp]
        L.oracle_kmer_spectrum.restype = i64
        L.oracle_kmer_observations.argtypes = [vp, i32, i64, i64, i32]
        L.oracle_kmer_observations.restype = i64
        L.oracle_bam_digest.argtypes = [ctypes.c_char_p, i32, vp]
        L.oracle_bam_digest.restype = i64
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


def umi_complexity(col: StrCol, dinuc_order: int = 0, threads: int = 1) -> dict:
    """Oracle H1 over a column. Returns dict field -> numpy array (+ 'valid'). threads > 1
    runs row ranges on host threads (the C loop is per row; identical results)."""
    L = lib()
    n = col.n
    out = {f: np.zeros(n, dtype=np.uint32 if f == "longest_homopolymer_run" else np.float64) for f in FIELDS}
    o, v, val = col._ptrs()

    def run(a, b):
        at = lambda arr: ctypes.c_void_p(arr.ctypes.data + a * arr.itemsize)
        L.oracle_umi_complexity_batch(ctypes.c_void_p(col.offsets.ctypes.data + 8 * a), 8, v, val, a, b - a,
                                      dinuc_order, at(out["shannon_entropy"]), at(out["linguistic_complexity"]),
                                      at(out["homopolymer_fraction"]), at(out["dinucleotide_entropy"]),
                                      at(out["longest_homopolymer_run"]), at(out["dust_score"]),
                                      at(out["combined_score"]))

    if threads <= 1 or n < 1 << 16:
        run(0, n)
    else:
        from concurrent.futures import ThreadPoolExecutor
        cuts = np.linspace(0, n, threads + 1).astype(np.int64)
        with ThreadPoolExecutor(threads) as ex:
            for f in [ex.submit(run, int(cuts[i]), int(cuts[i + 1])) for i in range(threads)]:
                f.result()
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


def umi_cluster(col: StrCol, umi_len: int = 0, max_distance: int = 1, threads: int = 1):
    """Oracle H3. Returns (cluster_id u32, valid bool, n_clusters, resolved L). threads > 1
    splits the row passes and the edge search over host threads (identical result)."""
    L = lib()
    cid = np.zeros(col.n, dtype=np.uint32)
    valid = np.zeros(col.n, dtype=np.uint8)
    rl = ctypes.c_int(0)
    o, v, val = col._ptrs()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    k = L.oracle_umi_cluster_mt(o, 8, v, val, 0, col.n, umi_len, max_distance, vp(cid), vp(valid),
                                ctypes.byref(rl), int(threads))
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
    """H3 spec by brute force: O(d^2) pairwise H2 distances
    (expressions.rs:1054-1069: equal byte length, then mismatching bytes) between ALL
    distinct non-null strings, regular or not. Ids: components holding a regular UMI
    (byte length umi_len <= 32, pure ACGT) first, by smallest regular string; then the
    rest by smallest string (byte-lexicographic)."""
    L = umi_len
    if L <= 0:
        L = next((len(x) for x in items if x is not None), 0)

    def is_regular(x):
        return 1 <= L <= 32 and len(x) == L and all(c in b"ACGT" for c in x)

    distinct = {bytes(x) for x in items if x is not None}
    # vertex order: regular strings (lexicographic = code order), then the others
    verts = sorted(x for x in distinct if is_regular(x)) + sorted(x for x in distinct if not is_regular(x))
    parent = list(range(len(verts)))

    def find(x):
        while parent[x] != x:
            x = parent[x]
        return x

    if max_distance == 1:
        for i in range(len(verts)):
            for j in range(i):
                a, b = verts[i], verts[j]
                if len(a) == len(b) and sum(1 for x, y in zip(a, b) if x != y) <= 1:
                    ri, rj = find(i), find(j)
                    if ri != rj:
                        parent[max(ri, rj)] = min(ri, rj)
    roots = sorted({find(i) for i in range(len(verts))})
    rank = {r: k for k, r in enumerate(roots)}
    vid = {u: rank[find(i)] for i, u in enumerate(verts)}
    out = [None if x is None else vid[bytes(x)] for x in items]
    return out, len(roots)


# --------------------------------------------------------------------------
# H4: k-mer spectra of read groups (oracle/kmer_oracle.cpp)
# --------------------------------------------------------------------------
def effective_k(k: int) -> int:
    """fracture.rs:246-256: Kmer4 / Kmer8 / Kmer16 / Kmer32 / Kmer64."""
    return 4 if k <= 4 else 8 if k <= 8 else 16 if k <= 16 else 32 if k <= 32 else 64


def kmer_spectrum(col: StrCol, k: int, min_cov: int, auto_k: bool = False, group_offsets=None, threads: int = 1):
    """Per-group spectra, concatenated in group order. Returns a dict with
    kmer_hi, kmer_lo (u64), exts (u8), counts (u16), group_offsets (n_groups+1, int64)
    and stats (n_groups x 5: k_eff, n_sequences, node_count, terminal_count, isolated_count).
    threads > 1: groups split over host threads (the C calls release the GIL)."""
    L = lib()
    go = np.array([0, col.n], dtype=np.int64) if group_offsets is None else np.asarray(group_offsets, np.int64)
    G = len(go) - 1
    offs, vals, valid = col._ptrs()
    stats = np.zeros((G, 5), dtype=np.int64)
    counts = np.zeros(G, dtype=np.int64)

    def run(g0, g1):
        his, los, exs, cns = [], [], [], []
        for g in range(g0, g1):
            cap = int(L.oracle_kmer_observations(offs, 8, int(go[g]), int(go[g + 1]), 4)) + 1
            km = np.zeros(2 * cap, dtype=np.uint64)
            ex = np.zeros(cap, dtype=np.uint8)
            cn = np.zeros(cap, dtype=np.uint16)
            st = np.zeros(5, dtype=np.int64)
            m = L.oracle_kmer_spectrum(offs, 8, vals, valid, 0, int(go[g]), int(go[g + 1]), int(k),
                                       int(bool(auto_k)), int(min_cov), km.ctypes.data_as(ctypes.c_void_p),
                                       ex.ctypes.data_as(ctypes.c_void_p), cn.ctypes.data_as(ctypes.c_void_p), cap,
                                       st.ctypes.data_as(ctypes.c_void_p))
            assert m >= 0
            his.append(km[0:2 * m:2])
            los.append(km[1:2 * m:2])
            exs.append(ex[:m])
            cns.append(cn[:m])
            stats[g] = st
            counts[g] = m
        return his, los, exs, cns

    cuts = np.linspace(0, G, max(1, min(threads, G)) + 1).astype(np.int64)
    if len(cuts) > 2:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(len(cuts) - 1) as ex:
            parts = list(ex.map(lambda ab: run(int(ab[0]), int(ab[1])), zip(cuts, cuts[1:])))
    else:
        parts = [run(0, G)]
    his = [a for p in parts for a in p[0]]
    los = [a for p in parts for a in p[1]]
    exs = [a for p in parts for a in p[2]]
    cns = [a for p in parts for a in p[3]]
    out_off = np.zeros(G + 1, dtype=np.int64)
    out_off[1:] = np.cumsum(counts)
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)
    return {"kmer_hi": cat(his, np.uint64), "kmer_lo": cat(los, np.uint64), "exts": cat(exs, np.uint8),
            "counts": cat(cns, np.uint16), "group_offsets": out_off, "stats": stats}


def py_kmer_spectrum(items: Sequence[Optional[bytes]], k: int, min_cov: int, auto_k: bool = False):
    """Independent pure-Python restatement of the same path (small inputs only):
    returns ([(kmer_str, exts, count)] sorted, (k_eff, n_seq, node, terminal, isolated))."""
    raw = [bytes(x) for x in items if x is not None]
    if auto_k:
        lens = [len(x) for x in raw if len(x) > 0]
        if not raw or not lens:
            k = 31
        else:
            mean = sum(lens) / len(lens)
            q = mean / 3.0
            kk = int(q + 0.5) if q >= 0 else -int(-q + 0.5)  # round half away from zero
            kk = 63 if kk == 0 else (kk - 1 if kk % 2 == 0 else kk)
            k = min(max(kk, 11), 63)
    if k > 64:
        return [], (0, 0, 0, 0, 0)
    seqs = []
    for x in raw:
        u = bytes(c - 32 if 97 <= c <= 122 else c for c in x)
        if all(c in b"ACGT" for c in u):
            seqs.append(u.decode())
    K = effective_k(k)
    if not seqs:
        return [], (K, 0, 0, 0, 0)
    obs = {}
    for s in seqs:
        for i in range(len(s) - K + 1):
            km = s[i:i + K]
            e = 0
            if i > 0:
                e |= 1 << "ACGT".index(s[i - 1])
            if i + K < len(s):
                e |= 1 << (4 + "ACGT".index(s[i + K]))
            c, ee = obs.get(km, (0, 0))
            obs[km] = (min(c + 1, 0xFFFF), ee | e)
    valid = {km: v for km, v in obs.items() if v[0] >= min_cov}
    out = []
    term = iso = 0
    for km in sorted(valid):
        c, e = valid[km]
        ne = 0
        for b in range(4):
            if (e >> b) & 1 and ("ACGT"[b] + km[:-1]) in valid:
                ne |= 1 << b
            if (e >> (4 + b)) & 1 and (km[1:] + "ACGT"[b]) in valid:
                ne |= 1 << (4 + b)
        out.append((km, ne, c))
        l0, r0 = (ne & 0xF) == 0, (ne >> 4) == 0
        term += int(l0 or r0)
        iso += int(l0 and r0)
    return out, (K, len(seqs), len(out), term, iso)


def kmer_to_str(hi: int, lo: int, K: int) -> str:
    v = (int(hi) << 64) | int(lo)
    return "".join("ACGT"[(v >> (2 * (K - 1 - i))) & 3] for i in range(K))
