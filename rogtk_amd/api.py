"""Host-side mirror of rogtk's UMI/Hamming expression API, backed by librogtk_hip.

Reference surface (rogtk/__init__.py) and what each call here replaces:

================================================  ==========================================
reference                                          rogtk_amd
================================================  ==========================================
``pl.col(c).umi.complexity_all()`` (:417)          ``col(c).umi.complexity_all()``
``.umi.all_scores()`` (:426)                       ``col(c).umi.all_scores()``
``.umi.shannon_entropy()`` … ``.dust_score()``     ``col(c).umi.<same name>()``
(:430-491)
``umi_complexity_scores(expr)`` (:493)             ``umi_complexity_scores(c)``
``pl.col(c).hamming.distance(target)`` (:331)      ``col(c).hamming.distance(target)``
``pl.col(c).hamming.within(target, 1)`` (:341)     ``col(c).hamming.within(target, 1)``
``df.group_by('umi')`` (caller, :206-214)          ``umi_cluster(c, max_distance=0|1)``
k-mer front end of ``assemble_sequences*`` per     ``kmer_spectrum(c, k, min_coverage,
group (fracture.rs:105-256, debruijn                auto_k, group_offsets)``
filter_kmers)
================================================  ==========================================

polars is not part of this build's image, so an "expression" is evaluated eagerly
on an Arrow column (any pyarrow string array / chunked array, a list of
str/None, or a numpy bytes array). Results are pyarrow arrays with the
reference's dtypes, field names and null propagation (null in -> null out):
Struct{shannon_entropy f64, linguistic_complexity f64, homopolymer_fraction f64,
dinucleotide_entropy f64, longest_homopolymer_run u32, dust_score f64,
combined_score f64} (src/expressions.rs:1219-1232), UInt32 (hamming distance,
u32::MAX on byte-length mismatch) and Boolean (within).

All computation runs in librogtk_hip.so on the GPU; errors are RogtkError.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Union

import numpy as np
import pyarrow as pa

from . import _lib
from .columns import ColumnLike, chunks, concat, validity_buffer

FIELDS = (
    ("shannon_entropy", pa.float64()),
    ("linguistic_complexity", pa.float64()),
    ("homopolymer_fraction", pa.float64()),
    ("dinucleotide_entropy", pa.float64()),
    ("longest_homopolymer_run", pa.uint32()),
    ("dust_score", pa.float64()),
    ("combined_score", pa.float64()),
)
_FIELD_NAMES = tuple(f for f, _ in FIELDS)
STRUCT_TYPE = pa.struct([pa.field(n, t) for n, t in FIELDS])


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


class _PinnedBlock:
    """A rogtk_host_alloc block (pinned host memory: direct DMA for the D2H of results),
    returned to the library's cache when the last array over it is collected."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        _lib.call("rogtk_host_alloc", nbytes, ctypes.byref(p))
        self.ptr, self.nbytes = p.value, nbytes

    def __del__(self):
        try:
            _lib.hip().rogtk_host_free(ctypes.c_void_p(self.ptr))
        except Exception:
            pass


def _out(n: int, dtype, zero: bool = False) -> np.ndarray:
    """Output array of n elements in pinned host memory (numpy views keep it alive)."""
    nbytes = max(n, 1) * np.dtype(dtype).itemsize
    blk = _PinnedBlock(nbytes)
    a = np.frombuffer(pa.foreign_buffer(blk.ptr, nbytes, base=blk), dtype=dtype)
    if zero:
        a[:] = 0
    return a


def _complexity_chunk(ch, want: tuple):
    n = ch.n
    out = {}
    for name, typ in FIELDS:
        if name in want:
            out[name] = _out(n, np.uint32 if name == "longest_homopolymer_run" else np.float64)
    sc = _lib.UmiScores(*[_ptr(out.get(name)) for name in _FIELD_NAMES])
    o, v, val = ch.ptrs()
    _lib.call("rogtk_umi_complexity_host", o, ch.offset_width, v, ch.values.size, val,
              ch.validity_offset, n, ctypes.byref(sc))
    return {k: a[:n] for k, a in out.items()}


def _field_array(name, typ, values, vbuf, n):
    return pa.Array.from_buffers(typ, n, [vbuf, pa.py_buffer(np.ascontiguousarray(values))])


def umi_complexity(column: ColumnLike, fields=_FIELD_NAMES):
    """All (or the selected) complexity fields. Returns {name: pa.Array}."""
    want = tuple(fields)
    parts = {name: [] for name in want}
    for ch in chunks(column):
        res = _complexity_chunk(ch, want)
        vbuf = validity_buffer(ch)
        for name, typ in FIELDS:
            if name in want:
                parts[name].append(_field_array(name, typ, res[name], vbuf, ch.n))
    return {name: concat(parts[name], dict(FIELDS)[name]) for name in want}


def umi_complexity_scores(column: ColumnLike) -> Union[pa.StructArray, pa.ChunkedArray]:
    """umi_complexity_all_expr (src/expressions.rs:1234-1284) as a StructArray."""
    arrays = []
    for ch in chunks(column):
        res = _complexity_chunk(ch, _FIELD_NAMES)
        vbuf = validity_buffer(ch)
        children = [_field_array(name, typ, res[name], vbuf, ch.n) for name, typ in FIELDS]
        # df.into_struct (expressions.rs:1283): struct rows stay valid, a null UMI gives
        # a row whose seven fields are null (:1258-1266)
        arrays.append(pa.StructArray.from_arrays(children, fields=list(STRUCT_TYPE)))
    return concat(arrays, STRUCT_TYPE)


def hamming_distance(column: ColumnLike, target: Union[str, bytes]):
    """hamming_distance_expr (src/expressions.rs:1048-1073): UInt32, u32::MAX on length mismatch."""
    return _hamming(column, target, None, want_dist=True)


def hamming_within(column: ColumnLike, target: Union[str, bytes], max_distance: int = 1):
    """hamming_within_expr (src/expressions.rs:1075-1101): Boolean, default max_distance 1."""
    return _hamming(column, target, max_distance, want_dist=False)


def _hamming(column, target, max_distance, want_dist):
    if target is None:
        raise TypeError("target is required")  # HammingKwargs.target: String (expressions.rs:1018)
    t = target.encode("utf-8") if isinstance(target, str) else bytes(target)
    tb = np.frombuffer(t, dtype=np.uint8) if t else np.zeros(1, np.uint8)
    maxd = 1 if max_distance is None else int(max_distance)
    if maxd < 0 or maxd > 0xFFFFFFFF:
        raise ValueError("max_distance must fit in u32")
    arrays = []
    for ch in chunks(column):
        n = ch.n
        dist = _out(n, np.uint32) if want_dist else None
        bits = None if want_dist else _out((n + 7) // 8, np.uint8)
        o, v, val = ch.ptrs()
        _lib.call("rogtk_hamming_host", o, ch.offset_width, v, ch.values.size, val, ch.validity_offset,
                  n, _ptr(tb), len(t), maxd, _ptr(dist), _ptr(bits))
        vbuf = validity_buffer(ch)
        if want_dist:
            arrays.append(pa.Array.from_buffers(pa.uint32(), n, [vbuf, pa.py_buffer(dist)]))
        else:
            arrays.append(pa.Array.from_buffers(pa.bool_(), n, [vbuf, pa.py_buffer(bits)]))
    return concat(arrays, pa.uint32() if want_dist else pa.bool_())


def umi_cluster(column: ColumnLike, umi_len: int = 0, max_distance: int = 1):
    """H3 cluster id per row: dense ids, exact (0) or Hamming<=1 components (1).

    Returns (pa.UInt32Array with nulls for null rows, n_clusters, resolved umi_len).
    A multi-chunk column is clustered as one batch (ids are global to the column).
    """
    arr = column
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks else pa.array([], type=arr.type)
    chs = list(chunks(arr))
    assert len(chs) == 1
    ch = chs[0]
    n = ch.n
    cid = _out(n, np.uint32)
    nclu = ctypes.c_int64(0)
    rl = ctypes.c_int(0)
    o, v, val = ch.ptrs()
    _lib.call("rogtk_umi_cluster_host", o, ch.offset_width, v, ch.values.size, val, ch.validity_offset,
              n, int(umi_len), int(max_distance), _ptr(cid), ctypes.byref(nclu), ctypes.byref(rl))
    out = pa.Array.from_buffers(pa.uint32(), n, [validity_buffer(ch), pa.py_buffer(cid)])
    return out, int(nclu.value), int(rl.value)


KMER_STATS = ("k_eff", "n_sequences", "node_count", "terminal_count", "isolated_count")


def kmer_spectrum(column: ColumnLike, k: int, min_coverage: int, auto_k: bool = False, group_offsets=None):
    """H4: k-mer spectra of read groups (include/rogtk_hip.h, rogtk_kmer_spectrum_host).

    ``group_offsets`` (n_groups + 1 row offsets, contiguous groups; None = one group)
    plays the role of polars' group_by: each group is what one call of the
    reference's assemble_sequences_expr sees. Returns a dict of numpy arrays:
    kmer_hi / kmer_lo (u64; hi only for k_eff 64), exts (u8), counts (u16),
    entry_offsets (n_groups + 1) and stats (n_groups x 5, columns KMER_STATS).
    """
    arr = column
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks else pa.array([], type=arr.type)
    chs = list(chunks(arr))
    assert len(chs) == 1
    ch = chs[0]
    n = ch.n
    o, v, val = ch.ptrs()
    cap = ctypes.c_int64(0)
    _lib.call("rogtk_kmer_capacity", o, ch.offset_width, n, ctypes.byref(cap))
    capn = max(int(cap.value), 1)
    go = None if group_offsets is None else np.ascontiguousarray(group_offsets, dtype=np.int64)
    G = 1 if go is None else len(go) - 1
    km = np.empty(2 * capn, dtype=np.uint64)
    ex = np.empty(capn, dtype=np.uint8)
    cn = np.empty(capn, dtype=np.uint16)
    eo = np.empty(G + 1, dtype=np.int64)
    st = np.empty(5 * G, dtype=np.int64)
    _lib.call("rogtk_kmer_spectrum_host", o, ch.offset_width, v, ch.values.size, val, ch.validity_offset, n,
              _ptr(go), 0 if go is None else G, int(k), int(bool(auto_k)), int(min_coverage), capn,
              _ptr(km), _ptr(ex), _ptr(cn), _ptr(eo), _ptr(st))
    m = int(eo[G])
    return {"kmer_hi": km[0:2 * m:2].copy(), "kmer_lo": km[1:2 * m:2].copy(), "exts": ex[:m].copy(),
            "counts": cn[:m].copy(), "entry_offsets": eo, "stats": st.reshape(G, 5)}


# ------------------------------------------------------------ namespaces
class UmiNamespace:
    """rogtk/__init__.py:412-491 (`pl.col(..).umi.*`)."""

    def __init__(self, column: ColumnLike):
        self._c = column

    def complexity_all(self):
        return umi_complexity_scores(self._c)

    def all_scores(self):
        return self.complexity_all()

    def _one(self, name):
        return umi_complexity(self._c, (name,))[name]

    def shannon_entropy(self):
        return self._one("shannon_entropy")

    def linguistic_complexity(self):
        return self._one("linguistic_complexity")

    def homopolymer_fraction(self):
        return self._one("homopolymer_fraction")

    def dinucleotide_entropy(self):
        return self._one("dinucleotide_entropy")

    def combined_score(self):
        return self._one("combined_score")

    def longest_homopolymer_run(self):
        return self._one("longest_homopolymer_run")

    def dust_score(self):
        return self._one("dust_score")

    def cluster(self, umi_len: int = 0, max_distance: int = 1):
        """Extension (no reference counterpart): H3 cluster ids."""
        return umi_cluster(self._c, umi_len, max_distance)[0]


class HammingExpr:
    """rogtk/__init__.py:326-349 (`pl.col(..).hamming.*`)."""

    def __init__(self, column: ColumnLike):
        self._c = column

    def distance(self, target: str):
        return hamming_distance(self._c, target)

    def within(self, target: str, max_distance: int = 1):
        return hamming_within(self._c, target, max_distance)


class Col:
    """Eager stand-in for a polars expression over one string column."""

    def __init__(self, column: ColumnLike):
        self.column = column
        self.umi = UmiNamespace(column)
        self.hamming = HammingExpr(column)
        from .strings import CigarNamespace, DnaNamespace

        self.dna = DnaNamespace(column)
        self.cigar = CigarNamespace(column)


def col(column: ColumnLike) -> Col:
    return Col(column)
