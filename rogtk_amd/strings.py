"""Element-wise DNA / CIGAR / PHRED string expressions on the GPU.

Mirrors the reference's Python surface (rogtk/__init__.py) on pyarrow columns:

    rogtk/__init__.py:57-69     DnaNamespace.reverse_complement  -> reverse_complement_series
    rogtk/__init__.py:72-80     parse_cigar(expr, block_dels)    -> parse_cigar_series
    rogtk/__init__.py:82-90     phred_to_numeric_str(expr, base) -> phred_to_numeric_series_str
    src/expressions.rs:598-630  phred_to_numeric_series (List[u8]; not registered in Python)
    rogtk/__init__.py:532-658   CigarNamespace.enrich_insertions / align_to_ref / align_to_query
    rogtk/__init__.py:661-696   extract_cigar_insertions(seq_col, cigar_col)

Every call runs rogtk_str_transform_host (rogtk_amd/csrc/strings.hip): a measuring
and a filling kernel over the rows, thread per row. There is no CPU path.
"""
from __future__ import annotations

import ctypes
from typing import List

import numpy as np
import pyarrow as pa

from . import _lib
from .columns import ColumnLike, _to_arrow

REVCOMP, PARSE_CIGAR, ALIGNED_REF, ALIGNED_QUERY, CIGAR_INSERTIONS, ENRICH_ALLELE, PHRED_STR, PHRED_LIST = range(1, 9)


def _single(col: ColumnLike) -> pa.Array:
    a = _to_arrow(col)
    if isinstance(a, pa.ChunkedArray):
        a = a.combine_chunks() if a.num_chunks != 1 else a.chunk(0)
    return a


def _desc(a: pa.Array, keep: list) -> _lib.StrCol:
    bufs = a.buffers()
    wide = pa.types.is_large_string(a.type) or pa.types.is_large_binary(a.type)
    odt = np.int64 if wide else np.int32
    n = len(a)
    offs = np.frombuffer(bufs[1], dtype=odt, count=a.offset + n + 1)[a.offset:] if bufs[1] is not None \
        else np.zeros(n + 1, dtype=odt)
    offs = np.ascontiguousarray(offs)
    vals = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None and bufs[2].size else np.zeros(1, np.uint8)
    valid = np.frombuffer(bufs[0], dtype=np.uint8) if a.null_count > 0 and bufs[0] is not None else None
    keep.extend([offs, vals, valid])
    return _lib.StrCol(offs.ctypes.data, odt().itemsize, vals.ctypes.data, vals.size,
                       None if valid is None else valid.ctypes.data, a.offset if valid is not None else 0, n)


def _transform(op: int, cols: List[ColumnLike], param: int = 0):
    """Rows of the output: the reference zips its inputs (the shortest wins); the aligned
    expressions broadcast a 1-row reference next to a longer query column
    (expressions.rs:344-349)."""
    arrays = [_single(c) for c in cols]
    lens = [len(a) for a in arrays]
    scalar_ref = op in (ALIGNED_REF, ALIGNED_QUERY) and lens[0] == 1 and lens[1] > 1
    n = min(lens[1:]) if scalar_ref else min(lens)
    arrays = [a if (scalar_ref and i == 0) else a.slice(0, n) for i, a in enumerate(arrays)]
    keep: list = []
    descs = (_lib.StrCol * len(arrays))(*[_desc(a, keep) for a in arrays])
    res = _lib.StrResult()
    lib = _lib.hip()
    _lib.check(lib.rogtk_str_transform_host(op, descs, len(arrays), n, int(param), ctypes.byref(res)))
    try:
        offs = np.ctypeslib.as_array(ctypes.cast(res.offsets, ctypes.POINTER(ctypes.c_int64)), (n + 1,)).copy()
        vals = np.ctypeslib.as_array(ctypes.cast(res.values, ctypes.POINTER(ctypes.c_uint8)),
                                     (max(res.values_len, 1),))[:res.values_len].copy()
        nbytes = max((n + 63) // 64 * 8, 8)
        bits = np.ctypeslib.as_array(ctypes.cast(res.validity, ctypes.POINTER(ctypes.c_uint8)), (nbytes,)).copy()
        nulls = int(res.null_count)
    finally:
        lib.rogtk_str_result_free(ctypes.byref(res))
    return n, offs, vals, bits, nulls


def _string_array(n, offs, vals, bits, nulls) -> pa.Array:
    vb = pa.py_buffer(bits) if nulls else None
    return pa.Array.from_buffers(pa.large_string(), n, [vb, pa.py_buffer(offs), pa.py_buffer(vals)], null_count=nulls)


def reverse_complement(column: ColumnLike) -> pa.Array:
    """reverse_complement_series (expressions.rs:957-977): chars reversed, A<->T, C<->G."""
    return _string_array(*_transform(REVCOMP, [column]))


def parse_cigar(column: ColumnLike, block_dels: bool = False) -> pa.Array:
    """parse_cigar_series (expressions.rs:450-505): "D,pos,len|I,pos,len|..."."""
    return _string_array(*_transform(PARSE_CIGAR, [column], int(bool(block_dels))))


def phred_to_numeric_str(column: ColumnLike, base: int = 33) -> pa.Array:
    """phred_to_numeric_series_str (expressions.rs:632-665): "q1|q2|..."."""
    return _string_array(*_transform(PHRED_STR, [column], base))


def phred_to_numeric(column: ColumnLike, base: int = 33) -> pa.Array:
    """phred_to_numeric_series (expressions.rs:598-630): List[UInt8]; rows of null
    strings are skipped by the reference's `for_each`, so the output is shorter."""
    n, offs, vals, bits, nulls = _transform(PHRED_LIST, [column], base)
    keep = np.unpackbits(bits, bitorder="little")[:n].astype(bool)
    lens = np.diff(offs)[keep]
    starts = offs[:-1][keep]
    idx = np.concatenate([np.arange(s, s + l) for s, l in zip(starts, lens)]) if len(lens) else np.zeros(0, np.int64)
    loffs = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=loffs[1:])
    return pa.LargeListArray.from_arrays(pa.array(loffs), pa.array(vals[idx.astype(np.int64)], type=pa.uint8()))


def extract_cigar_insertions(seq_col: ColumnLike, cigar_col: ColumnLike) -> pa.Array:
    """extract_cigar_insertions_expr (expressions.rs:207-251): "pos:SEQ|..." sorted by pos."""
    return _string_array(*_transform(CIGAR_INSERTIONS, [seq_col, cigar_col]))


class DnaNamespace:
    """rogtk/__init__.py:57-69 (`pl.col(..).dna.*`)."""

    def __init__(self, column: ColumnLike):
        self._c = column

    def reverse_complement(self):
        return reverse_complement(self._c)


class CigarNamespace:
    """rogtk/__init__.py:532-658 (`pl.col(..).cigar.*`); the column is the allele (enrich)
    or the reference sequence (align_to_*), which may be a 1-row scalar."""

    def __init__(self, column: ColumnLike):
        self._c = column

    def enrich_insertions(self, seq_col: ColumnLike, cigar_col: ColumnLike):
        """enrich_allele_insertions_expr (expressions.rs:172-205): [pos:NI] -> [pos:NI:SEQ]."""
        return _string_array(*_transform(ENRICH_ALLELE, [self._c, seq_col, cigar_col]))

    def align_to_ref(self, query_col: ColumnLike, cigar_col: ColumnLike):
        """cigar_aligned_ref_expr (expressions.rs:338-394)."""
        return _string_array(*_transform(ALIGNED_REF, [self._c, query_col, cigar_col]))

    def align_to_query(self, query_col: ColumnLike, cigar_col: ColumnLike):
        """cigar_aligned_query_expr (expressions.rs:396-444)."""
        return _string_array(*_transform(ALIGNED_QUERY, [self._c, query_col, cigar_col]))
