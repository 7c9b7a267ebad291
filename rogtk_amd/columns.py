"""Arrow string columns as the C ABI sees them (offsets, values, validity).

The reference receives polars String series (possibly multi-chunk) through the
polars plugin ABI (src/expressions.rs:1236 `inputs[0].str()?`). Here a column is
any of: pyarrow (Large)StringArray / ChunkedArray, a Python sequence of
str/bytes/None, or a numpy fixed-width bytes array ('S<L>'). Each chunk is handed
to librogtk_hip as plain host buffers with offsets rebased to 0.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Iterator, Optional, Sequence, Union

import numpy as np
import pyarrow as pa

ColumnLike = Union[pa.Array, pa.ChunkedArray, Sequence[Optional[Union[str, bytes]]], np.ndarray]


@dataclass
class HostChunk:
    """One Arrow string chunk as contiguous host buffers (offsets start at 0)."""

    offsets: np.ndarray           # int32 or int64, n+1
    values: np.ndarray            # uint8
    validity: Optional[np.ndarray]  # uint8 bitmap (LSB order) or None
    validity_offset: int
    n: int
    arrow: pa.Array               # the source chunk (for its validity buffer / name)

    @property
    def offset_width(self) -> int:
        return self.offsets.dtype.itemsize

    def ptrs(self):
        vp = lambda a: None if a is None else ctypes.c_void_p(a.ctypes.data)
        return vp(self.offsets), vp(self.values), vp(self.validity)


def _to_arrow(col: ColumnLike) -> Union[pa.Array, pa.ChunkedArray]:
    if isinstance(col, (pa.Array, pa.ChunkedArray)):
        t = col.type
        if pa.types.is_string(t) or pa.types.is_large_string(t):
            return col
        if pa.types.is_binary(t) or pa.types.is_large_binary(t):
            return col
        if pa.types.is_string_view(t):
            return col.cast(pa.large_string())
        raise TypeError(f"expected a string column, got {t}")
    if isinstance(col, np.ndarray):
        if col.dtype.kind == "S":
            return pa.array(list(col), type=pa.large_binary())
        if col.dtype.kind in ("U", "O"):
            return pa.array(list(col), type=pa.large_string())
        raise TypeError(f"expected bytes/str numpy array, got {col.dtype}")
    items = list(col)
    if any(isinstance(x, (bytes, bytearray)) for x in items):
        return pa.array([None if x is None else bytes(x) for x in items], type=pa.large_binary())
    return pa.array(items, type=pa.large_string())


def chunks(col: ColumnLike) -> Iterator[HostChunk]:
    arr = _to_arrow(col)
    parts = arr.chunks if isinstance(arr, pa.ChunkedArray) else [arr]
    for a in parts:
        yield _chunk(a)


def _chunk(a: pa.Array) -> HostChunk:
    n = len(a)
    bufs = a.buffers()
    validity_buf, offsets_buf, values_buf = bufs[0], bufs[1], bufs[2]
    wide = pa.types.is_large_string(a.type) or pa.types.is_large_binary(a.type)
    odt = np.int64 if wide else np.int32
    offs = np.frombuffer(offsets_buf, dtype=odt, count=a.offset + n + 1)[a.offset:]
    base = int(offs[0]) if n + 1 > 0 else 0
    end = int(offs[-1])
    if values_buf is not None and end > base:
        values = np.frombuffer(values_buf, dtype=np.uint8, count=end)[base:end]
    else:
        values = np.zeros(1, dtype=np.uint8)
    offs = np.ascontiguousarray(offs - base, dtype=odt) if base else np.ascontiguousarray(offs)
    validity = None
    voff = 0
    if a.null_count > 0 and validity_buf is not None:
        validity = np.frombuffer(validity_buf, dtype=np.uint8)
        voff = a.offset
    return HostChunk(offs, np.ascontiguousarray(values), validity, voff, n, a)


def validity_buffer(chunk: HostChunk) -> Optional[pa.Buffer]:
    """Validity bitmap for an output of `chunk` (null in -> null out), offset 0."""
    if chunk.validity is None:
        return None
    bits = np.unpackbits(chunk.validity, bitorder="little")[chunk.validity_offset:chunk.validity_offset + chunk.n]
    return pa.py_buffer(np.packbits(bits, bitorder="little"))


def concat(arrays, typ):
    if not arrays:
        return pa.array([], type=typ)
    if len(arrays) == 1:
        return arrays[0]
    return pa.chunked_array(arrays, type=typ)
