"""Paired FASTQ ingest: librogtk_hip's native gzip reader
(rogtk_amd/csrc/fastq.cpp) restating parse_paired_fastqs (src/lib.rs:232-428).

``iter_paired_fastqs`` yields pyarrow RecordBatches with the reference schema
(read_id, start, end, cbc, umi, cbc_qual, umi_qual, seq, qual; lib.rs:258-268):
the ``umi`` column feeds H1-H3 (umi_complexity_scores, umi_cluster, or
device.stage_strings for the packed SoA) without Python strings.
``parse_paired_fastqs`` is the reference pyfunction: the same batches written to a
SNAPPY Parquet file (lib.rs:270-276), 10M rows per row group.
"""
from __future__ import annotations

import ctypes
from typing import Iterator, Optional

import numpy as np
import pyarrow as pa

from . import _lib

COLUMNS = ("read_id", "start", "end", "cbc", "umi", "cbc_qual", "umi_qual", "seq", "qual")
SCHEMA = pa.schema([pa.field(c, pa.string(), nullable=False) for c in COLUMNS])


def _array(off_ptr, val_ptr, n: int) -> pa.Array:
    offs = np.ctypeslib.as_array(ctypes.cast(off_ptr, ctypes.POINTER(ctypes.c_int64)), shape=(n + 1,)).copy()
    nbytes = int(offs[-1])
    vals = ctypes.string_at(val_ptr, nbytes) if nbytes else b""
    if nbytes < 2 ** 31 - 1:
        return pa.Array.from_buffers(pa.string(), n, [None, pa.py_buffer(offs.astype(np.int32)), pa.py_buffer(vals)])
    return pa.Array.from_buffers(pa.large_string(), n, [None, pa.py_buffer(offs), pa.py_buffer(vals)])


def iter_paired_fastqs(in_fn1: str, in_fn2: str, cbc_len: int, umi_len: int, limit: Optional[int] = None,
                       do_rev_comp: Optional[bool] = None, batch_records: int = 10_000_000) -> Iterator[pa.RecordBatch]:
    lib = _lib.hip()
    h = ctypes.c_void_p()
    _lib.check(lib.rogtk_fastq_pair_open(in_fn1.encode(), in_fn2.encode(), int(cbc_len), int(umi_len),
                                         -1 if limit is None else int(limit), int(bool(do_rev_comp)), ctypes.byref(h)))
    try:
        offs = (ctypes.c_void_p * 9)()
        vals = (ctypes.c_void_p * 9)()
        n = ctypes.c_int64(0)
        while True:
            _lib.check(lib.rogtk_fastq_pair_next(h, int(batch_records), ctypes.byref(n), offs, vals))
            if n.value == 0:
                return
            yield pa.RecordBatch.from_arrays([_array(offs[i], vals[i], n.value) for i in range(9)], schema=SCHEMA)
    finally:
        lib.rogtk_fastq_pair_close(h)


def parse_paired_fastqs(in_fn1: str, in_fn2: str, cbc_len: int, umi_len: int, out_fn: str,
                        limit: Optional[int] = None, do_rev_comp: Optional[bool] = None) -> None:
    """lib.rs:232-428: paired FASTQ -> SNAPPY Parquet with the reference schema."""
    import pyarrow.parquet as pq

    with pq.ParquetWriter(out_fn, SCHEMA, compression="snappy") as w:
        wrote = False
        for b in iter_paired_fastqs(in_fn1, in_fn2, cbc_len, umi_len, limit, do_rev_comp):
            w.write_batch(b)
            wrote = True
        if not wrote:
            w.write_batch(pa.RecordBatch.from_arrays([pa.array([], pa.string())] * 9, schema=SCHEMA))
