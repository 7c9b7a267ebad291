"""BAM -> Arrow conversion with per-record decoding on the GPU.

Host-side mirror of rogtk's BAM converters (src/bam.rs, src/bam_htslib.rs; registered in
src/lib.rs:489-505, re-exported by rogtk/__init__.py:17-56). Every converter writes the
reference's schema (create_bam_schema, bam.rs:3203-3221; + source_file for bams_*,
bam.rs:609-632):

    name Utf8 (non-null), chrom Utf8, start UInt32, end UInt32, flags UInt32 (non-null),
    [sequence Utf8], [quality_scores Utf8], [source_file Utf8 (non-null)]

The per-record semantics come in three flavours, selected by which reference function is
mirrored (include/rogtk_hip.h, ROGTK_BAM_*):

* "noodles" — extract_record_data_enhanced (bam.rs:170-262): bam_to_parquet,
  bams_to_parquet, bam_to_arrow_ipc, bams_to_arrow_ipc, bam_to_arrow_ipc_parallel,
  bam_to_arrow_ipc_gzp_parallel.
* "htslib" — process_htslib_records_to_batch (bam.rs:3028-3148):
  bam_to_arrow_ipc_htslib_{parallel,optimized,mmap_parallel,multi_reader_parallel},
  bams_to_arrow_ipc_htslib_optimized.
* "htslib_blocks" — process_htslib_records_to_batch (bam_htslib.rs:154-241):
  bam_to_arrow_ipc_htslib_bgzf_blocks.

BGZF blocks are inflated on host threads (zlib); framing is one u32 per record; every
field of every record is decoded by GPU kernels (rogtk_amd/csrc/bam.hip). Rows come out
in file order. The reference's threaded writers may emit batches in any order ("no order
preservation", bam.rs:1979-1981); file order is one of its possible outputs. Thread,
buffer and worker knobs of the reference signatures are accepted and do not change
results.
"""
from __future__ import annotations

import ctypes
from concurrent.futures import ThreadPoolExecutor
import os
import time
from typing import Iterator, List, Optional, Sequence

import numpy as np
import pyarrow as pa

from . import _lib

MODES = {"noodles": 0, "htslib": 1, "htslib_blocks": 2}
# records decoded per GPU batch (independent of the output batch_size, which only
# slices the Arrow record batches the way the reference batches its writes)
DECODE_RECORDS = 1 << 20


def bam_schema(include_sequence: bool = True, include_quality: bool = True,
               include_source_file: bool = False) -> pa.Schema:
    """create_bam_schema (bam.rs:3203-3221) / create_bam_schema_with_source (:609-632)."""
    fields = [pa.field("name", pa.string(), nullable=False), pa.field("chrom", pa.string()),
              pa.field("start", pa.uint32()), pa.field("end", pa.uint32()),
              pa.field("flags", pa.uint32(), nullable=False)]
    if include_sequence:
        fields.append(pa.field("sequence", pa.string()))
    if include_quality:
        fields.append(pa.field("quality_scores", pa.string()))
    if include_source_file:
        fields.append(pa.field("source_file", pa.string(), nullable=False))
    return pa.schema(fields)


def _np_from(ptr: int, dtype, count: int) -> np.ndarray:
    if count <= 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    buf = (ctypes.c_char * (count * np.dtype(dtype).itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=count).copy()


def _validity(ptr: int, n: int):
    if not ptr or n == 0:
        return None, 0
    bits = _np_from(ptr, np.uint8, (n + 7) // 8)
    nulls = n - int(np.unpackbits(bits, bitorder="little")[:n].sum())
    return (pa.py_buffer(bits), nulls) if nulls else (None, 0)


def bam_split_points(path: str, n: int) -> List[int]:
    """Compressed offsets [0, b_1, .., file_size] cutting one BAM file into <= n ranges at
    BGZF block starts near file_size * i / n (the reference's discover_split_points,
    src/bam_htslib.rs:247-290; never inside the header's blocks). Host only."""
    pts = (ctypes.c_int64 * (max(int(n), 1) + 1))()
    k = ctypes.c_int()
    _lib.call("rogtk_bam_split_points", os.fsencode(path), max(int(n), 1), pts, ctypes.byref(k))
    return [int(pts[i]) for i in range(k.value + 1)]


def bam_find_record(path: str, c_begin: int) -> int:
    """Bytes to skip in the stream inflated from the block at c_begin before the first
    record that starts in it (chained SAMv1 structural checks). Host only."""
    skip = ctypes.c_int64()
    _lib.call("rogtk_bam_find_record", os.fsencode(path), int(c_begin), ctypes.byref(skip))
    return int(skip.value)


class BamReader:
    """A BAM file open for GPU decoding (rogtk_bam_open / _next / _close); with rng =
    (c_begin, c_end, skip) only the records that start in the blocks [c_begin, c_end)
    (rogtk_bam_open_range)."""

    def __init__(self, path: str, n_threads: int = 0, rng=None):
        self._h = ctypes.c_void_p()
        if rng is None:
            _lib.call("rogtk_bam_open", os.fsencode(path), int(n_threads), ctypes.byref(self._h))
        else:
            c0, c1, skip = rng
            _lib.call("rogtk_bam_open_range", os.fsencode(path), int(n_threads), int(c0), int(c1), int(skip),
                      ctypes.byref(self._h))

    def tail(self) -> int:
        """Bytes of this range's last record past its end (the next range's skip; -1: the
        range ran to the end of the file). Valid once the range is exhausted."""
        t = ctypes.c_int64()
        _lib.call("rogtk_bam_range_tail", self._h, ctypes.byref(t))
        return int(t.value)

    def batch_bytes(self) -> int:
        t = ctypes.c_int64()
        _lib.call("rogtk_bam_batch_bytes", self._h, ctypes.byref(t))
        return int(t.value)

    def check(self, stream) -> None:
        """Device-mode batches: fail if a record overran its block_size (syncs `stream`)."""
        _lib.call("rogtk_bam_check", self._h, ctypes.c_void_p(stream.cuda_stream))

    def close(self) -> None:
        if self._h:
            _lib.call("rogtk_bam_close", self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def timers(self) -> dict:
        """Seconds spent per stage so far (rogtk_bam_timers)."""
        t = (ctypes.c_double * 6)()
        _lib.call("rogtk_bam_timers", self._h, t)
        return dict(zip(("read", "move_frame_blocks", "inflate", "frame_records", "h2d_decode", "d2h"), list(t)))

    def reference_names(self) -> List[str]:
        n = ctypes.c_int64()
        off, val, txt = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        tl = ctypes.c_int64()
        _lib.call("rogtk_bam_header", self._h, ctypes.byref(n), ctypes.byref(off), ctypes.byref(val),
                  ctypes.byref(txt), ctypes.byref(tl))
        o = _np_from(off.value, np.int64, n.value + 1)
        v = _np_from(val.value, np.uint8, int(o[-1]) if len(o) else 0).tobytes()
        return [v[o[i]:o[i + 1]].decode() for i in range(n.value)]

    def next_batch(self, max_records: int, mode: str = "noodles", include_sequence: bool = True,
                   include_quality: bool = True) -> Optional[pa.RecordBatch]:
        """Up to max_records records as a RecordBatch of the reference schema; None at the end."""
        b = _lib.BamBatch()
        n = ctypes.c_int64()
        _lib.call("rogtk_bam_next", self._h, int(max_records), MODES[mode], int(bool(include_sequence)),
                  int(bool(include_quality)), ctypes.byref(n), ctypes.byref(b))
        n = int(n.value)
        if n == 0:
            return None
        cols = []

        def string_col(c):
            off = _np_from(b.offsets[c], np.int64, n + 1)
            vals = _np_from(b.values[c], np.uint8, int(off[-1]))
            vbuf, nulls = _validity(b.validity[c], n)
            if off[-1] < 2 ** 31:
                return pa.Array.from_buffers(pa.string(), n, [vbuf, pa.py_buffer(off.astype(np.int32)),
                                                              pa.py_buffer(vals)], null_count=nulls)
            arr = pa.Array.from_buffers(pa.large_string(), n, [vbuf, pa.py_buffer(off), pa.py_buffer(vals)],
                                        null_count=nulls)
            return arr.cast(pa.string())

        def u32_col(c):
            vals = _np_from(b.u32[c], np.uint32, n)
            vbuf, nulls = _validity(b.u32_validity[c], n)
            return pa.Array.from_buffers(pa.uint32(), n, [vbuf, pa.py_buffer(vals)], null_count=nulls)

        cols = [string_col(0), string_col(1), u32_col(0), u32_col(1), u32_col(2)]
        if include_sequence:
            cols.append(string_col(2))
        if include_quality:
            cols.append(string_col(3))
        return pa.RecordBatch.from_arrays(cols, schema=bam_schema(include_sequence, include_quality))


def iter_bam_batches(bam_path: str, batch_size: int = 50000, include_sequence: bool = True,
                     include_quality: bool = True, mode: str = "noodles", limit: Optional[int] = None,
                     n_threads: int = 0) -> Iterator[pa.RecordBatch]:
    """Record batches of <= batch_size rows (the last one shorter), at most `limit` rows."""
    if not os.path.exists(bam_path):
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, f"BAM file does not exist: {bam_path}")
    if batch_size <= 0:
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, "batch_size must be greater than 0")
    bs = min(int(batch_size), 1_000_000)  # effective_batch_size (bam.rs:306)
    left = None if limit is None else int(limit)
    with BamReader(bam_path, n_threads) as r:
        while left is None or left > 0:
            want = DECODE_RECORDS if left is None else min(DECODE_RECORDS, left)
            rb = r.next_batch(want, mode, include_sequence, include_quality)
            if rb is None:
                break
            if left is not None:
                left -= rb.num_rows
            for a in range(0, rb.num_rows, bs):
                yield rb.slice(a, bs)


def _with_source(rb: pa.RecordBatch, source: str, schema: pa.Schema) -> pa.RecordBatch:
    """add_source_file_column (bam.rs:634-643)."""
    col = _repeat_str(source, rb.num_rows)
    return pa.RecordBatch.from_arrays(list(rb.columns) + [col], schema=schema)


def _convert(paths: Sequence[str], out_path: str, fmt: str, batch_size: int, include_sequence: bool,
             include_quality: bool, limit: Optional[int], mode: str, include_source_file: bool = False,
             compression: str = "snappy") -> None:
    if not paths:
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, "No BAM files provided")
    if batch_size <= 0:
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, "batch_size must be greater than 0")
    for p in paths:
        if not os.path.exists(p):
            raise _lib.RogtkError(_lib.ROGTK_E_INVALID, f"BAM file does not exist: {p}")
    parent = os.path.dirname(out_path)
    if parent:
        os.makedirs(parent, exist_ok=True)
    schema = bam_schema(include_sequence, include_quality, include_source_file)
    if fmt == "ipc":
        writer = pa.ipc.new_file(out_path, schema)
    else:
        import pyarrow.parquet as pq
        writer = pq.ParquetWriter(out_path, schema, compression=_parquet_codec(compression))
    left = None if limit is None else int(limit)
    try:
        for p in paths:
            if left is not None and left <= 0:
                break
            source = os.path.basename(p) or p
            for rb in iter_bam_batches(p, batch_size, include_sequence, include_quality, mode, left):
                if left is not None:
                    left -= rb.num_rows
                if include_source_file:
                    rb = _with_source(rb, source, schema)
                if fmt == "ipc":
                    writer.write_batch(rb)
                else:
                    writer.write_table(pa.Table.from_batches([rb], schema=schema))
    finally:
        writer.close()


def _parquet_codec(compression: str) -> str:
    """parse_compression (bam.rs:3287-3300): unknown names fall back to snappy."""
    c = compression.lower()
    return {"snappy": "snappy", "gzip": "gzip", "lz4": "lz4", "zstd": "zstd", "brotli": "brotli",
            "uncompressed": "none", "none": "none"}.get(c, "snappy")


# ------------------------------------------------- the reference's converters
def bam_to_parquet(bam_path, parquet_path, batch_size=50000, include_sequence=True, include_quality=True,
                   compression="snappy", limit=None):
    """bam.rs:264-416 (noodles record semantics)."""
    _convert([bam_path], parquet_path, "parquet", batch_size, include_sequence, include_quality, limit, "noodles",
             compression=compression)


def bams_to_parquet(bam_paths, parquet_path, batch_size=50000, include_sequence=True, include_quality=True,
                    compression="snappy", limit=None, include_source_file=False):
    """bam.rs:418-607."""
    _convert(list(bam_paths), parquet_path, "parquet", batch_size, include_sequence, include_quality, limit,
             "noodles", include_source_file, compression)


def bam_to_arrow_ipc(bam_path, arrow_ipc_path, batch_size=50000, include_sequence=True, include_quality=True,
                     limit=None):
    """bam.rs:645-787."""
    _convert([bam_path], arrow_ipc_path, "ipc", batch_size, include_sequence, include_quality, limit, "noodles")


def bams_to_arrow_ipc(bam_paths, arrow_ipc_path, batch_size=50000, include_sequence=True, include_quality=True,
                      limit=None, include_source_file=False):
    """bam.rs:789-970."""
    _convert(list(bam_paths), arrow_ipc_path, "ipc", batch_size, include_sequence, include_quality, limit,
             "noodles", include_source_file)


def bam_to_arrow_ipc_parallel(bam_path, arrow_ipc_path, batch_size=50000, include_sequence=True,
                              include_quality=True, num_threads=4, preserve_order=False, limit=None):
    """bam.rs:972-1264."""
    _convert([bam_path], arrow_ipc_path, "ipc", batch_size, include_sequence, include_quality, limit, "noodles")


def bam_to_arrow_ipc_gzp_parallel(bam_path, arrow_ipc_path, batch_size=50000, include_sequence=True,
                                  include_quality=True, decompression_threads=4, processing_threads=2,
                                  preserve_order=False, limit=None):
    """bam.rs:1266-1582."""
    _convert([bam_path], arrow_ipc_path, "ipc", batch_size, include_sequence, include_quality, limit, "noodles")


def bam_to_arrow_ipc_htslib_parallel(bam_path, arrow_ipc_path, batch_size=15000, include_sequence=True,
                                     include_quality=True, bgzf_threads=8, writing_threads=8, read_buffer_mb=1024,
                                     write_buffer_mb=256, limit=None):
    """bam.rs:1584-1843 (htslib record semantics)."""
    _convert([bam_path], arrow_ipc_path, "ipc", batch_size, include_sequence, include_quality, limit, "htslib")


def bam_to_arrow_ipc_htslib_optimized(bam_path, arrow_ipc_path, batch_size=15000, include_sequence=True,
                                      include_quality=True, max_bgzf_threads=16, writing_threads=6,
                                      read_buffer_mb=2048, write_buffer_mb=512, limit=None):
    """bam.rs:1845-2116."""
    _convert([bam_path], arrow_ipc_path, "ipc", batch_size, include_sequence, include_quality, limit, "htslib")


def bams_to_arrow_ipc_htslib_optimized(bam_paths, arrow_ipc_path, batch_size=15000, include_sequence=True,
                                       include_quality=True, max_bgzf_threads=4, writing_threads=6,
                                       read_buffer_mb=2048, write_buffer_mb=128, limit=None,
                                       include_source_file=False):
    """bam.rs:2118-2344."""
    _convert(list(bam_paths), arrow_ipc_path, "ipc", batch_size, include_sequence, include_quality, limit,
             "htslib", include_source_file)


def bam_to_arrow_ipc_htslib_mmap_parallel(bam_path, arrow_ipc_path, batch_size=15000, include_sequence=True,
                                          include_quality=True, num_workers=4, chunk_size_mb=64,
                                          bgzf_threads_per_worker=2, limit=None):
    """bam.rs:2346-2609."""
    _convert([bam_path], arrow_ipc_path, "ipc", batch_size, include_sequence, include_quality, limit, "htslib")


def bam_to_arrow_ipc_htslib_multi_reader_parallel(bam_path, arrow_ipc_path, batch_size=15000,
                                                  include_sequence=True, include_quality=True, num_readers=2,
                                                  bgzf_threads=4, writing_threads=10, read_buffer_mb=1024,
                                                  write_buffer_mb=256, limit=None):
    """bam.rs:2825-3026."""
    _convert([bam_path], arrow_ipc_path, "ipc", batch_size, include_sequence, include_quality, limit, "htslib")


def bam_to_arrow_ipc_htslib_bgzf_blocks(bam_path, arrow_ipc_path, batch_size=20000, include_sequence=True,
                                        include_quality=True, bgzf_threads=4, writing_threads=8,
                                        read_buffer_mb=None, write_buffer_mb=None, limit=None,
                                        num_block_workers=None):
    """bam_htslib.rs:507-... (0-based start, bam_endpos end, IUPAC bases)."""
    _convert([bam_path], arrow_ipc_path, "ipc", batch_size, include_sequence, include_quality, limit,
             "htslib_blocks")


# ------------------------------------------------- config C5: BAM -> UMI clusters
UMI_SOURCES = {"sequence": 0, "name": 1}


def _next_dev(reader: BamReader, max_records: int, mode: str, include_sequence: bool, stream):
    b = _lib.BamBatch()
    n = ctypes.c_int64()
    _lib.call("rogtk_bam_next_dev", reader._h, int(max_records), MODES[mode], int(bool(include_sequence)), 0,
              ctypes.byref(n), ctypes.byref(b), ctypes.c_void_p(stream.cuda_stream))
    return int(n.value), b


class _DevColumn:
    """A growable device string column (int64 offsets, values, validity words) that device
    batches are appended to without host synchronisation (rogtk_bam_umi_append /
    rogtk_bam_append_strings: the running byte count lives on the device; capacities grow
    from host-known bounds, by copies enqueued on the same stream)."""

    def __init__(self, dev, stream, rows: int = 1 << 20, nbytes: int = 1 << 24):
        import torch
        self.dev, self.stream = dev, stream
        self.off = torch.empty(rows + 1, dtype=torch.int64, device=dev)
        self.val = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        self.vw = torch.zeros(rows // 64 + 1, dtype=torch.int64, device=dev)
        self.base = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ovf = torch.zeros(1, dtype=torch.int64, device=dev)
        self.rows = 0
        self.bound = 0  # host-side upper bound of the value bytes used

    def _reserve(self, n: int, nbytes: int) -> None:
        import torch
        rows, bound = self.rows + n, self.bound + nbytes
        if rows + 1 > self.off.numel():
            o = torch.empty(max(2 * self.off.numel(), rows + 1), dtype=torch.int64, device=self.dev)
            o[: self.off.numel()].copy_(self.off)
            self.off = o
        if rows // 64 + 1 > self.vw.numel():
            w = torch.zeros(max(2 * self.vw.numel(), rows // 64 + 1), dtype=torch.int64, device=self.dev)
            w[: self.vw.numel()].copy_(self.vw)
            self.vw = w
        if bound > self.val.numel():
            v = torch.empty(max(2 * self.val.numel(), bound), dtype=torch.uint8, device=self.dev)
            v[: self.val.numel()].copy_(self.val)
            self.val = v

    def append_umi(self, b, n: int, src: int, umi_len: int, sep: str, bound: int) -> None:
        self._reserve(n, bound)
        _lib.call("rogtk_bam_umi_append", ctypes.byref(b), n, src, int(umi_len), ord(sep),
                  ctypes.c_void_p(self.off.data_ptr()), ctypes.c_void_p(self.val.data_ptr()), self.val.numel(),
                  ctypes.c_void_p(self.vw.data_ptr()), self.rows, ctypes.c_void_p(self.base.data_ptr()),
                  ctypes.c_void_p(self.ovf.data_ptr()), ctypes.c_void_p(self.stream.cuda_stream))
        self.rows += n
        self.bound += bound

    def append_strings(self, off_ptr: int, val_ptr: int, n: int, bound: int) -> None:
        self._reserve(n, bound)
        _lib.call("rogtk_bam_append_strings", ctypes.c_void_p(off_ptr), ctypes.c_void_p(val_ptr), n,
                  ctypes.c_void_p(self.off.data_ptr()), ctypes.c_void_p(self.val.data_ptr()), self.val.numel(),
                  self.rows, ctypes.c_void_p(self.base.data_ptr()), ctypes.c_void_p(self.ovf.data_ptr()),
                  ctypes.c_void_p(self.stream.cuda_stream))
        self.rows += n
        self.bound += bound

    def finish(self):
        """(offsets [n + 1], values, validity words, n) on the device: one host sync."""
        import torch
        n = self.rows
        if n == 0:
            z = torch.zeros(1, dtype=torch.int64, device=self.dev)
            return z, torch.zeros(1, dtype=torch.uint8, device=self.dev), torch.zeros(1, dtype=torch.int64,
                                                                                      device=self.dev), 0
        tot, ovf = (int(x) for x in torch.cat([self.base, self.ovf]).cpu().tolist())
        if ovf:
            raise _lib.RogtkError(_lib.ROGTK_E_OVERFLOW, f"bam column: {ovf} rows past the value capacity")
        return self.off[: n + 1], self.val[: max(tot, 1)], self.vw[: (n + 63) // 64], n

    def to_host_strings(self) -> pa.Array:
        off, val, _, n = self.finish()
        o = off.cpu().numpy() if n else np.zeros(1, np.int64)
        v = val.cpu().numpy()[: int(o[-1])] if n else np.zeros(0, np.uint8)
        return pa.Array.from_buffers(pa.large_string(), n, [None, pa.py_buffer(o), pa.py_buffer(v)]).cast(pa.string())


def bam_umis_dev(bam_path: str, umi_len: int = 12, source: str = "sequence", sep: str = "_",
                 mode: str = "htslib", n_threads: int = 0, with_names: bool = False, rng=None,
                 return_tail: bool = False):
    """Decode a BAM file (or the range rng = (c_begin, c_end, skip) of it) on the GPU and
    return its UMI column in HBM (torch tensors: int64 offsets [n + 1], uint8 values, int64
    validity words, n), plus the read names (host pyarrow array) when asked, plus the
    range's tail when asked. UMI = the first umi_len bases of SEQ ("sequence") or the read
    name after its last `sep` byte ("name", UMI-tools READNAME_<UMI>). The host never waits
    for the GPU inside the file: batches are decoded and appended on the current stream
    while the reader inflates the next ones; one sync at the end."""
    import torch

    caller = torch.cuda.current_stream()
    # the decode, the appends and their buffers on one real stream: a NULL (default) stream
    # would make every batch synchronous (rogtk_bam_next_dev), and work on it is not ordered
    # with the reader's own non-blocking stream
    stream = caller if caller.cuda_stream else torch.cuda.Stream()
    stream.wait_stream(caller)
    dev = torch.device("cuda", torch.cuda.current_device())
    src = UMI_SOURCES[source]
    with torch.cuda.stream(stream):
        umi = _DevColumn(dev, stream, nbytes=(1 << 20) * max(int(umi_len), 1))
        names = _DevColumn(dev, stream, nbytes=1 << 26) if with_names else None
        with BamReader(bam_path, n_threads, rng) as r:
            while True:
                n, b = _next_dev(r, DECODE_RECORDS, mode, src == 0, stream)
                if n == 0:
                    break
                raw = r.batch_bytes()
                name_bound = 3 * raw + 7 * n  # lossy UTF-8: <= 3 bytes per byte; "unknown"
                umi.append_umi(b, n, src, umi_len, sep, n * int(umi_len) if src == 0 else name_bound)
                if names is not None:
                    names.append_strings(b.offsets[0], b.values[0], n, name_bound)
            r.check(stream)
            tail = r.tail()
            if os.environ.get("ROGTK_BAM_TIMING") == "1":
                print(f"reader {rng}: {r.timers()}", flush=True)
        out = umi.finish(), (names.to_host_strings() if names is not None else None)
    caller.wait_stream(stream)
    if stream is not caller:  # the column is used on the caller's stream from here on
        for t in out[0][:3]:
            t.record_stream(caller)
    return out + (tail,) if return_tail else out


def _repeat_str(s: str, n: int) -> pa.Array:
    """A string column of n copies of s, built from buffers (round 6: pa.array over a
    Python list of 1M strings cost a fresh process ~0.6 s the first time, most of a rank's
    first bams_umi_cluster call)."""
    b = s.encode()
    big = n * len(b) >= 2 ** 31
    offs = np.arange(n + 1, dtype=np.int64 if big else np.int32) * len(b)
    arr = pa.Array.from_buffers(pa.large_string() if big else pa.string(), n,
                                [None, pa.py_buffer(offs), pa.py_buffer(b * n)])
    return arr.cast(pa.string()) if big else arr


def _concat_dev(offs, vals, valids, counts, dev):
    """The ranges' device UMI columns concatenated in order (rogtk_concat_strings_dev: the
    library's own kernels, no host sync; round 6 - torch's cat and bit kernels cost a fresh
    process ~0.5 s of module loading in its first call)."""
    import torch
    n = sum(counts)
    if n == 0:
        z = torch.zeros(1, dtype=torch.int64, device=dev)
        return z, torch.zeros(1, dtype=torch.uint8, device=dev), torch.zeros(1, dtype=torch.int64, device=dev), 0
    if len(offs) == 1:
        return offs[0], vals[0], valids[0], n
    cap = sum(int(v.numel()) for v in vals)
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    val = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
    vw = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
    scratch = torch.empty(2, dtype=torch.int64, device=dev)  # running byte count, overflow
    k = len(offs)
    P = ctypes.c_void_p * k
    _lib.call("rogtk_concat_strings_dev", k, P(*[o.data_ptr() for o in offs]), P(*[v.data_ptr() for v in vals]),
              P(*[w.data_ptr() for w in valids]), (ctypes.c_int64 * k)(*[int(c) for c in counts]),
              ctypes.c_void_p(off.data_ptr()), ctypes.c_void_p(val.data_ptr()), cap, ctypes.c_void_p(vw.data_ptr()),
              ctypes.c_void_p(scratch.data_ptr()), ctypes.c_void_p(scratch.data_ptr() + 8),
              ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    return off, val, vw, n


def _umi_table(off, val, vw, n, names, cid, n_clusters, extra=None) -> pa.Table:
    o = off.cpu().numpy()
    v = val.cpu().numpy()
    bits = vw.cpu().numpy().view(np.uint8)[: (n + 7) // 8] if n else np.zeros(1, np.uint8)
    valid = np.unpackbits(bits, bitorder="little")[:n].astype(bool)
    vbuf = None if valid.all() else pa.py_buffer(np.packbits(valid, bitorder="little"))
    umi = pa.Array.from_buffers(pa.large_string(), n, [vbuf, pa.py_buffer(o), pa.py_buffer(v)]).cast(pa.string())
    ids = cid[:n].cpu().numpy().view(np.uint32)
    cl = pa.Array.from_buffers(pa.uint32(), n, [vbuf, pa.py_buffer(ids.copy())])
    cols = {"name": names if names is not None else pa.array([], pa.string()), "umi": umi, "cluster_id": cl}
    cols.update(extra or {})
    t = pa.table(cols)
    return t.replace_schema_metadata({"n_clusters": str(int(n_clusters))})


def _umi_ranges(bam_paths: Sequence[str], per_file: int, split: bool):
    """[(file index, range index, c_begin, c_end)]: each file cut into up to `per_file`
    ranges at BGZF block starts (bam_split_points) when split, else whole files."""
    out = []
    for fi, p in enumerate(bam_paths):
        pts = bam_split_points(p, per_file) if split and per_file > 1 else [0, -1]
        out += [(fi, i, pts[i], pts[i + 1]) for i in range(len(pts) - 1)]
    return out


def bams_umi_cluster(bam_paths: Sequence[str], umi_len: int = 12, max_distance: int = 1, source: str = "sequence",
                     sep: str = "_", mode: str = "htslib", n_threads: int = 0, group=None,
                     split: bool = True, ranges_per_file: int = 0) -> pa.Table:
    """Config C5 across ranks (one process per GPU): every file is cut into up to `world`
    ranges at BGZF block starts (split=True; the reference's discover_split_points +
    process_file_segment_with_pool, src/bam_htslib.rs:247-420), range j of the list goes to
    rank j % world and is decoded on its GPU, and the ranks merge their UMI clusters with
    the all-to-all H3 (rogtk_amd.dist.umi_cluster_sharded). A range after the first starts
    at the first record that starts in its blocks: the rank finds it by chained record
    checks, then every rank's guess is compared with the previous range's exact tail (one
    all-reduce) and a range whose guess was wrong is decoded again from the tail, so the
    rows are exactly the file's records whatever the guesses. Returns this rank's rows
    {name, umi, cluster_id, source} in range order: ids are those of umi_cluster over all
    files' UMIs together (they depend only on the set of distinct UMIs),
    identical on every rank. ranges_per_file > 0 overrides the cut (default: world)."""
    import torch

    from . import dist as RD

    W = RD.world(group)
    r = torch.distributed.get_rank(group) if W > 1 else 0
    paths = list(bam_paths)
    tm = [("start", time.perf_counter())] if os.environ.get("ROGTK_BAM_TIMING") == "1" else None
    ranges = _umi_ranges(paths, ranges_per_file or W, split)
    mine = [j for j in range(len(ranges)) if j % W == r]
    dev = torch.device("cuda", torch.cuda.current_device())
    res = {}  # range index -> (column, names, skip used, tail, error)
    # this rank's ranges decode concurrently (round 5): one host thread per range, each with
    # its own reader (its share of the inflate threads) and its own device stream, as the
    # reference hands its segments to a worker pool (bam_htslib.rs:665-725)
    per_reader = max(1, (n_threads or 16) // max(len(mine), 1)) if len(mine) > 1 else n_threads

    def decode(j, skip):
        torch.cuda.set_device(dev)  # a worker thread starts on the process's default device
        t0 = time.perf_counter()
        fi, i, c0, c1 = ranges[j]
        if skip is None:
            skip = 0 if i == 0 else bam_find_record(paths[fi], c0)
        try:
            col, nm, tail = bam_umis_dev(paths[fi], umi_len, source, sep, mode, per_reader, with_names=True,
                                         rng=None if (c0 == 0 and c1 < 0) else (c0, c1, skip), return_tail=True)
            res[j] = (col, nm, skip, tail, None)
            if tm is not None:
                print(f"range {j}: {t0 - tm[0][1]:.4f} .. {time.perf_counter() - tm[0][1]:.4f} s, {col[3]} rows",
                      flush=True)
        except _lib.RogtkError as e:
            if ranges[j][1] == 0:
                raise  # a range that starts with the header: a real error
            # a wrong guess can frame garbage: decoded again below; kept to re-raise if the
            # guess turns out right (then the error is the file's)
            res[j] = (None, None, skip, -3, e)

    def decode_all(jobs):
        if len(jobs) == 1:
            decode(*jobs[0])
            return
        with ThreadPoolExecutor(max_workers=len(jobs)) as ex:
            for f in [ex.submit(decode, j, skip) for j, skip in jobs]:
                f.result()
        torch.cuda.synchronize(dev)  # the workers' streams, before the columns are used here

    if tm is not None:
        tm.append(("split", time.perf_counter()))
    decode_all([(j, None) for j in mine])
    if tm is not None:
        tm.append(("decode", time.perf_counter()))
    # check every guessed skip against the previous range's tail (exact once that range's
    # own start is); at most len(ranges) rounds, one in practice
    for _ in range(len(ranges)):
        t = torch.full((len(ranges), 2), -(2 ** 62), dtype=torch.int64)
        for j in mine:
            t[j, 0], t[j, 1] = res[j][2], res[j][3]
        if W > 1:
            tt = t.to(dev) if torch.distributed.get_backend(group) == "nccl" else t
            torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX, group=group)
            t = tt.cpu()
        bad = [j for j in range(len(ranges))
               if ranges[j][1] > 0 and (t[j, 0] != t[j - 1, 1] or t[j - 1, 1] < 0)]
        for j in mine:  # a failed range whose start was right: the error is real
            if res[j][4] is not None and ranges[j][1] > 0 and t[j - 1, 1] >= 0 and t[j, 0] == t[j - 1, 1]:
                raise res[j][4]
        if tm is not None:
            print(f"settle: skips {[int(t[j, 0]) for j in range(len(ranges))]}, tails "
                  f"{[int(t[j, 1]) for j in range(len(ranges))]}, redo {bad}", flush=True)
        if not bad:
            break
        decode_all([(j, int(t[j - 1, 1])) for j in bad if j in mine and t[j - 1, 1] >= 0])
    else:
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, "bam ranges: record boundaries did not settle")
    parts = [res[j][0] for j in mine]
    names = [res[j][1] if res[j][1] is not None else pa.array([], pa.string()) for j in mine]
    srcs = [_repeat_str(paths[ranges[j][0]], res[j][0][3]) for j in mine]
    off, val, vw, n = _concat_dev([p[0] for p in parts], [p[1] for p in parts], [p[2] for p in parts],
                                  [p[3] for p in parts], dev) if parts else _concat_dev([], [], [], [], dev)
    if tm is not None:
        torch.cuda.synchronize(dev)
        tm.append(("settle+concat", time.perf_counter()))
    if W == 1:  # no exchange: the single-GPU H3 on the whole column (same ids)
        cid, k = _cluster_dev(off, val, vw, n, umi_len, max_distance)
    else:
        cid, k = RD.umi_cluster_sharded(off, val, n, umi_len, max_distance, validity=vw.view(torch.uint8),
                                        group=group)
    if tm is not None:
        torch.cuda.synchronize(dev)
        tm.append(("cluster", time.perf_counter()))
    nm = pa.concat_arrays(names) if names else pa.array([], pa.string())
    src = pa.concat_arrays(srcs) if srcs else pa.array([], pa.string())
    out = _umi_table(off, val, vw, n, nm, cid, k, {"source": src})
    if tm is not None:
        tm.append(("table", time.perf_counter()))
        print("bams_umi_cluster timing (s): " + ", ".join(f"{a}={b - tm[i][1]:.4f}" for i, (a, b) in
                                                         enumerate(tm[1:])), flush=True)
    return out


def _cluster_dev(off, val, vw, n, umi_len, max_distance):
    """rogtk_umi_cluster_dev on a device UMI column: (cluster_id int32 tensor, n_clusters)."""
    import torch

    stream = torch.cuda.current_stream()
    cid = torch.empty(max(n, 1), dtype=torch.int32, device=off.device)
    ncl = ctypes.c_int64(0)
    _lib.call("rogtk_umi_cluster_dev", ctypes.c_void_p(off.data_ptr()), ctypes.c_void_p(val.data_ptr()),
              ctypes.c_void_p(vw.data_ptr()), n, int(umi_len), int(max_distance), ctypes.c_void_p(cid.data_ptr()),
              ctypes.byref(ncl), ctypes.c_void_p(stream.cuda_stream))
    return cid, ncl.value


def bam_umi_cluster(bam_path: str, umi_len: int = 12, max_distance: int = 1, source: str = "sequence",
                    sep: str = "_", mode: str = "htslib", n_threads: int = 0) -> pa.Table:
    """Config C5: BAM -> GPU decode -> UMI column -> H3 cluster ids (and the UMI).
    Returns a Table {name, umi, cluster_id} with the H3 semantics of umi_cluster
    (DESIGN.md §4): dense ids, regular UMIs first, irregular ones after, null -> null."""
    (off, val, vw, n), names = bam_umis_dev(bam_path, umi_len, source, sep, mode, n_threads, with_names=True)
    cid, ncl = _cluster_dev(off, val, vw, n, umi_len, max_distance)
    return _umi_table(off, val, vw, n, names, cid, ncl)
