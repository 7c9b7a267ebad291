"""Host-side mirror of rogtk's assembly expressions (H4.4 + H5), backed by librogtk_hip.

reference (rogtk/__init__.py -> src/expressions.rs)          rogtk_amd
===========================================================  ==============================
``assemble_sequences(expr, k=10, min_coverage=5, ...)``        ``assemble_sequences(column, ...)``
(:104-156 -> expressions.rs:695-762)
``assemble_sequences_with_anchors(expr, start_col, end_col``  ``assemble_sequences_with_anchors(...)``
(:158-234 -> expressions.rs:770-849)
``sweep_assembly_params(...)`` (:236-287 -> :880-955)          ``sweep_assembly_params(...)``
``optimize_assembly(...)`` (:289-323 -> fracture_opt.rs:283)   ``optimize_assembly(...)``
``df.group_by(key).agg(assemble_sequences(...))``              ``assemble_groups(...)`` /
(:206-214, one plugin call per group)                          ``assemble_column_groups(...)`` (round 6)
===========================================================  ==============================

Each call is one polars group (the reference registers them ``returns_scalar``).
The k-mer spectrum runs on the GPU (rogtk_kmer_spectrum_host); graph building,
compression and path finding run in native C++ on the host, as in the reference
(include/rogtk_hip.h; semantics and what is parity-unpinned: rogtk_amd/csrc/assembly.cpp).
``export_graphs`` / ``prefix`` (DOT / CSV files) are accepted and ignored.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import pyarrow as pa

from . import _lib
from .columns import ColumnLike, chunks


def _group(column: ColumnLike):
    arr = column
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks else pa.array([], type=arr.type)
    chs = list(chunks(arr))
    assert len(chs) == 1
    return chs[0]


def _enc(s: Optional[str]):
    return None if s is None else (s.encode() if isinstance(s, str) else bytes(s))


def _assemble(column, k, min_coverage, method, start_anchor, end_anchor, min_length, only_largest, auto_k) -> str:
    ch = _group(column)
    o, v, val = ch.ptrs()
    need = ctypes.c_int64(0)
    nc = ctypes.c_int64(0)
    cap = max(int(ch.values.size) * 2 + 1024, 4096)
    while True:
        buf = ctypes.create_string_buffer(cap)
        try:
            _lib.call("rogtk_assemble_host", o, ch.offset_width, v, ch.values.size, val, ch.validity_offset, ch.n,
                      int(k), int(min_coverage), _enc(method), _enc(start_anchor), _enc(end_anchor),
                      int(bool(only_largest)), -1 if min_length is None else int(min_length), int(bool(auto_k)),
                      buf, cap, ctypes.byref(need), ctypes.byref(nc))
        except _lib.RogtkError as e:
            if e.code == _lib.ROGTK_E_OVERFLOW and need.value > cap:
                cap = int(need.value)
                continue
            raise
        return buf.raw[: need.value].decode()


def assemble_sequences(column: ColumnLike, k: int = 10, min_coverage: int = 5, method: str = "shortest_path",
                       start_anchor: Optional[str] = None, end_anchor: Optional[str] = None,
                       min_length: Optional[int] = None, export_graphs: bool = False, only_largest: bool = False,
                       auto_k: bool = False, prefix: Optional[str] = None) -> str:
    """assemble_sequences_expr: the group's contig(s) joined by '\\n'. The expression
    always asks for the largest contig only (expressions.rs:751), whatever only_largest says."""
    return _assemble(column, k, min_coverage, method, start_anchor, end_anchor, min_length, True, auto_k)


def assemble_sequences_with_anchors(column: ColumnLike, start_anchor_col: ColumnLike, end_anchor_col: ColumnLike,
                                    k: int = 17, min_coverage: int = 25, method: str = "shortest_path",
                                    min_length: Optional[int] = None, export_graphs: bool = False,
                                    auto_k: bool = False, prefix: Optional[str] = None) -> str:
    """expressions.rs:770-849: anchors from row 0 of the anchor columns; shortest_path only."""
    sa = pa.array(start_anchor_col) if not isinstance(start_anchor_col, (pa.Array, pa.ChunkedArray)) else start_anchor_col
    ea = pa.array(end_anchor_col) if not isinstance(end_anchor_col, (pa.Array, pa.ChunkedArray)) else end_anchor_col
    if len(sa) == 0 or sa[0].as_py() is None:
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, "start_anchor column is empty")
    if len(ea) == 0 or ea[0].as_py() is None:
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, "end_anchor column is empty")
    if method == "compression":
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID,
                              "compression method is not supported with dynamic anchors; use shortest_path")
    if method == "shortest_path_auto":
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID,
                              "shortest_path_auto method is not supported with dynamic anchors; use shortest_path")
    if method != "shortest_path":
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, "Invalid assembly method for dynamic anchors. Must be 'shortest_path'")
    s0, e0 = sa[0].as_py(), ea[0].as_py()
    return _assemble(column, k, min_coverage, "shortest_path", s0, e0, min_length, True, auto_k)


SWEEP_TYPE = pa.struct([("k", pa.int64()), ("min_coverage", pa.int64()), ("contig_length", pa.int64())])
OPTIMIZE_TYPE = pa.struct([("contig", pa.string()), ("k", pa.uint32()), ("min_coverage", pa.uint32()),
                           ("length", pa.uint32()), ("input_sequences", pa.uint32())])


def sweep_assembly_params(column: ColumnLike, k_start: int = 5, k_end: int = 32, k_step: int = 1,
                          cov_start: int = 1, cov_end: int = 150, cov_step: int = 1, method: str = "shortest_path",
                          start_anchor: Optional[str] = None, end_anchor: Optional[str] = None,
                          min_length: Optional[int] = None, export_graphs: bool = False,
                          prefix: Optional[str] = None, auto_k: bool = False) -> pa.StructArray:
    """sweep_assembly_params_expr: one row per (k, min_coverage) of the grid, largest
    contig length (0 when none). The k-mer spectrum is computed once per effective k."""
    ch = _group(column)
    o, v, val = ch.ptrs()
    nk = max(0, (k_end - k_start) // k_step + 1) if k_step > 0 and k_end >= k_start else 0
    nc = max(0, (cov_end - cov_start) // cov_step + 1) if cov_step > 0 and cov_end >= cov_start else 0
    cap = max(nk * nc, 1)
    ok, oc, ol = (np.zeros(cap, dtype=np.int64) for _ in range(3))
    n = ctypes.c_int64(0)
    p = lambda a: ctypes.c_void_p(a.ctypes.data)
    _lib.call("rogtk_assembly_sweep_host", o, ch.offset_width, v, ch.values.size, val, ch.validity_offset, ch.n,
              int(k_start), int(k_end), int(k_step), int(cov_start), int(cov_end), int(cov_step), _enc(method),
              _enc(start_anchor), _enc(end_anchor), cap, p(ok), p(oc), p(ol), ctypes.byref(n))
    m = int(n.value)
    return pa.StructArray.from_arrays([pa.array(ok[:m]), pa.array(oc[:m]), pa.array(ol[:m])],
                                      fields=list(SWEEP_TYPE))


def optimize_assembly(column: ColumnLike, method: str = "shortest_path", start_anchor: Optional[str] = None,
                      end_anchor: Optional[str] = None, start_k: int = 31, start_min_coverage: int = 1,
                      min_length: Optional[int] = None, export_graphs: bool = False, prefix: Optional[str] = None,
                      max_iterations: Optional[int] = None, explore_k: Optional[bool] = None,
                      prioritize_length: Optional[bool] = None) -> dict:
    """optimize_assembly_expr (fracture_opt.rs:283-356): greedy beam over (k, min_coverage)."""
    if start_anchor is None or end_anchor is None:
        raise ValueError("Both start_anchor and end_anchor are required")
    ch = _group(column)
    o, v, val = ch.ptrs()
    out4 = (ctypes.c_uint32 * 4)()
    need = ctypes.c_int64(0)
    cap = max(int(ch.values.size) * 2 + 1024, 4096)
    while True:
        buf = ctypes.create_string_buffer(cap)
        try:
            _lib.call("rogtk_assembly_optimize_host", o, ch.offset_width, v, ch.values.size, val, ch.validity_offset,
                      ch.n, _enc(method), _enc(start_anchor), _enc(end_anchor), int(start_k), int(start_min_coverage),
                      50 if max_iterations is None else int(max_iterations), int(bool(explore_k)),
                      int(bool(prioritize_length)), buf, cap, ctypes.byref(need), out4)
        except _lib.RogtkError as e:
            if e.code == _lib.ROGTK_E_OVERFLOW and need.value > cap:
                cap = int(need.value)
                continue
            raise
        return {"contig": buf.raw[: need.value].decode(), "k": out4[0], "min_coverage": out4[1],
                "length": out4[2], "input_sequences": out4[3]}


def assemble_groups(spectrum: dict, method: str = "compression", start_anchor: Optional[str] = None,
                    end_anchor: Optional[str] = None, min_length: Optional[int] = None, only_largest: bool = True,
                    n_threads: int = 0):
    """Batched H5 (round 6): every group of one k-mer spectrum result (a device or host
    dict of rogtk_amd.device.kmer_spectrum_* / a group_spectra call: kmers, exts, counts,
    entry_offsets, stats) assembled at once on host threads (rogtk_assemble_groups_host).
    The spectrum must be taken at the assembly's min_coverage: its entries are then the
    preliminary graph of each group (fracture.rs:343-348). Returns (LargeString array of
    one string per group - its contigs joined by '\\n', as assemble_sequences_expr's row -,
    int64 contig counts). only_largest=True is what the expression asks for
    (expressions.rs:751)."""
    def host(t, dt):
        a = t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)
        return np.ascontiguousarray(a.view(dt) if a.dtype != dt and a.dtype.itemsize == np.dtype(dt).itemsize else a,
                                    dtype=dt)
    km = host(spectrum["kmers"], np.uint64).reshape(-1)
    ex = host(spectrum["exts"], np.uint8)
    cn = host(spectrum["counts"], np.uint16)
    eo = host(spectrum["entry_offsets"], np.int64)
    st = host(spectrum["stats"], np.int64).reshape(-1)
    G = len(eo) - 1
    p = lambda a: ctypes.c_void_p(a.ctypes.data) if a.size else None
    h = ctypes.c_void_p()
    _lib.call("rogtk_assemble_groups_host", p(km), p(ex), p(cn), p(eo), p(st), G, _enc(method), _enc(start_anchor),
              _enc(end_anchor), int(bool(only_largest)), -1 if min_length is None else int(min_length),
              int(n_threads), ctypes.byref(h))
    try:
        ng, nb = ctypes.c_int64(0), ctypes.c_int64(0)
        _lib.call("rogtk_assembly_result_sizes", h, ctypes.byref(ng), ctypes.byref(nb))
        offs = np.zeros(int(ng.value) + 1, np.int64)
        vals = np.zeros(max(int(nb.value), 1), np.uint8)
        nc = np.zeros(max(int(ng.value), 1), np.int64)
        _lib.call("rogtk_assembly_result_copy", h, p(offs), p(vals), p(nc))
    finally:
        _lib.call("rogtk_assembly_result_free", h)
    arr = pa.Array.from_buffers(pa.large_string(), int(ng.value), [None, pa.py_buffer(offs), pa.py_buffer(vals)])
    return arr, nc[: int(ng.value)]


def assemble_column_groups(offsets, values, keys, k: int = 10, min_coverage: int = 5, method: str = "compression",
                           start_anchor: Optional[str] = None, end_anchor: Optional[str] = None,
                           min_length: Optional[int] = None, only_largest: bool = True, n_threads: int = 0,
                           batch_rows: int = 10_000_000):
    """A device read column grouped by `keys` (e.g. H3 cluster ids: the caller's
    group_by('umi'), rogtk/__init__.py:206-214) and assembled per group: the k-mer spectra
    of all groups on the GPU (device.group_spectra at min_coverage), then assemble_groups
    per spectrum call. Returns (rows in group order, group offsets, strings per group,
    contig counts)."""
    from . import device as D

    outs, counts = [], []

    def consume(g0, g1, r):
        a, c = assemble_groups(r, method, start_anchor, end_anchor, min_length, only_largest, n_threads)
        outs.append(a)
        counts.append(c)

    rows, go, G, _ = D.group_spectra(offsets, values, keys, k, min_coverage, batch_rows=batch_rows, consume=consume)
    arr = pa.concat_arrays(outs) if outs else pa.array([], type=pa.large_string())
    return rows, go, arr, (np.concatenate(counts) if counts else np.zeros(0, np.int64))
