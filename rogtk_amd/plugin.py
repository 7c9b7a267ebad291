"""polars plugin surface of librogtk_hip.so (the drop-in boundary).

The reference registers its expressions with polars' ``register_plugin_function``
(rogtk/__init__.py:138-156, 216-234, 266-287, 305-323, 333-349, 419-526); polars then
calls ``_polars_plugin_<function_name>`` in the first shared library of the package
directory. librogtk_hip.so is the only shared library in ``rogtk_amd/`` and exports
those symbols (rogtk_amd/csrc/polars_plugin.cpp), so:

* with polars installed, ``register_polars()`` registers the reference's ``umi`` and
  ``hamming`` expression namespaces and the module-level functions below return
  ``pl.Expr`` exactly as rogtk's do (same function names, kwargs and defaults);
* without polars (this image), ``call_plugin`` drives the same symbols through the same
  calling convention polars uses: inputs exported over the Arrow C Data Interface into
  ``SeriesExport`` structs, kwargs pickled with protocol 5, the result imported back.
  The tests use it to check the ABI end to end.
"""
from __future__ import annotations

import ctypes
import pickle
from pathlib import Path
from typing import Any, Dict, Iterable, List, Optional, Sequence

import pyarrow as pa

from . import _lib

PLUGIN_PATH = Path(__file__).parent

# every expression the reference's Python registers for this path
EXPRESSIONS = (
    "umi_complexity_all_expr", "umi_shannon_entropy_expr", "umi_linguistic_complexity_expr",
    "umi_homopolymer_fraction_expr", "umi_dinucleotide_entropy_expr", "umi_combined_score_expr",
    "umi_longest_homopolymer_expr", "umi_dust_score_expr", "hamming_distance_expr", "hamming_within_expr",
    "assemble_sequences_expr", "assemble_sequences_with_anchors_expr", "sweep_assembly_params_expr",
    "optimize_assembly_expr",
    # element-wise string expressions (expressions.rs:29-665, 957-977)
    "reverse_complement_series", "parse_cigar_series", "cigar_aligned_ref_expr", "cigar_aligned_query_expr",
    "extract_cigar_insertions_expr", "enrich_allele_insertions_expr", "phred_to_numeric_series_str",
    "phred_to_numeric_series",
)


# ------------------------------------------------------------ C Data Interface
class ArrowSchema(ctypes.Structure):
    pass


ArrowSchema._fields_ = [
    ("format", ctypes.c_char_p), ("name", ctypes.c_char_p), ("metadata", ctypes.c_char_p),
    ("flags", ctypes.c_int64), ("n_children", ctypes.c_int64),
    ("children", ctypes.POINTER(ctypes.POINTER(ArrowSchema))), ("dictionary", ctypes.POINTER(ArrowSchema)),
    ("release", ctypes.c_void_p), ("private_data", ctypes.c_void_p),
]


class ArrowArray(ctypes.Structure):
    _fields_ = [
        ("length", ctypes.c_int64), ("null_count", ctypes.c_int64), ("offset", ctypes.c_int64),
        ("n_buffers", ctypes.c_int64), ("n_children", ctypes.c_int64), ("buffers", ctypes.c_void_p),
        ("children", ctypes.c_void_p), ("dictionary", ctypes.c_void_p), ("release", ctypes.c_void_p),
        ("private_data", ctypes.c_void_p),
    ]


class SeriesExport(ctypes.Structure):
    pass


_SERIES_RELEASE = ctypes.CFUNCTYPE(None, ctypes.POINTER(SeriesExport))
SeriesExport._fields_ = [
    ("field", ctypes.POINTER(ArrowSchema)), ("arrays", ctypes.POINTER(ctypes.POINTER(ArrowArray))),
    ("len", ctypes.c_size_t), ("release", ctypes.c_void_p), ("private_data", ctypes.c_void_p),
]


class CallerContext(ctypes.Structure):
    _fields_ = [("bitflags", ctypes.c_uint64)]


_EXPR_FN = ctypes.CFUNCTYPE(None, ctypes.POINTER(SeriesExport), ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                            ctypes.POINTER(SeriesExport), ctypes.POINTER(CallerContext))
_FIELD_FN = ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowSchema), ctypes.c_size_t, ctypes.POINTER(ArrowSchema),
                             ctypes.c_char_p, ctypes.c_size_t)


def _symbol(name: str, proto):
    lib = _lib.hip()
    return proto(("_polars_plugin_" + name, lib))


def last_error() -> str:
    fn = _lib.hip()._polars_plugin_get_last_error_message
    fn.restype = ctypes.c_char_p
    return (fn() or b"").decode(errors="replace")


def plugin_version() -> int:
    fn = _lib.hip()._polars_plugin_get_version
    fn.restype = ctypes.c_uint32
    return int(fn())


def serialize_kwargs(kwargs: Optional[Dict[str, Any]]) -> bytes:
    """polars' plugins._serialize_kwargs: empty -> b"", else pickle protocol 5."""
    if not kwargs:
        return b""
    return pickle.dumps(kwargs, protocol=5)


class _Exported:
    """One input series exported as polars would (export_series): a schema, one
    ArrowArray per chunk, and a release that frees the containers only."""

    def __init__(self, column, name: str):
        if isinstance(column, pa.ChunkedArray):
            chunks = list(column.chunks)
            typ = column.type
        else:
            arr = column if isinstance(column, pa.Array) else pa.array(column, type=pa.string())
            chunks, typ = [arr], arr.type
        self.schema = ArrowSchema()
        pa.field(name, typ)._export_to_c(ctypes.addressof(self.schema))
        self.arrays = [ArrowArray() for _ in chunks]
        for a, ch in zip(self.arrays, chunks):
            ch._export_to_c(ctypes.addressof(a))
        self.ptrs = (ctypes.POINTER(ArrowArray) * max(len(chunks), 1))(*[ctypes.pointer(a) for a in self.arrays])
        self.released = False

        def _release(p):
            # the containers are owned by this Python object; free the schema
            e = p.contents
            if e.field and e.field.contents.release:
                ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowSchema))(e.field.contents.release)(e.field)
            e.release = None
            self.released = True

        self._cb = _SERIES_RELEASE(_release)

    def fill(self, e: SeriesExport) -> None:
        e.field = ctypes.pointer(self.schema)
        e.arrays = ctypes.cast(self.ptrs, ctypes.POINTER(ctypes.POINTER(ArrowArray)))
        e.len = len(self.arrays)
        e.release = ctypes.cast(self._cb, ctypes.c_void_p).value
        e.private_data = 1


def call_plugin(function_name: str, inputs: Sequence, kwargs: Optional[Dict[str, Any]] = None,
                names: Optional[Sequence[str]] = None) -> pa.ChunkedArray:
    """Call ``_polars_plugin_<function_name>`` the way polars does; returns the result
    series as a pyarrow ChunkedArray (its name: ``.name`` attribute of the returned
    object's field, see ``call_plugin_field``). Raises RogtkError with the plugin's
    last-error message on failure."""
    result, _ = call_plugin_named(function_name, inputs, kwargs, names)
    return result


def call_plugin_named(function_name: str, inputs: Sequence, kwargs: Optional[Dict[str, Any]] = None,
                      names: Optional[Sequence[str]] = None):
    names = list(names) if names is not None else [f"c{i}" for i in range(len(inputs))]
    ex = [_Exported(c, n) for c, n in zip(inputs, names)]
    arr = (SeriesExport * max(len(ex), 1))()
    for i, e in enumerate(ex):
        e.fill(arr[i])
    out = SeriesExport()
    ctx = CallerContext(0)
    kw = serialize_kwargs(kwargs)
    fn = _symbol(function_name, _EXPR_FN)
    fn(arr, len(ex), kw, len(kw), ctypes.byref(out), ctypes.byref(ctx))
    if not all(e.released for e in ex):
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, "plugin did not release its inputs")
    if not out.private_data:
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, last_error())
    # polars' import_series: the field, then each array moved out; then release the export
    field = pa.Field._import_from_c(ctypes.addressof(out.field.contents))
    chunks = [pa.Array._import_from_c(ctypes.addressof(out.arrays[i].contents), field.type) for i in range(out.len)]
    ctypes.CFUNCTYPE(None, ctypes.POINTER(SeriesExport))(out.release)(ctypes.byref(out))
    return pa.chunked_array(chunks, type=field.type), field.name


def call_plugin_field(function_name: str, input_fields: Iterable[pa.Field],
                      kwargs: Optional[Dict[str, Any]] = None) -> pa.Field:
    """``_polars_plugin_field_<function_name>``: the output field polars plans with."""
    fields = list(input_fields)
    arr = (ArrowSchema * max(len(fields), 1))()
    for i, f in enumerate(fields):
        f._export_to_c(ctypes.addressof(arr[i]))
    out = ArrowSchema()
    kw = serialize_kwargs(kwargs)
    _symbol("field_" + function_name, _FIELD_FN)(arr, len(fields), ctypes.byref(out), kw, len(kw))
    for i in range(len(fields)):
        if arr[i].release:
            ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowSchema))(arr[i].release)(ctypes.byref(arr[i]))
    if not out.release:
        raise _lib.RogtkError(_lib.ROGTK_E_INVALID, last_error())
    return pa.Field._import_from_c(ctypes.addressof(out))


# ------------------------------------------------------------ polars registration
def register_polars():
    """With polars importable: the reference's registrations (rogtk/__init__.py), with
    plugin_path = this package directory. Returns the namespace classes and functions,
    or None when polars is absent (it is not part of this image)."""
    try:
        import polars as pl
        from polars.plugins import register_plugin_function
    except ImportError:
        return None

    def reg(name, args, kwargs=None, **flags):
        return register_plugin_function(plugin_path=PLUGIN_PATH, function_name=name, args=args, kwargs=kwargs,
                                        **flags)

    @pl.api.register_expr_namespace("hamming")
    class HammingExpr:  # rogtk/__init__.py:326-349
        def __init__(self, expr):
            self._expr = expr

        def distance(self, target: str):
            return reg("hamming_distance_expr", self._expr, {"target": target}, is_elementwise=True)

        def within(self, target: str, max_distance: int = 1):
            return reg("hamming_within_expr", self._expr, {"target": target, "max_distance": max_distance},
                       is_elementwise=True)

    @pl.api.register_expr_namespace("umi")
    class UmiNamespace:  # rogtk/__init__.py:412-491
        def __init__(self, expr):
            self._expr = expr

        def complexity_all(self):
            return reg("umi_complexity_all_expr", self._expr, is_elementwise=True)

        def all_scores(self):
            return self.complexity_all()

        def shannon_entropy(self):
            return reg("umi_shannon_entropy_expr", self._expr, is_elementwise=True)

        def linguistic_complexity(self):
            return reg("umi_linguistic_complexity_expr", self._expr, is_elementwise=True)

        def homopolymer_fraction(self):
            return reg("umi_homopolymer_fraction_expr", self._expr, is_elementwise=True)

        def dinucleotide_entropy(self):
            return reg("umi_dinucleotide_entropy_expr", self._expr, is_elementwise=True)

        def combined_score(self):
            return reg("umi_combined_score_expr", self._expr, is_elementwise=True)

        def longest_homopolymer_run(self):
            return reg("umi_longest_homopolymer_expr", self._expr, is_elementwise=True)

        def dust_score(self):
            return reg("umi_dust_score_expr", self._expr, is_elementwise=True)

    def umi_complexity_scores(expr):  # :493-526
        return reg("umi_complexity_all_expr", expr, is_elementwise=True)

    def assemble_sequences(expr, k=10, min_coverage=5, method="shortest_path", start_anchor=None,
                           end_anchor=None, min_length=None, export_graphs=False, only_largest=False,
                           auto_k=False, prefix=None):  # :104-156
        return reg("assemble_sequences_expr", expr,
                   {"k": k, "min_coverage": min_coverage, "method": method, "start_anchor": start_anchor,
                    "end_anchor": end_anchor, "min_length": min_length, "export_graphs": export_graphs,
                    "only_largest": only_largest, "auto_k": auto_k, "prefix": prefix},
                   returns_scalar=True, is_elementwise=False)

    def assemble_sequences_with_anchors(expr, start_anchor_col, end_anchor_col, k=17, min_coverage=25,
                                        method="shortest_path", min_length=None, export_graphs=False,
                                        auto_k=False, prefix=None):  # :158-234
        return reg("assemble_sequences_with_anchors_expr", [expr, start_anchor_col, end_anchor_col],
                   {"k": k, "min_coverage": min_coverage, "method": method, "start_anchor": None,
                    "end_anchor": None, "min_length": min_length, "export_graphs": export_graphs,
                    "only_largest": False, "auto_k": auto_k, "prefix": prefix},
                   returns_scalar=True, is_elementwise=False)

    def sweep_assembly_params(expr, k_start=5, k_end=32, k_step=1, cov_start=1, cov_end=150, cov_step=1,
                              method="shortest_path", start_anchor=None, end_anchor=None, min_length=None,
                              export_graphs=False, prefix=None, auto_k=False):  # :236-287
        return reg("sweep_assembly_params_expr", expr,
                   {"k_start": k_start, "k_end": k_end, "k_step": k_step, "cov_start": cov_start,
                    "cov_end": cov_end, "cov_step": cov_step, "method": method, "start_anchor": start_anchor,
                    "end_anchor": end_anchor, "min_length": min_length, "export_graphs": export_graphs,
                    "prefix": prefix, "auto_k": auto_k},
                   returns_scalar=True, is_elementwise=False)

    def optimize_assembly(expr, method="shortest_path", start_anchor=None, end_anchor=None, start_k=31,
                          start_min_coverage=1, min_length=None, export_graphs=False, prefix=None,
                          max_iterations=None, explore_k=None, prioritize_length=None):  # :289-323
        if start_anchor is None or end_anchor is None:
            raise ValueError("Both start_anchor and end_anchor are required")
        return reg("optimize_assembly_expr", expr,
                   {"method": method, "start_anchor": start_anchor, "end_anchor": end_anchor,
                    "start_k": start_k, "start_min_coverage": start_min_coverage, "min_length": min_length,
                    "export_graphs": export_graphs, "prefix": prefix, "max_iterations": max_iterations,
                    "explore_k": explore_k, "prioritize_length": prioritize_length},
                   returns_scalar=True, is_elementwise=False)

    return {"HammingExpr": HammingExpr, "UmiNamespace": UmiNamespace, "umi_complexity_scores": umi_complexity_scores,
            "assemble_sequences": assemble_sequences,
            "assemble_sequences_with_anchors": assemble_sequences_with_anchors,
            "sweep_assembly_params": sweep_assembly_params, "optimize_assembly": optimize_assembly}


def kwargs_as_parsed(kwargs: Optional[Dict[str, Any]] = None, raw: Optional[bytes] = None) -> str:
    """The kwargs as the plugin's pickle reader sees them ("key=value" lines, sorted)."""
    data = serialize_kwargs(kwargs) if raw is None else raw
    need = ctypes.c_int64(0)
    cap = 1 << 16
    buf = ctypes.create_string_buffer(cap)
    rc = _lib.hip().rogtk_plugin_kwargs_debug(data, len(data), buf, cap, ctypes.byref(need))
    if rc == _lib.ROGTK_E_OVERFLOW:
        cap = int(need.value)
        buf = ctypes.create_string_buffer(cap)
        rc = _lib.hip().rogtk_plugin_kwargs_debug(data, len(data), buf, cap, ctypes.byref(need))
    if rc != 0:
        raise _lib.RogtkError(rc, last_error())
    return buf.raw[: need.value].decode()
