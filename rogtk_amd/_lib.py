"""ctypes binding of the in-tree C-ABI libraries (include/rogtk_hip.h).

The product path has no fallback: if ``librogtk_hip.so`` is missing the import of
anything that computes raises ``RogtkError`` with the build instruction. There is
no CPU implementation of the kernels anywhere in this package.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
HIP_LIB_PATH = os.path.join(_HERE, "librogtk_hip.so")
SYNTH_LIB_PATH = os.path.join(_HERE, "_synth", "librogtk_synth.so")

ROGTK_OK = 0
ROGTK_E_INVALID = 1
ROGTK_E_HIP = 2
ROGTK_E_UNSUPPORTED = 3
ROGTK_E_NODEVICE = 4
ROGTK_E_OVERFLOW = 5


class RogtkError(RuntimeError):
    """Raised for every non-zero status returned across the C ABI."""

    def __init__(self, code: int, message: str):
        super().__init__(f"[rogtk status {code}] {message}")
        self.code = code


class UmiScores(ctypes.Structure):
    """rogtk_umi_scores (include/rogtk_hip.h): field order of
    umi_complexity_struct_output_type (reference src/expressions.rs:1219-1232)."""

    _fields_ = [
        ("shannon_entropy", ctypes.c_void_p),
        ("linguistic_complexity", ctypes.c_void_p),
        ("homopolymer_fraction", ctypes.c_void_p),
        ("dinucleotide_entropy", ctypes.c_void_p),
        ("longest_homopolymer_run", ctypes.c_void_p),
        ("dust_score", ctypes.c_void_p),
        ("combined_score", ctypes.c_void_p),
    ]


class BamBatch(ctypes.Structure):
    """rogtk_bam_batch (include/rogtk_hip.h): string columns name / chrom / sequence /
    quality_scores, u32 columns start / end / flags (create_bam_schema, bam.rs:3203-3221)."""

    _fields_ = [
        ("offsets", ctypes.c_void_p * 4),
        ("values", ctypes.c_void_p * 4),
        ("validity", ctypes.c_void_p * 4),
        ("u32", ctypes.c_void_p * 3),
        ("u32_validity", ctypes.c_void_p * 3),
    ]


class StrCol(ctypes.Structure):
    """rogtk_str_col (include/rogtk_hip.h): one Arrow string column."""

    _fields_ = [
        ("offsets", ctypes.c_void_p),
        ("offset_width", ctypes.c_int),
        ("values", ctypes.c_void_p),
        ("values_len", ctypes.c_int64),
        ("validity", ctypes.c_void_p),
        ("validity_offset", ctypes.c_int64),
        ("n", ctypes.c_int64),
    ]


class StrResult(ctypes.Structure):
    """rogtk_str_result (include/rogtk_hip.h): library-allocated LargeUtf8 output."""

    _fields_ = [
        ("n", ctypes.c_int64),
        ("offsets", ctypes.c_void_p),
        ("values", ctypes.c_void_p),
        ("values_len", ctypes.c_int64),
        ("validity", ctypes.c_void_p),
        ("null_count", ctypes.c_int64),
    ]


_vp, _i64, _i32, _u32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32
_P_SCORES = ctypes.POINTER(UmiScores)
_P_I64 = ctypes.POINTER(ctypes.c_int64)
_P_I32 = ctypes.POINTER(ctypes.c_int)
_P_F64 = ctypes.POINTER(ctypes.c_double)

# name -> (argtypes) ; every function returns int status except the two strings
SIGNATURES = {
    "rogtk_device_count": [_P_I32],
    "rogtk_stage_strings": [_vp, _i32, _vp, _vp, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp],
    "rogtk_umi_score_assign_packed": [_vp, _vp, _i64, _i32, _P_SCORES, _vp, _i64, _u32, _vp, _vp, _vp, _i64, _vp,
                                      _i32, _vp],
    "rogtk_umi_score_packed": [_vp, _vp, _i64, _i32, _P_SCORES, _vp, _i64, _u32, _vp, _vp, _vp],
    "rogtk_umi_score_rows": [_vp, _i32, _vp, _vp, _vp, _i64, _i64, _P_SCORES, _vp, _i64, _u32, _vp,
                             _vp, _vp],
    "rogtk_cluster_workspace_size": [_i32, _i64, _P_I64],
    "rogtk_cluster_bitmap_words": [_i32, _P_I64],
    "rogtk_cluster_init": [_vp, _i32, _i64, _vp],
    "rogtk_cluster_mark": [_vp, _vp, _i64, _i32, _vp, _i64, _vp],
    "rogtk_cluster_local_bitmap": [_vp, _i32, _i64, _vp, _vp],
    "rogtk_cluster_resolve": [_vp, _i32, _i64, _vp, _i32, _i32, _vp],
    "rogtk_cluster_assign": [_vp, _i32, _i64, _vp, _vp, _i64, _vp, _vp],
    "rogtk_cluster_assign_deferred": [_vp, _i32, _i64, _vp, _vp, _i64, _vp, _vp],
    "rogtk_cluster_sync": [_vp, _vp, ctypes.POINTER(ctypes.c_int)],
    "rogtk_cluster_stats": [_vp, _i32, _i64, _P_I64, _vp],
    "rogtk_cluster_release": [_vp],
    "rogtk_cluster_rounds": [_vp, _vp, ctypes.POINTER(ctypes.c_int)],
    "rogtk_cluster_set_spec_rounds": [_i32],
    "rogtk_cluster_set_lookback_polls": [_i32],
    "rogtk_cluster_set_mark_method": [_i32],
    "rogtk_long_codes": [_vp, _i32, _vp, _vp, _i64, _i64, _i32, _vp, _vp, _vp],
    "rogtk_unique_codes": [_vp, _vp, _i64, _i32, _vp, _P_I64, _vp],
    "rogtk_owner_counts": [_vp, _i64, _i32, _i32, _P_I64, _vp],
    "rogtk_masked_records": [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _P_I64, _vp],
    "rogtk_clique_edges": [_vp, _vp, _vp, _i64, _i32, _vp, _i64, _vp, _P_I64, _vp],
    "rogtk_cc_labels": [_i64, _vp, _i64, _vp, _P_I64, _vp],
    "rogtk_assign_codes": [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp],
    "rogtk_group_strings": [_vp, _vp, _i64, _i64, _u32, _vp, _P_I64, _vp],
    "rogtk_irregular_merge": [_vp, _vp, _i64, _i64, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _P_I64, _vp],
    "rogtk_cluster_mark_bitmap_temp_bytes": [_i64, _i32, _P_I64],
    "rogtk_cluster_mark_bitmap_phase": [_vp, _vp, _i64, _i32, _vp, _vp, _i64, _i32, _vp],
    "rogtk_cluster_mark_bitmap": [_vp, _vp, _i64, _i32, _vp, _vp, _i64, _vp],
    "rogtk_umi_cluster_dev": [_vp, _vp, _vp, _i64, _i32, _i32, _vp, ctypes.POINTER(_i64), _vp],
    "rogtk_route_pack": [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp],
    "rogtk_bam_open": [ctypes.c_char_p, _i32, ctypes.POINTER(_vp)],
    "rogtk_bam_open_range": [ctypes.c_char_p, _i32, _i64, _i64, _i64, ctypes.POINTER(_vp)],
    "rogtk_bam_range_tail": [_vp, _P_I64],
    "rogtk_bam_split_points": [ctypes.c_char_p, _i32, _P_I64, _P_I32],
    "rogtk_bam_find_record": [ctypes.c_char_p, _i64, _P_I64],
    "rogtk_bam_header": [_vp, ctypes.POINTER(_i64), ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                         ctypes.POINTER(_i64)],
    "rogtk_bam_next": [_vp, _i64, _i32, _i32, _i32, ctypes.POINTER(_i64), ctypes.POINTER(BamBatch)],
    "rogtk_bam_next_dev": [_vp, _i64, _i32, _i32, _i32, ctypes.POINTER(_i64), ctypes.POINTER(BamBatch), _vp],
    "rogtk_bam_umi_dev": [ctypes.POINTER(BamBatch), _i64, _i32, _i32, _i32, _vp, _vp, _i64, _vp, _vp],
    "rogtk_bam_close": [_vp],
    "rogtk_bam_umi_append": [ctypes.POINTER(BamBatch), _i64, _i32, _i32, _i32, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp],
    "rogtk_bam_append_strings": [_vp, _vp, _i64, _vp, _vp, _i64, _i64, _vp, _vp, _vp],
    "rogtk_bam_batch_bytes": [_vp, _P_I64],
    "rogtk_bam_check": [_vp, _vp],
    "rogtk_bam_timers": [_vp, _vp],
    "rogtk_copy": [_vp, _vp, _i64, _vp],
    "rogtk_plugin_kwargs_debug": [ctypes.c_char_p, _i64, ctypes.c_char_p, _i64, ctypes.POINTER(_i64)],
    "rogtk_umi_complexity_host": [_vp, _i32, _vp, _i64, _vp, _i64, _i64, _P_SCORES],
    "rogtk_hamming_host": [_vp, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _u32, _vp, _vp],
    "rogtk_umi_cluster_host": [_vp, _i32, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _P_I64,
                               _P_I32],
    "rogtk_kmer_capacity": [_vp, _i32, _i64, _P_I64],
    "rogtk_kmer_set_path": [_i32],
    "rogtk_kmer_set_filter": [_i32],
    "rogtk_group_by_key": [_vp, _i64, _vp, _vp, _P_I64, _vp],
    "rogtk_kmer_spectrum_dev": [_vp, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i64, _i64, _vp, _vp, _vp, _vp,
                                _vp, _P_I64, _vp],
    "rogtk_kmer_path_stats": [_P_I64],
    "rogtk_kmer_certified_groups": [_P_I64],
    "rogtk_kmer_lds_rows": [_P_I64],
    "rogtk_kmer_debug_filter": [_vp, _i64],
    "rogtk_read_block_words": [_i64],
    "rogtk_host_alloc": [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)],
    "rogtk_host_free": [_vp],
    "rogtk_event_create": [_i32, ctypes.POINTER(ctypes.c_void_p)],
    "rogtk_event_destroy": [_vp],
    "rogtk_event_record": [_vp, _vp],
    "rogtk_event_attach_next": [_vp],
    "rogtk_event_attach_done": [_vp],
    "rogtk_stream_wait_event": [_vp, _vp],
    "rogtk_event_query": [_vp, _P_I32],
    "rogtk_event_synchronize": [_vp],
    "rogtk_pack_reads": [_vp, _vp, _vp, _i64, _i64, _i32, _vp, _vp, _vp],
    "rogtk_max_row_len": [_vp, _i64, _P_I64, _vp],
    "rogtk_kmer_spectrum_fused": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i64, _i64, _vp, _vp, _vp,
                                  _vp, _vp, _P_I64, _i64, _i64, _vp],
    "rogtk_kmer_spectrum_blocks": [_vp, _i32, _i64, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i64, _i64, _vp,
                                   _vp, _vp, _vp, _vp, _P_I64, _vp],
    "rogtk_kmer_spectrum_host": [_vp, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _i32, _i32, _i64, _i64, _vp,
                                 _vp, _vp, _vp, _vp],
    "rogtk_assemble_host": [_vp, _i32, _vp, _i64, _vp, _i64, _i64, _i32, _i64, ctypes.c_char_p, ctypes.c_char_p,
                            ctypes.c_char_p, _i32, _i64, _i32, _vp, _i64, _P_I64, _P_I64],
    "rogtk_assembly_sweep_host": [_vp, _i32, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
                                  ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, _i64, _vp, _vp, _vp, _P_I64],
    "rogtk_assembly_optimize_host": [_vp, _i32, _vp, _i64, _vp, _i64, _i64, ctypes.c_char_p, ctypes.c_char_p,
                                     ctypes.c_char_p, _i64, _i64, _i64, _i32, _i32, _vp, _i64, _P_I64, _vp],
    "rogtk_concat_strings_dev": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp],
    "rogtk_assemble_groups_host": [_vp, _vp, _vp, _vp, _vp, _i64, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                   _i32, _i64, _i32, _vp],
    "rogtk_assembly_result_sizes": [_vp, _P_I64, _P_I64],
    "rogtk_assembly_result_copy": [_vp, _vp, _vp, _vp],
    "rogtk_assembly_result_free": [_vp],
    "rogtk_fastq_pair_open": [ctypes.c_char_p, ctypes.c_char_p, _i64, _i64, _i64, _i32, _vp],
    "rogtk_fastq_pair_next": [_vp, _i64, _P_I64, _vp, _vp],
    "rogtk_fastq_pair_close": [_vp],
    "rogtk_str_temp_bytes": [_i64, _P_I64],
    "rogtk_str_measure": [_i32, ctypes.POINTER(StrCol), _i32, _i64, _i64, _vp, _vp, _vp, _i64, _vp],
    "rogtk_str_fill": [_i32, ctypes.POINTER(StrCol), _i32, _i64, _i64, _vp, _vp, _vp],
    "rogtk_str_transform_host": [_i32, ctypes.POINTER(StrCol), _i32, _i64, _i64, ctypes.POINTER(StrResult)],
    "rogtk_profile_enable": [_i32],
    "rogtk_profile_select": [ctypes.c_char_p],
    "rogtk_profile_reset": [],
    "rogtk_profile_read": [ctypes.c_char_p, _P_F64, _P_I64],
    "rogtk_profile_read_span": [ctypes.c_char_p, _P_F64, _P_I64],
}

# functions returning void
VOID_SIGNATURES = {
    "rogtk_str_result_free": [ctypes.POINTER(StrResult)],
}

_lock = threading.Lock()
_hip = None
_synth = None


def _bind_one_hip_runtime() -> None:
    """Make the process use ONE HIP runtime.

    The torch wheel ships its own libamdhip64 (SONAME libamdhip64.so.7) that its
    libc10_hip NEEDs as "libamdhip64.so" through torch/lib's RPATH; librogtk_hip
    NEEDs "libamdhip64.so.7". Loading torch first makes the dynamic linker satisfy
    our dependency with torch's already-loaded runtime (SONAME match), so device
    pointers and streams from torch tensors are valid in our calls. Loading ours
    first would pull /opt/rocm's runtime AND later torch's second copy.
    """
    try:
        import torch  # noqa: F401
    except ImportError:  # plain C-ABI use without torch: /opt/rocm's runtime
        pass


def hip() -> ctypes.CDLL:
    """Load librogtk_hip.so (fails loudly when the extension was not built)."""
    global _hip
    with _lock:
        if _hip is None:
            _bind_one_hip_runtime()
            if not os.path.exists(HIP_LIB_PATH):
                raise RogtkError(ROGTK_E_NODEVICE,
                                 f"{HIP_LIB_PATH} is missing: build it with "
                                 "`python -c 'import __graft_entry__ as g; g.build()'` "
                                 "(make -C rogtk_amd/csrc). There is no CPU fallback.")
            lib = ctypes.CDLL(HIP_LIB_PATH)
            for name, argtypes in SIGNATURES.items():
                if not hasattr(lib, name):  # a missing export fails loudly at its first call
                    continue
                fn = getattr(lib, name)
                fn.argtypes = argtypes
                fn.restype = ctypes.c_int
            for name, argtypes in VOID_SIGNATURES.items():
                if hasattr(lib, name):
                    getattr(lib, name).argtypes = argtypes
                    getattr(lib, name).restype = None
            lib.rogtk_version.restype = ctypes.c_char_p
            lib.rogtk_version.argtypes = []
            lib.rogtk_last_error.restype = ctypes.c_char_p
            lib.rogtk_last_error.argtypes = []
            _hip = lib
    return _hip


def synth() -> ctypes.CDLL:
    global _synth
    with _lock:
        if _synth is None:
            if not os.path.exists(SYNTH_LIB_PATH):
                raise RogtkError(ROGTK_E_NODEVICE, f"{SYNTH_LIB_PATH} is missing: run make -C rogtk_amd/csrc")
            lib = ctypes.CDLL(SYNTH_LIB_PATH)
            u64, f64 = ctypes.c_uint64, ctypes.c_double
            lib.rogtk_synth_umis_ascii.argtypes = [u64, _i32, u64, f64, f64, f64, u64, u64, _vp]
            lib.rogtk_synth_umis_ascii.restype = None
            lib.rogtk_synth_umis_codes.argtypes = [u64, _i32, u64, f64, u64, u64, _vp]
            lib.rogtk_synth_umis_codes.restype = ctypes.c_int
            lib.rogtk_synth_reads.argtypes = [u64, _i32, u64, f64, u64, u64, _vp]
            lib.rogtk_synth_reads.restype = None
            lib.rogtk_synth_molecules.argtypes = [u64, u64, u64, u64, _vp]
            lib.rogtk_synth_molecules.restype = None
            _synth = lib
    return _synth


def check(status: int) -> None:
    """Raise RogtkError carrying rogtk_last_error() for a non-zero status."""
    if status != ROGTK_OK:
        msg = hip().rogtk_last_error()
        raise RogtkError(status, msg.decode("utf-8", "replace") if msg else "unknown error")


def call(name: str, *args) -> None:
    check(getattr(hip(), name)(*args))


def version() -> str:
    return hip().rogtk_version().decode()


def device_count() -> int:
    n = ctypes.c_int(0)
    check(hip().rogtk_device_count(ctypes.byref(n)))
    return n.value
