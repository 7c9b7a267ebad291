"""Device-resident pipeline over the packed 2-bit SoA (level-1 C ABI).

PyTorch is only plumbing here: tensors provide HBM allocations and the HIP
stream (torch's current stream) whose handle is passed through the C ABI; every
byte of compute happens in librogtk_hip's kernels.

Layout in HBM for a batch of n reads (DESIGN.md §Data layout):
  codes         uint32[n]        2 bits/base, first base most significant
  regular_bits  uint64[ceil(n/64)]  row is packable (else: byte path / null)
  scores        6 x float64[n] + uint32[n]   (SoA, one array per field)
  hamming       uint32[n] distance and/or uint64[ceil(n/64)] within bits
  cluster_id    uint32[n]
  cluster ws    presence u8[4^L] | bitmap u64[4^L/64] | rank tables | D/parent u32[max_distinct] | labels
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib

_FIELDS = ("shannon_entropy", "linguistic_complexity", "homopolymer_fraction",
           "dinucleotide_entropy", "longest_homopolymer_run", "dust_score", "combined_score")


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _s(stream: Optional[torch.cuda.Stream] = None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class StreamEvent:
    """Stream-ordering event (rogtk_event_*): never timed; device_scope=True releases at
    device scope only, so a record does not write the L2 back to memory (torch's events
    release at system scope). Same record / wait / synchronize / query shape as
    torch.cuda.Event, for the pipeline's cross-stream hand-offs."""

    __slots__ = ("_ev",)

    def __init__(self, device_scope: bool = True):
        h = ctypes.c_void_p()
        _lib.call("rogtk_event_create", 1 if device_scope else 0, ctypes.byref(h))
        self._ev = h

    def record(self, stream: Optional[torch.cuda.Stream] = None):
        _lib.call("rogtk_event_record", self._ev, _s(stream))

    def attach_next(self):
        """Record this event on the dispatch packet of the next kernel this thread launches
        through the library (no marker packet of its own); attach_done() says whether one
        did, and disarms."""
        _lib.call("rogtk_event_attach_next", self._ev)

    def attach_done(self) -> bool:
        taken = ctypes.c_int32(0)
        _lib.call("rogtk_event_attach_done", ctypes.byref(taken))
        return bool(taken.value)

    def wait(self, stream: Optional[torch.cuda.Stream] = None):
        """`stream` waits for this event's last record."""
        _lib.call("rogtk_stream_wait_event", _s(stream), self._ev)

    def query(self) -> bool:
        done = ctypes.c_int32(0)
        _lib.call("rogtk_event_query", self._ev, ctypes.byref(done))
        return bool(done.value)

    def synchronize(self):
        _lib.call("rogtk_event_synchronize", self._ev)

    def __del__(self):
        ev = getattr(self, "_ev", None)
        if ev is not None and ev.value:
            try:
                _lib.call("rogtk_event_destroy", ev)
            except Exception:  # interpreter shutdown
                pass
            self._ev = None


def wait_for(stream: torch.cuda.Stream, ev) -> None:
    """`stream` waits for `ev` (a StreamEvent or a torch.cuda.Event)."""
    if isinstance(ev, StreamEvent):
        ev.wait(stream)
    else:
        stream.wait_event(ev)


class PackedBatch:
    """The packed SoA of one batch (device tensors)."""

    def __init__(self, codes: torch.Tensor, umi_len: int, regular_bits: Optional[torch.Tensor] = None):
        if codes.dtype != torch.int32 or not codes.is_cuda or not codes.is_contiguous():
            raise TypeError("codes must be a contiguous int32 (bit pattern of uint32) CUDA tensor")
        if not 1 <= umi_len <= 16:
            raise ValueError("packed path supports umi_len 1..16")
        self.codes = codes
        self.umi_len = int(umi_len)
        self.regular_bits = regular_bits
        self.n = codes.numel()


def alloc_scores(n: int, device, fields=_FIELDS) -> Dict[str, torch.Tensor]:
    out = {}
    for f in fields:
        dt = torch.int32 if f == "longest_homopolymer_run" else torch.float64
        out[f] = torch.empty(max(n, 4), dtype=dt, device=device)
    return out


def _scores_struct(scores: Optional[Dict[str, torch.Tensor]]):
    if not scores:
        return None
    return ctypes.byref(_lib.UmiScores(*[_p(scores.get(f)) for f in _FIELDS]))


def stage_strings(offsets: torch.Tensor, values: torch.Tensor, n: int, umi_len: int,
                  validity: Optional[torch.Tensor] = None, validity_offset: int = 0, stream=None):
    """Arrow strings already in HBM -> (PackedBatch, irregular_rows int64[n], n_irregular int64[1])."""
    dev = offsets.device
    codes = torch.empty(max(n, 4), dtype=torch.int32, device=dev)
    regbits = torch.empty(max((n + 63) // 64, 1), dtype=torch.int64, device=dev)
    irr = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    nirr = torch.zeros(1, dtype=torch.int64, device=dev)
    ow = offsets.element_size()
    _lib.call("rogtk_stage_strings", _p(offsets), ow, _p(values), _p(validity), validity_offset, n, umi_len,
              _p(codes), _p(regbits), _p(irr), _p(nirr), _s(stream))
    batch = PackedBatch(codes[:n] if n else codes[:0], umi_len if 1 <= umi_len <= 16 else 16, regbits)
    batch.n = n
    return batch, irr, nirr


def score_packed(batch: PackedBatch, scores: Optional[Dict[str, torch.Tensor]] = None,
                 target: Optional[bytes] = None, max_distance: int = 1,
                 hamming_distance: Optional[torch.Tensor] = None,
                 hamming_within_bits: Optional[torch.Tensor] = None, stream=None) -> None:
    """The fused hot kernel: H1 scores + H2 Hamming in one pass over the codes."""
    t = None
    tl = 0
    if target is not None:
        tb = target.encode() if isinstance(target, str) else bytes(target)
        t = ctypes.create_string_buffer(tb, max(len(tb), 1))
        tl = len(tb)
    _lib.call("rogtk_umi_score_packed", _p(batch.codes), _p(batch.regular_bits), batch.n, batch.umi_len,
              _scores_struct(scores), t, tl, max_distance, _p(hamming_distance), _p(hamming_within_bits), _s(stream))


def score_assign_packed(batch: PackedBatch, engine: "ClusterEngine", cluster_id: torch.Tensor,
                        scores: Optional[Dict[str, torch.Tensor]] = None, target: Optional[bytes] = None,
                        max_distance: int = 1, hamming_distance: Optional[torch.Tensor] = None,
                        hamming_within_bits: Optional[torch.Tensor] = None, deferred: bool = False,
                        stream=None) -> None:
    """score_packed + engine.assign(batch, cluster_id) in one pass over the codes (the
    engine's resolve must have been enqueued; deferred as in ClusterEngine.assign)."""
    t = None
    tl = 0
    if target is not None:
        tb = target.encode() if isinstance(target, str) else bytes(target)
        t = ctypes.create_string_buffer(tb, max(len(tb), 1))
        tl = len(tb)
    if cluster_id.dtype != torch.int32 or cluster_id.numel() < batch.n or not cluster_id.is_contiguous():
        raise ValueError("cluster_id: contiguous int32 with >= n elements")
    _lib.call("rogtk_umi_score_assign_packed", _p(batch.codes), _p(batch.regular_bits), batch.n, batch.umi_len,
              _scores_struct(scores), t, tl, max_distance, _p(hamming_distance), _p(hamming_within_bits),
              _p(engine.ws), engine.max_distinct, _p(cluster_id), 1 if deferred else 0, _s(stream))


def score_rows(offsets: torch.Tensor, values: torch.Tensor, rows: torch.Tensor,
               n_rows_dev: Optional[torch.Tensor], max_rows: int, max_len: int,
               scores: Optional[Dict[str, torch.Tensor]] = None, target: Optional[bytes] = None,
               max_distance: int = 1, hamming_distance=None, hamming_within_bits=None, stream=None):
    """Byte path for listed rows (irregular UMIs) of a device Arrow string column."""
    t = None
    tl = 0
    if target is not None:
        tb = target.encode() if isinstance(target, str) else bytes(target)
        t = ctypes.create_string_buffer(tb, max(len(tb), 1))
        tl = len(tb)
    _lib.call("rogtk_umi_score_rows", _p(offsets), offsets.element_size(), _p(values), _p(rows),
              _p(n_rows_dev), max_rows, max_len, _scores_struct(scores), t, tl, max_distance,
              _p(hamming_distance), _p(hamming_within_bits), _s(stream))


class ClusterEngine:
    """H3 over the packed SoA: workspace + the mark/bitmap/resolve/assign phases."""

    def __init__(self, umi_len: int, max_distinct: int, device, stream=None):
        self.umi_len = int(umi_len)
        self.max_distinct = int(min(max_distinct, 4 ** self.umi_len))
        nbytes = ctypes.c_int64(0)
        _lib.call("rogtk_cluster_workspace_size", self.umi_len, self.max_distinct, ctypes.byref(nbytes))
        words = ctypes.c_int64(0)
        _lib.call("rogtk_cluster_bitmap_words", self.umi_len, ctypes.byref(words))
        self.words = int(words.value)
        self.ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=device)
        self.local_bitmap = torch.empty(self.words, dtype=torch.int64, device=device)
        _lib.call("rogtk_cluster_init", _p(self.ws), self.umi_len, self.max_distinct, _s(stream))

    def __del__(self):
        try:
            _lib.call("rogtk_cluster_release", _p(self.ws))
        except Exception:
            pass

    @property
    def workspace_bytes(self) -> int:
        return self.ws.numel()

    def mark(self, batch: PackedBatch, stream=None) -> None:
        _lib.call("rogtk_cluster_mark", _p(batch.codes), _p(batch.regular_bits), batch.n, self.umi_len,
                  _p(self.ws), self.max_distinct, _s(stream))

    def mark_temp(self, n: int) -> torch.Tensor:
        """The scratch of mark_bitmap for n rows (kept, grown on demand)."""
        need = ctypes.c_int64(0)
        _lib.call("rogtk_cluster_mark_bitmap_temp_bytes", n, self.umi_len, ctypes.byref(need))
        if getattr(self, "_mark_temp", None) is None or self._mark_temp.numel() < need.value:
            self._mark_temp = torch.empty(need.value, dtype=torch.uint8, device=self.local_bitmap.device)
        return self._mark_temp

    def mark_bitmap(self, batch: PackedBatch, stream=None, phase: int = 0):
        """mark + build_local_bitmap in one: code slices or partition sort + LDS bitmap
        (7 <= L <= 13). Returns local_bitmap. phase 1 / 2: the slice-bucket pass / the rest
        (rogtk_cluster_mark_bitmap_phase), the caller ordering 2 after 1."""
        self.mark_temp(batch.n)
        if phase:
            _lib.call("rogtk_cluster_mark_bitmap_phase", _p(batch.codes), _p(batch.regular_bits), batch.n,
                      self.umi_len, _p(self.local_bitmap), _p(self._mark_temp), self._mark_temp.numel(), int(phase),
                      _s(stream))
        else:
            _lib.call("rogtk_cluster_mark_bitmap", _p(batch.codes), _p(batch.regular_bits), batch.n, self.umi_len,
                      _p(self.local_bitmap), _p(self._mark_temp), self._mark_temp.numel(), _s(stream))
        return self.local_bitmap

    def build_local_bitmap(self, stream=None) -> torch.Tensor:
        _lib.call("rogtk_cluster_local_bitmap", _p(self.ws), self.umi_len, self.max_distinct,
                  _p(self.local_bitmap), _s(stream))
        return self.local_bitmap

    def resolve(self, bitmaps: torch.Tensor, n_bitmaps: int, max_distance: int, stream=None) -> None:
        """Rank tables, components and labels of the OR of n_bitmaps bitmaps (enqueue-only)."""
        if bitmaps.numel() != n_bitmaps * self.words:
            raise ValueError("bitmaps must hold n_bitmaps * words int64 words")
        _lib.call("rogtk_cluster_resolve", _p(self.ws), self.umi_len, self.max_distinct, _p(bitmaps),
                  int(n_bitmaps), int(max_distance), _s(stream))

    def assign(self, batch: PackedBatch, cluster_id: torch.Tensor, stream=None, deferred: bool = False) -> None:
        """cluster ids of the batch's rows. deferred=True: no host wait for the resolve's
        convergence flags; sync() before reading cluster_id re-runs it if needed."""
        fn = "rogtk_cluster_assign_deferred" if deferred else "rogtk_cluster_assign"
        _lib.call(fn, _p(self.ws), self.umi_len, self.max_distinct, _p(batch.codes), _p(batch.regular_bits),
                  batch.n, _p(cluster_id), _s(stream))

    def sync(self, stream=None) -> bool:
        """Completes the pending resolve (+ deferred assign) on `stream`; True when that
        enqueued more work (the speculative rounds were not enough)."""
        redone = ctypes.c_int(0)
        _lib.call("rogtk_cluster_sync", _p(self.ws), _s(stream), ctypes.byref(redone))
        return bool(redone.value)

    def stats(self, stream=None) -> Dict[str, int]:
        out = (ctypes.c_int64 * 4)()
        _lib.call("rogtk_cluster_stats", _p(self.ws), self.umi_len, self.max_distinct, out, _s(stream))
        return {"n_distinct": out[0], "n_clusters": out[1], "overflow": out[2], "error": out[3]}

    def rounds(self, stream=None) -> int:
        """Global hook rounds the last resolve needed (diagnostics)."""
        r = ctypes.c_int(0)
        _lib.call("rogtk_cluster_rounds", _p(self.ws), _s(stream), ctypes.byref(r))
        return r.value


def set_spec_rounds(n: int) -> None:
    """Hook rounds launched speculatively per resolve (0 = default 4); results never change."""
    _lib.call("rogtk_cluster_set_spec_rounds", int(n))


def set_lookback_polls(n: int) -> None:
    """Look-back polls of the single-pass rank-table scan before a block recounts its
    prefix from the bitmaps (-1 = default; 0 forces the recount); results never change."""
    _lib.call("rogtk_cluster_set_lookback_polls", int(n))


MARK_AUTO, MARK_SORT, MARK_SLICES = 0, 1, 2


def set_mark_method(method: int) -> None:
    """mark_bitmap method: 0 auto (LDS code slices for umi_len <= 12, partition sort for 13),
    1 partition sort, 2 code slices; identical bitmaps."""
    _lib.call("rogtk_cluster_set_mark_method", int(method))


def cluster_batch(engine: ClusterEngine, batch: PackedBatch, cluster_id: torch.Tensor,
                  max_distance: int = 1, group=None, marked: bool = False, stream=None) -> None:
    """mark -> local bitmap -> (all-gather over ranks) -> resolve -> assign."""
    from .dist import gather_bitmaps

    if not marked and 7 <= batch.umi_len <= 13:  # the presence bitmap in one call (code slices / sort)
        local = engine.mark_bitmap(batch, stream)
    else:
        if not marked:
            engine.mark(batch, stream)
        local = engine.build_local_bitmap(stream)
    bitmaps, nb = gather_bitmaps(local, group)
    engine.resolve(bitmaps, nb, max_distance, stream)
    engine.assign(batch, cluster_id, stream)


def group_by_key(keys: torch.Tensor, stream=None):
    """polars group_by on the device (e.g. H3 cluster ids, int32/uint32 tensor):
    returns (rows int64[n] ordered by key (stable), group_offsets int64[G + 1], G)."""
    n = keys.numel()
    rows = torch.empty(max(n, 1), dtype=torch.int64, device=keys.device)
    go = torch.empty(n + 1, dtype=torch.int64, device=keys.device)
    ng = ctypes.c_int64(0)
    _lib.call("rogtk_group_by_key", _p(keys), n, _p(rows), _p(go), ctypes.byref(ng), _s(stream))
    G = int(ng.value)
    return rows[:n], go[:G + 1] if n else go[:1].zero_(), G


def kmer_spectrum_dev(offsets: torch.Tensor, values: torch.Tensor, group_offsets: torch.Tensor, k: int,
                      min_coverage: int, capacity: int, rows: Optional[torch.Tensor] = None,
                      validity: Optional[torch.Tensor] = None, validity_offset: int = 0, stream=None):
    """H4 on a device-resident column (int64 offsets, uint8 values). Returns a dict of
    device tensors: kmers (int64 [m, 2]: hi, lo words), exts (uint8), counts (int16 bits
    of u16), entry_offsets (int64 G + 1), stats (int64 G x 5)."""
    dev = values.device
    G = group_offsets.numel() - 1
    n_rows = rows.numel() if rows is not None else offsets.numel() - 1
    cap = max(int(capacity), 1)
    km = torch.empty((cap, 2), dtype=torch.int64, device=dev)
    ex = torch.empty(cap, dtype=torch.uint8, device=dev)
    cn = torch.empty(cap, dtype=torch.int16, device=dev)
    eo = torch.empty(G + 1, dtype=torch.int64, device=dev)
    st = torch.empty((G, 5), dtype=torch.int64, device=dev)
    m = ctypes.c_int64(0)
    _lib.call("rogtk_kmer_spectrum_dev", _p(offsets), _p(values), _p(validity), int(validity_offset), _p(rows),
              n_rows, _p(group_offsets), G, int(k), int(min_coverage), cap, _p(km), _p(ex), _p(cn), _p(eo),
              _p(st), ctypes.byref(m), _s(stream))
    n = int(m.value)
    return {"kmers": km[:n], "exts": ex[:n], "counts": cn[:n], "entry_offsets": eo, "stats": st}


def max_row_len(offsets: torch.Tensor, stream=None) -> int:
    """The longest row of an int64-offsets column (rogtk_max_row_len: a reduction kernel and
    one 8-byte read)."""
    m = ctypes.c_int64(0)
    _lib.call("rogtk_max_row_len", _p(offsets), max(offsets.numel() - 1, 0), ctypes.byref(m), _s(stream))
    return int(m.value)


def kmer_spectrum_fused(offsets: torch.Tensor, values: torch.Tensor, group_offsets: torch.Tensor, k: int,
                        min_coverage: int, capacity: int, max_len: int, rows: Optional[torch.Tensor] = None,
                        validity: Optional[torch.Tensor] = None, validity_offset: int = 0, stream=None):
    """kmer_spectrum_dev with the grouped rows packed straight from their ASCII bytes
    (rogtk_kmer_spectrum_fused; rows of at most 224 bases): same outputs, bit-exact."""
    dev = values.device
    G = group_offsets.numel() - 1
    n_rows = rows.numel() if rows is not None else offsets.numel() - 1
    cap = max(int(capacity), 1)
    km = torch.empty((cap, 2), dtype=torch.int64, device=dev)
    ex = torch.empty(cap, dtype=torch.uint8, device=dev)
    cn = torch.empty(cap, dtype=torch.int16, device=dev)
    eo = torch.empty(G + 1, dtype=torch.int64, device=dev)
    st = torch.empty((G, 5), dtype=torch.int64, device=dev)
    m = ctypes.c_int64(0)
    _lib.call("rogtk_kmer_spectrum_fused", _p(offsets), _p(values), values.numel(), _p(validity),
              int(validity_offset), _p(rows), n_rows, _p(group_offsets), G, int(k), int(min_coverage), cap, _p(km),
              _p(ex), _p(cn), _p(eo), _p(st), ctypes.byref(m), int(max_len), offsets.numel() - 1, _s(stream))
    n = int(m.value)
    return {"kmers": km[:n], "exts": ex[:n], "counts": cn[:n], "entry_offsets": eo, "stats": st}


class PackedReads:
    """A read column as fixed-size 2-bit blocks in HBM (rogtk_pack_reads): block_words u64
    per row (meta + bases), so a grouped row is staged as whole 64-B lines."""

    # the block size packed first when the caller gives no bound (rows up to 224 bases, the
    # short-read case); a column with longer rows is packed again at its own size
    GUESS_LEN = 224

    def __init__(self, offsets: torch.Tensor, values: torch.Tensor, validity: Optional[torch.Tensor] = None,
                 validity_offset: int = 0, max_len: Optional[int] = None, stream=None):
        n = offsets.numel() - 1
        self.n = n
        # the longest row comes out of the pack kernel itself (a per-wave reduction into one
        # device word; no separate pass over the offsets, no torch kernel); read back once
        self._max_dev = torch.empty(1, dtype=torch.int64, device=values.device)
        guess = self.GUESS_LEN if max_len is None else int(max_len)
        self._pack(offsets, values, validity, validity_offset, guess, stream)
        if max_len is None:
            got = 0
            if n:  # one 8-byte read, ordered after the pack on its stream
                with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream()):
                    got = int(self._max_dev.cpu()[0])
            if got > (self.block_words - 1) * 32:  # a row did not fit the guessed blocks
                self._pack(offsets, values, validity, validity_offset, got, stream)
            self.max_len = got
        else:
            self.max_len = int(max_len)

    def _pack(self, offsets, values, validity, validity_offset, max_len, stream):
        self.block_words = int(_lib.hip().rogtk_read_block_words(int(max_len)))
        if self.block_words == 0:
            raise ValueError(f"reads up to {max_len} bases: too long for the block layout (max 992)")
        self.blocks = torch.empty(max(self.n * self.block_words, 1), dtype=torch.int64, device=values.device)
        _lib.call("rogtk_pack_reads", _p(offsets), _p(values), _p(validity), int(validity_offset), self.n,
                  self.block_words, _p(self.blocks), _p(self._max_dev), _s(stream))


def kmer_spectrum_blocks(packed: PackedReads, offsets: torch.Tensor, values: torch.Tensor,
                         group_offsets: torch.Tensor, k: int, min_coverage: int, capacity: int,
                         rows: Optional[torch.Tensor] = None, validity: Optional[torch.Tensor] = None,
                         validity_offset: int = 0, stream=None):
    """kmer_spectrum_dev over a PackedReads column (same outputs, bit-exact)."""
    dev = values.device
    G = group_offsets.numel() - 1
    n_rows = rows.numel() if rows is not None else offsets.numel() - 1
    cap = max(int(capacity), 1)
    km = torch.empty((cap, 2), dtype=torch.int64, device=dev)
    ex = torch.empty(cap, dtype=torch.uint8, device=dev)
    cn = torch.empty(cap, dtype=torch.int16, device=dev)
    eo = torch.empty(G + 1, dtype=torch.int64, device=dev)
    st = torch.empty((G, 5), dtype=torch.int64, device=dev)
    m = ctypes.c_int64(0)
    _lib.call("rogtk_kmer_spectrum_blocks", _p(packed.blocks), packed.block_words, packed.max_len, _p(offsets),
              _p(values), _p(validity), int(validity_offset), _p(rows), n_rows, _p(group_offsets), G, int(k),
              int(min_coverage), cap, _p(km), _p(ex), _p(cn), _p(eo), _p(st), ctypes.byref(m), _s(stream))
    n = int(m.value)
    return {"kmers": km[:n], "exts": ex[:n], "counts": cn[:n], "entry_offsets": eo, "stats": st}


def group_spectra(offsets: torch.Tensor, values: torch.Tensor, keys: torch.Tensor, k: int, min_coverage: int,
                  batch_rows: int = 100_000_000, consume=None, stream=None, packed="auto",
                  max_len: Optional[int] = None):
    """The C3 front end after H3 (rogtk/__init__.py:206-214: group_by('umi') then
    assemble per group): rows grouped by key (stable; e.g. H3 cluster ids), then k-mer
    spectra (filter_kmers + CountFilter + censored exts, fracture.rs:105-116) over runs of
    consecutive groups of at most batch_rows rows per call (a group is never split; a
    larger group gets a call of its own). Output capacity per call = its rows x
    max(0, longest row - 3) / max(min_coverage, 1): every valid k-mer takes at least
    min_coverage of the call's observations.
    Returns (rows int64[n] in group order, group_offsets int64[G + 1], G, calls): with
    consume=None, calls lists (g0, g1, result) per call, each result (kmer_spectrum_dev's
    dict for groups g0..g1-1) copied to its own size so the next call can reuse the
    capacity; else consume(g0, g1, result) is called per call (the result's buffers are
    reused afterwards) and calls is empty.
    packed: "auto" stages every call's grouped rows straight from their ASCII bytes with
    the 2-bit packing and repeat certificate fused in (kmer_spectrum_fused, round 5) when the
    rows fit 224 bases, else packs the column once into 2-bit blocks (PackedReads) that every
    call stages from; "fused" / "blocks" force one of the two; a PackedReads to reuse; None
    for the ASCII staging path (no certificate). max_len: a bound on the rows' lengths the
    caller knows (e.g. the sequencer's read length; rows past it fail the call on the device
    check), else the longest row is found by a reduction kernel (one 8-byte read)."""
    if isinstance(packed, PackedReads):
        max_len = packed.max_len
    elif max_len is None:  # the longest row by a reduction kernel (no torch kernel, one 8-byte read)
        max_len = max_row_len(offsets, stream=stream)
    if isinstance(packed, str):
        mode = ("fused" if max_len <= 224 and values.data_ptr() % 16 == 0 else "blocks") if packed == "auto" \
            else packed
        if mode not in ("fused", "blocks"):
            raise ValueError("packed must be 'auto', 'fused', 'blocks', a PackedReads or None")
        packed = "fused"
        if mode == "blocks":
            try:
                packed = PackedReads(offsets, values, max_len=max_len, stream=stream)
            except ValueError:
                packed = None
    rows, go, G = group_by_key(keys, stream=stream)
    if G == 0:
        return rows, go, G, []
    # output capacity per call: rows x (longest row - 3) bounds the valid entries (each
    # row adds at most len - 3 k-mers, k_eff >= 4)
    per_row = max(0, max_len - 3)
    n_grouped = rows.numel()
    if n_grouped <= batch_rows:  # one call: no copy of the group offsets to the host
        cuts, bounds = [0, G], {0: 0, G: n_grouped}
    else:
        goh = go.cpu().numpy()
        cuts = [0]
        while cuts[-1] < G:
            g0 = cuts[-1]
            g1 = int(np.searchsorted(goh, goh[g0] + batch_rows, side="right")) - 1
            cuts.append(min(G, max(g1, g0 + 1)))
        bounds = {g: int(goh[g]) for g in cuts}
    calls = []
    for g0, g1 in zip(cuts, cuts[1:]):
        a, b = bounds[g0], bounds[g1]
        r = rows[a:b]
        cap = (b - a) * per_row // max(int(min_coverage), 1)
        if packed == "fused":
            res = kmer_spectrum_fused(offsets, values, go[g0:g1 + 1] - a, k, min_coverage, cap, max_len, rows=r,
                                      stream=stream)
        elif packed is not None:
            res = kmer_spectrum_blocks(packed, offsets, values, go[g0:g1 + 1] - a, k, min_coverage, cap, rows=r,
                                       stream=stream)
        else:
            res = kmer_spectrum_dev(offsets, values, go[g0:g1 + 1] - a, k, min_coverage, cap, rows=r, stream=stream)
        if consume is not None:
            consume(g0, g1, res)
        else:
            calls.append((g0, g1, {key: t.clone() for key, t in res.items()}))
        del res
    return rows, go, G, calls


def profile_enable(on: bool = True) -> None:
    _lib.call("rogtk_profile_enable", 1 if on else 0)


def profile_select(kernel: str | None = None) -> None:
    """Bracket only `kernel`'s launches with events (None: every kernel)."""
    _lib.call("rogtk_profile_select", (kernel or "").encode())


def profile_reset() -> None:
    _lib.call("rogtk_profile_reset")


def profile_read(kernel: str):
    ms = ctypes.c_double(0)
    n = ctypes.c_int64(0)
    _lib.call("rogtk_profile_read", kernel.encode(), ctypes.byref(ms), ctypes.byref(n))
    return ms.value, n.value


def profile_read_span(kernel: str):
    """(total ms, launches) of the kernel's own execution spans (in-kernel clocks; the
    kernels that support it: score_packed)."""
    ms = ctypes.c_double(0)
    n = ctypes.c_int64(0)
    _lib.call("rogtk_profile_read_span", kernel.encode(), ctypes.byref(ms), ctypes.byref(n))
    return ms.value, n.value
