"""Streaming pipeline over packed batches: three HIP streams, `depth` batches in flight.

The hot path has three phases with different limits on MI355X:
  main stream     the local presence bitmap (umi_len 7..13: code slices in LDS, or a
                  partition sort + one LDS bitmap slice per partition; else the
                  XCD-partitioned presence mark + the presence->bitmap pass), then
                  k_score_packed (H1 scores + H2 Hamming): HBM-bandwidth bound
  resolve stream  [RCCL all-gather of the bitmaps] + rank tables + LDS-local and
                  global connected components: latency bound (small tables, many
                  dependent steps)
  assign stream   cluster_id[row] = label(code): random-gather bound
Batch k's resolve overlaps batch k+1's scoring and batch k-1's assign, so a
steady-state step costs max(phase) instead of the sum. Each slot owns its
workspace and outputs; events order every cross-stream hand-off:
  main(k)    waits assign(k - depth) (slot reuse)   -> records marked(k)
  resolve(k) waits marked(k)                         -> records resolved(k)
  assign(k)  waits resolved(k)                       -> records assigned(k)
(reuse_gate="resolve", an A/B option: only resolve(k) waits assign(k - depth) and the
mark waits resolve(k - depth); score, mark, resolve and assign then all overlap, and at
10M reads the step slowed 0.375 -> 0.401 ms: score 119 -> 195 us, assign 125 -> 200 us.)
Resolve is enqueue-only (rogtk_cluster_resolve); assign completes a resolve whose
speculative rounds were not enough, so results never depend on timing.

assign_on="resolve" (option; "separate" is the default): the assign of batch k runs right behind its resolve on
the resolve stream, as a deferred assign (no host wait); the slot's convergence flags
are checked when the slot is reused or at drain(), which re-runs the rounds, labels and
assign on the resolve stream in the rare case the speculative rounds were not enough.
The assign's random gathers then never run beside the next batch's latency-bound
resolve kernels (hook round 0 took 111 us beside assign, 31 us alone), but the host's
wait for batch k-1's flags moves onto the critical cycle: 0.487 vs 0.430 ms/step at 10M.
"""
from __future__ import annotations

from collections import deque
from typing import Optional

import torch

from . import device as D
from .dist import gather_bitmaps
from .dist import collective as dist_collective


_ON_MAIN = object()  # slot.assigned: the assign ran on the main stream, no event recorded


class _Slot:
    def __init__(self, umi_len, max_distinct, n_max, dev, with_scores, with_distance=False):
        self.eng = D.ClusterEngine(umi_len, max_distinct, dev)
        self.scores = D.alloc_scores(n_max, dev) if with_scores else None
        self.within = torch.empty(max((n_max + 63) // 64, 1), dtype=torch.int64, device=dev)
        # H2 hamming_distance_expr column (expressions.rs:1048-1073), when asked
        self.dist = torch.empty(max(n_max, 1), dtype=torch.int32, device=dev) if with_distance else None
        self.cid = torch.empty(max(n_max, 4), dtype=torch.int32, device=dev)
        self.assigned = None  # D.StreamEvent or torch.cuda.Event (UmiPipeline.device_events)
        self.resolved = None
        self.mark_batch = None  # split_mark: the batch whose mark phase 2 is still to enqueue


class UmiPipeline:
    def __init__(self, umi_len: int, max_distinct: int, n_max: int, device=None, depth: int = 3,
                 target: Optional[bytes] = b"ACGTACGTACGT", max_hamming: int = 1, max_distance: int = 1,
                 group=None, with_scores: bool = True, priorities=(0, 0, 0), mark: str = "auto",
                 on_assigned=None, score_alone: bool = False, exchange=None, resolve_streams: int = 1,
                 assign_on: str = "main", reuse_gate: str = "auto", assign_early: bool = True,
                 mark_first: bool = True, device_events: bool = True, mark_stream: bool = False,
                 fused_assign: bool = False, with_distance: bool = False, assign_lag: int = 0,
                 split_mark: bool = True):
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.umi_len, self.max_distance, self.target, self.max_hamming = umi_len, max_distance, target, max_hamming
        self.group = group
        if mark == "auto":  # rogtk_cluster_mark_bitmap where it applies (measured fastest)
            mark = "sort" if 7 <= umi_len <= 13 else "xcd"
        if mark == "slices":  # the method of rogtk_cluster_mark_bitmap is a process-wide knob
            mark = "sort"
        if mark not in ("xcd", "sort"):
            raise ValueError("mark must be 'xcd' (XCD-partitioned mark kernel) or 'sort' (code slices / partition "
                             "sort + LDS bitmap, umi_len 7..13)")
        self.sort_mark = mark == "sort"
        self.slots = [_Slot(umi_len, max_distinct, n_max, dev, with_scores, with_distance) for _ in range(depth)]
        # priorities: (main, resolve, assign); lower = higher priority (torch convention)
        self.caller = torch.cuda.current_stream(dev)
        self.main = torch.cuda.Stream(dev, priority=priorities[0])
        self.main.wait_stream(self.caller)
        # resolve_streams > 1: consecutive batches resolve on different streams, so two
        # latency-bound resolve chains overlap (needs depth >= resolve_streams + 1)
        if resolve_streams < 1 or (resolve_streams > 1 and depth < resolve_streams + 1):
            raise ValueError("resolve_streams must be >= 1 and < depth")
        self.s_resolves = [torch.cuda.Stream(dev, priority=priorities[1]) for _ in range(resolve_streams)]
        self.s_resolve = self.s_resolves[0]
        # assign_on "main": the assign of batch k-1 runs on the main stream right behind
        # batch k's score kernel, so the serial cycle mark -> score -> assign -> mark has
        # no cross-stream hop (each cost ~20-25 us of idle GPU in the round-3 timeline)
        self.s_assign = self.main if assign_on == "main" else torch.cuda.Stream(dev, priority=priorities[2])
        self.queue = deque()
        # assign lags resolve by one batch only when a second slot exists: with one
        # slot the next batch's resolve would overwrite the tables assign reads
        self.lag = resolve_streams if depth > 1 else 0
        # assign_lag > 0: batch k-lag's assign is enqueued at batch k's submit (a longer
        # window for its resolve; needs depth > assign_lag, each slot waits one batch longer)
        if assign_lag:
            if not 0 < assign_lag < depth or assign_lag < resolve_streams:
                raise ValueError("assign_lag must be in [resolve_streams, depth)")
            self.lag = assign_lag
        # on_assigned(slot, batch): called with the assign stream current, after the
        # batch's assign and before its slot may be reused (e.g. to copy outputs out)
        self.on_assigned = on_assigned
        # assign_early: batch k-1's assign is enqueued right after batch k's score kernel
        # (host order), not after batch k's resolve (the host's enqueue of a resolve takes
        # longer than the GPU needs to reach the assign)
        self.assign_early = assign_early
        # mark_first: batch k's presence bitmap (mark) runs before its score kernel on the
        # main stream, so its resolve overlaps the score instead of following it (round 3:
        # 0.367-0.369 vs 0.398-0.408 ms/step at 10M reads, interleaved on one box; the score
        # kernel then also runs beside fewer resolve kernels: 99 vs 130 us). (Round 4 also
        # measured the presence mark fused into the score kernel as byte stores + a bitmap
        # pass: 0.484 vs 0.305 ms/step; removed in round 5. Round 5 measured and removed two
        # more orders: assign(k-1) between mark(k) and score(k), so the local CC runs beside
        # the assign rather than the score kernel, and the mark's slice ranking folded into
        # the score kernel (its segments read back by the slice mark): 0.31-0.32 and
        # 0.346-0.349 vs 0.306 ms/step, the folded score kernel 167 vs 100 us.)
        self.mark_first = mark_first
        # split_mark (round 5): the presence mark's slice-bucket pass stays on the main stream
        # (mark(k) -> score(k)), its slice mark + merge move to the head of the resolve stream:
        # they run beside the score kernel, in the time the resolve would otherwise spend
        # waiting for the score kernel's waves to leave room for its local CC (a 1024-thread
        # workgroup needs 4 waves on every SIMD), so the main chain is ~30 us shorter and the
        # resolve chain is not longer. Applies to the code-slice mark with the default order.
        self.split_mark = bool(split_mark and self.sort_mark and mark_first and assign_on in ("main", "separate")
                               and not mark_stream and not fused_assign)
        # device_events: the cross-stream hand-offs use StreamEvents released at device
        # scope (rogtk_event_*) instead of torch events, whose system-scope release writes
        # the L2 back at every record (round 3: each record / wait between two kernels of
        # the step cost ~20 us of idle GPU in the kernel timeline)
        self.device_events = device_events
        # mark_stream: the presence bitmap of batch k on a stream of its own (it reads only
        # the codes and writes the slot's local bitmap, which nothing but the slot's
        # previous resolve reads), so the main stream carries only score + assign and the
        # mark overlaps them; the resolve then waits for the mark and for the slot's
        # previous assign explicitly
        if mark_stream and assign_on == "resolve":
            raise ValueError("mark_stream needs assign_on != 'resolve'")
        self.s_mark = torch.cuda.Stream(dev, priority=priorities[0]) if mark_stream else self.main
        if mark_stream:
            self.mark_first = True
        # fused_assign: batch k's score kernel runs only after its resolve and also writes
        # its cluster ids (rogtk_umi_score_assign_packed: one pass over the codes instead of
        # a score pass and an assign pass). The main stream then runs mark(k) and
        # score+assign(k - depth + 1), so the resolve of a batch overlaps depth - 1 marks
        # and score+assign passes of earlier batches.
        if fused_assign and (mark_stream or assign_on == "resolve" or depth < 2 or not with_scores):
            raise ValueError("fused_assign needs depth >= 2, scores, the mark on the main stream and "
                             "assign_on != 'resolve'")
        self.fused_assign = fused_assign
        # score_alone: assign of the previous batch waits for this batch's score kernel,
        # so the HBM-bound score overlaps only the latency-bound resolve kernels
        self.score_alone = score_alone
        # exchange(local_bitmap) -> (bitmaps, n): the cross-rank step (default: the
        # all-gather of rogtk_amd.dist); tools may substitute an emulation
        self.exchange = exchange if exchange is not None else (lambda bm: gather_bitmaps(bm, self.group))
        # across ranks the bitmap all-gather runs on its own stream, right behind the mark,
        # so it overlaps the previous batch's resolve instead of lengthening the resolve
        # stream's chain (a substituted exchange may reuse one buffer: it stays in line)
        self.s_comm = torch.cuda.Stream(dev) if exchange is None and dist_collective(group) else None
        if self.s_comm is not None:
            #  with a comm stream the split mark would hold batch k's all-gather
            # behind resolve(k - 1) (phase 2 sits on the resolve stream): the whole mark stays
            # on the main stream, so the all-gather overlaps the previous resolve
            self.split_mark = False
        self.last_scored: Optional[torch.cuda.Event] = None
        self.k = 0
        self.last_assigned: Optional[torch.cuda.Event] = None
        # assign_on "resolve": assign(k) is enqueued right behind resolve(k) on the same
        # stream as a deferred assign (no host wait for the resolve's flags), so it never
        # competes with the latency-bound resolve kernels of the next batch; the flags
        # are checked when the slot comes round again (or at drain)
        if assign_on not in ("resolve", "separate", "main"):
            raise ValueError("assign_on must be 'resolve', 'separate' or 'main'")
        self.assign_on = assign_on
        if assign_on == "resolve" and resolve_streams != 1:
            raise ValueError("assign_on='resolve' uses one resolve stream")
        # reuse_gate: what waits for the assign of the slot's previous batch.
        #   "score":   the main stream (score + mark of batch k wait for assign(k - depth))
        #   "resolve": only the resolve of batch k (its rank / label tables are the ones
        #              assign(k - depth) reads); the mark waits for resolve(k - depth), the
        #              reader of the presence bitmap it overwrites. Score and mark then run
        #              ahead of the assign, off the critical cycle resolve -> assign -> resolve.
        #   "auto":    "score" (measured faster: every kernel here is memory-system bound,
        #              so overlapping all four phases slows each of them more than it hides)
        if reuse_gate not in ("auto", "score", "resolve"):
            raise ValueError("reuse_gate must be 'auto', 'score' or 'resolve'")
        if reuse_gate == "auto":
            reuse_gate = "score"
        if reuse_gate == "resolve" and on_assigned is not None:
            raise ValueError("reuse_gate='resolve' needs on_assigned=None")
        self.reuse_gate = reuse_gate
        # lazy_assigned: with the assign, the mark and the slot-reuse gate all on the main
        # stream, nothing waits for a slot's assign through an event: resolve(k + depth),
        # which rewrites the tables assign(k) reads, waits for mark(k + depth) on the main
        # stream, which the host enqueues after assign(k) because assign lags its batch by
        # `lag` < depth submits. So no event is recorded after the assign (each record or
        # wait on the main stream costs ~12 us of device time in the round-3 timeline); one
        # is recorded on demand by settle(). (Recording every hand-off measured neutral.)
        self.lazy_assigned = (self.s_assign is self.main and self.s_mark is self.main and reuse_gate == "score"
                              and assign_on == "main" and not fused_assign and on_assigned is None)
        if self.lazy_assigned:
            assert self.lag < len(self.slots), "the main stream must order assign(k) before mark(k + depth)"

    def submit(self, batch: D.PackedBatch):
        """Enqueue one batch; returns its slot. Scores and Hamming outputs are valid once the
        slot's events have fired. Cluster ids (slot.cid) are FINAL only after drain(), after
        settle(slot), or inside on_assigned: without on_assigned the assign is deferred and
        may be built from the speculative rounds (slot.assigned / last_assigned mark that
        assign, not a settled one); the slot is settled before its reuse."""
        slot = self.slots[self.k % len(self.slots)]
        producer = torch.cuda.current_stream(self.main.device)  # batch producer -> main
        if producer == self.main or producer.query():
            pass  # nothing pending on the producer: no hand-off (saves an event wait per step)
        elif self.device_events:
            ready = D.StreamEvent()
            ready.record(producer)
            ready.wait(self.main)
            if self.s_mark is not self.main:
                ready.wait(self.s_mark)
        else:
            self.main.wait_stream(producer)
            if self.s_mark is not self.main:
                self.s_mark.wait_stream(producer)
        if self.assign_on == "resolve":
            return self._submit_assign_on_resolve(slot, batch)
        if self.fused_assign:
            return self._submit_fused(slot, batch)
        if self.on_assigned is None:
            self._settle(slot, self.s_assign)
        gate_resolve = self.reuse_gate == "resolve"
        if slot.assigned is not None and not gate_resolve and self.s_assign is not self.main:
            D.wait_for(self.main, slot.assigned)
        if self.mark_first:
            # the presence bitmap needs only the codes: mark first, so the latency-bound
            # resolve of this batch starts while its score kernel streams (host order:
            # mark, score, the previous assign, then the ~15 launches of the resolve, so no
            # GPU queue waits for the host)
            marked = self._mark(slot, batch, gate_resolve)
            self._score(slot, batch)
        else:
            self._score(slot, batch)
            marked = None
        if self.assign_early:
            # the previous batch's assign goes in right behind this batch's score kernel,
            # before the ~20 launches of this batch's mark + resolve: the GPU can start it
            # as soon as its resolve and this score are done instead of waiting for the
            # host to get through this batch's enqueues
            while self.queue and len(self.queue) >= max(self.lag, 1):
                self._assign_oldest()
        if marked is None:
            marked = self._mark(slot, batch, gate_resolve)
        resolved = self._resolve(slot, marked, gate_resolve)
        slot.resolved = resolved
        self.queue.append((slot, batch, resolved))
        if not self.assign_early or self.lag == 0:
            while len(self.queue) > self.lag:
                self._assign_oldest()
        self.k += 1
        return slot

    def _event(self):
        return D.StreamEvent() if self.device_events else torch.cuda.Event()

    def _attach_event(self):
        """An event recorded by a kernel's own dispatch packet (the split mark's bucket pass,
        the resolve's last kernel), which another stream waits for. Created WITHOUT
        hipEventDisableSystemFence: as the stop event of a dispatch, a
        device-scope event may leave the packet without the agent-scope release that makes
        the kernel's L2 lines visible to a consumer on another XCD; interleaved A/B (round 6,
        profiles/r06_event_scope_ab.txt): 0.2843-0.2883 vs 0.2851-0.29 ms/step, sustained equal."""
        if not self.device_events:
            return torch.cuda.Event()
        return D.StreamEvent(device_scope=False)

    def _score(self, slot: _Slot, batch: D.PackedBatch):
        D.score_packed(batch, slot.scores, self.target, self.max_hamming, slot.dist, slot.within, stream=self.main)
        if self.score_alone and self.s_assign is not self.main:
            self.last_scored = self._event()
            self.last_scored.record(self.main)

    def _mark(self, slot: _Slot, batch: D.PackedBatch, gate_resolve: bool):
        """Presence bitmap of the batch on the mark stream (the main stream unless
        mark_stream); returns its event."""
        ms = self.s_mark
        if (gate_resolve or ms is not self.main) and slot.resolved is not None:
            D.wait_for(ms, slot.resolved)  # the previous resolve read the bitmap
        if self.split_mark:  # phase 2 runs at the head of the resolve (_resolve)
            marked = self._attach_event()
            if isinstance(marked, D.StreamEvent):
                # the bucket pass's own dispatch packet records the event (no marker packet
                # between it and the score kernel); disarmed whatever happens
                marked.attach_next()
                try:
                    slot.eng.mark_bitmap(batch, stream=ms, phase=1)
                finally:
                    taken = marked.attach_done()
                if not taken:
                    marked.record(ms)
            else:
                slot.eng.mark_bitmap(batch, stream=ms, phase=1)
                marked.record(ms)
            slot.mark_batch = batch
            return marked
        elif self.sort_mark:
            slot.eng.mark_bitmap(batch, stream=ms)
        else:
            slot.eng.mark(batch, stream=ms)
            slot.eng.build_local_bitmap(stream=ms)
        marked = self._event()
        marked.record(ms)
        return marked

    def _resolve(self, slot: _Slot, marked, gate_resolve: bool):
        """[exchange on the comm stream], the resolve on a resolve stream after `marked`;
        returns the resolve's completion event."""
        sr = self.s_resolves[self.k % len(self.s_resolves)]
        if self.split_mark:  # the rest of the presence mark, at the head of the resolve stream
            with torch.cuda.stream(sr):
                D.wait_for(sr, marked)
                slot.eng.mark_bitmap(slot.mark_batch, stream=sr, phase=2)
                slot.mark_batch = None
                # the resolve below is on this stream: an event only for the comm stream
                marked = None
                if self.s_comm is not None:
                    marked = self._event()
                    marked.record(sr)
        if self.s_comm is not None:
            with torch.cuda.stream(self.s_comm):
                D.wait_for(self.s_comm, marked)
                bitmaps, nb = self.exchange(slot.eng.local_bitmap)
                gathered = self._event()
                gathered.record(self.s_comm)
        with torch.cuda.stream(sr):
            if marked is not None:
                D.wait_for(sr, marked)
            if (gate_resolve or self.s_mark is not self.main) and slot.assigned is not None:
                D.wait_for(sr, slot.assigned)  # assign(k - depth) reads the tables rewritten here
            if self.s_comm is not None:
                D.wait_for(sr, gathered)
                bitmaps.record_stream(sr)  # allocated on the comm stream
            else:
                bitmaps, nb = self.exchange(slot.eng.local_bitmap)
            resolved = self._attach_event()
            if isinstance(resolved, D.StreamEvent):
                # recorded on the resolve's last kernel's dispatch packet
                resolved.attach_next()
                try:
                    slot.eng.resolve(bitmaps, nb, self.max_distance, stream=sr)
                finally:
                    taken = resolved.attach_done()
                if not taken:
                    resolved.record(sr)
            else:
                slot.eng.resolve(bitmaps, nb, self.max_distance, stream=sr)
                resolved.record(sr)
        return resolved

    def _settle(self, slot: _Slot, stream=None):
        """The slot's previous batch is final: its resolve converged (or is completed now,
        with its assign re-run, on `stream`, the stream its assign ran on)."""
        stream = self.s_resolve if stream is None else stream
        if slot.assigned is None:
            return
        if slot.eng.sync(stream=stream):
            slot.assigned = self._event()
            slot.assigned.record(stream)
            self.last_assigned = slot.assigned

    def _submit_assign_on_resolve(self, slot: _Slot, batch: D.PackedBatch):
        self._settle(slot)
        if slot.assigned is not None:
            D.wait_for(self.main, slot.assigned)
        D.score_packed(batch, slot.scores, self.target, self.max_hamming, slot.dist, slot.within, stream=self.main)
        if self.sort_mark:
            slot.eng.mark_bitmap(batch, stream=self.main)
        else:
            slot.eng.mark(batch, stream=self.main)
            slot.eng.build_local_bitmap(stream=self.main)
        marked = self._event()
        marked.record(self.main)
        sr = self.s_resolve
        with torch.cuda.stream(sr):
            D.wait_for(sr, marked)
            bitmaps, nb = self.exchange(slot.eng.local_bitmap)
            slot.eng.resolve(bitmaps, nb, self.max_distance, stream=sr)
            slot.eng.assign(batch, slot.cid, stream=sr, deferred=self.on_assigned is None)
            if self.on_assigned is not None:
                self.on_assigned(slot, batch)
            slot.assigned = self._event()
            slot.assigned.record(sr)
        self.last_assigned = slot.assigned
        self.k += 1
        return slot

    def _submit_fused(self, slot: _Slot, batch: D.PackedBatch):
        # the slot's previous batch (k - depth) had its score+assign enqueued on the main
        # stream in an earlier submit, before this mark: the main stream orders the reuse
        if self.on_assigned is None:
            self._settle(slot, self.main)
        marked = self._mark(slot, batch, False)
        while len(self.queue) >= len(self.slots) - 1:
            self._score_assign_oldest()
        resolved = self._resolve(slot, marked, False)
        slot.resolved = resolved
        self.queue.append((slot, batch, resolved))
        self.k += 1
        return slot

    def _score_assign_oldest(self):
        slot, batch, resolved = self.queue.popleft()
        D.wait_for(self.main, resolved)
        D.score_assign_packed(batch, slot.eng, slot.cid, slot.scores, self.target, self.max_hamming, slot.dist,
                              slot.within, deferred=self.on_assigned is None, stream=self.main)
        if self.on_assigned is not None:
            with torch.cuda.stream(self.main):
                self.on_assigned(slot, batch)
        slot.assigned = self._event()
        slot.assigned.record(self.main)
        self.last_assigned = slot.assigned

    def _assign_oldest(self):
        slot, batch, resolved = self.queue.popleft()
        D.wait_for(self.s_assign, resolved)
        if self.score_alone and self.last_scored is not None and self.s_assign is not self.main:
            D.wait_for(self.s_assign, self.last_scored)
        # without a consumer hook the assign is deferred (no host wait for the resolve's
        # flags: the host would otherwise stall behind the resolve stream's queue and
        # enqueue the next batch late); the slot is settled before its reuse / at drain
        slot.eng.assign(batch, slot.cid, stream=self.s_assign, deferred=self.on_assigned is None)
        if self.on_assigned is not None:
            with torch.cuda.stream(self.s_assign):
                self.on_assigned(slot, batch)
        if self.lazy_assigned:
            slot.assigned = _ON_MAIN  # ordered by the main stream; an event only on demand
            self.last_assigned = None
            return
        slot.assigned = self._event()
        slot.assigned.record(self.s_assign)
        self.last_assigned = slot.assigned

    def settle(self, slot):
        """Make slot.cid final now (enqueues the slot's assign if it is still queued, waits
        for its resolve's flags, re-runs the rounds, labels and assign in the rare
        non-converged case); the current stream then waits for it. Returns slot.cid."""
        while any(q[0] is slot for q in self.queue):
            self._score_assign_oldest() if self.fused_assign else self._assign_oldest()
        self._settle(slot, self.s_assign if self.assign_on != "resolve" else None)
        if slot.assigned is _ON_MAIN:
            slot.assigned = self._event()
            slot.assigned.record(self.main)
        if slot.assigned is not None:
            D.wait_for(torch.cuda.current_stream(self.main.device), slot.assigned)
        return slot.cid

    def drain(self):
        """Finish every submitted batch; the main stream waits for the last assign."""
        if self.assign_on == "resolve":
            for slot in self.slots:
                self._settle(slot)
        while self.queue:
            self._score_assign_oldest() if self.fused_assign else self._assign_oldest()
        if self.assign_on != "resolve" and self.on_assigned is None:
            for slot in self.slots:
                self._settle(slot, self.s_assign)
        if self.last_assigned is not None:
            D.wait_for(self.main, self.last_assigned)
        torch.cuda.current_stream(self.main.device).wait_stream(self.main)
