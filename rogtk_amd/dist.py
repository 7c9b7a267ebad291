"""Multi-GPU exchange for H3 and H4 (one process per GPU, torch.distributed).

Reads shard by record; H1/H2 need no exchange. H3 needs the global set of
distinct UMIs: every rank publishes its 4^L-bit presence bitmap (2 MiB at L=12)
with ONE all-gather (RCCL over xGMI with backend "nccl"; gloo on CPU for tests),
then every rank resolves the same global components redundantly inside
rogtk_cluster_resolve (which ORs the gathered bitmaps while it scans them), so
cluster ids are bit-identical for 1, 2, 4 or 8 GPUs with no second exchange.

An all-gather of N bitmaps moves (N-1)/N * N * 2 MiB per rank; a ring all-reduce
would need a bitwise-OR reduction RCCL does not offer, and a byte-wise MAX on a
4^L-byte table moves 8x the bytes.

H4 (k-mer spectra per UMI group) needs each group's reads on one rank: route_rows
packs the rows by owner rank on the device (rogtk_route_pack) and moves them with
one all-to-all of bytes plus three small all-to-alls of per-row metadata.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def collective(group=None) -> bool:
    """A process group exists: the exchanges go through it (RCCL with backend "nccl"),
    at world 1 too (tests/test_gpu_rccl.py runs the whole RCCL call sequence that way)."""
    return dist.is_available() and dist.is_initialized()


def world(group=None) -> int:
    if not collective(group):
        return 1
    return dist.get_world_size(group)


def gather_bitmaps(local: torch.Tensor, group=None):
    """All-gather one bitmap per rank into a [world * words] tensor (rank-major)."""
    if not collective(group):
        return local, 1
    n = world(group)
    out = torch.empty(n * local.numel(), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local, group=group)
    elif local.is_cuda:  # gloo with device tensors (multi-rank rehearsal on one GPU): stage via host
        host = torch.empty(n * local.numel(), dtype=local.dtype)
        dist.all_gather(list(host.chunk(n)), local.cpu(), group=group)
        out.copy_(host)
    else:
        dist.all_gather(list(out.chunk(n)), local, group=group)
    return out, n


def shard_range(n_total: int, rank: int, world_size: int):
    """Contiguous record range of one rank (weak or strong scaling alike)."""
    per = n_total // world_size
    rem = n_total % world_size
    start = rank * per + min(rank, rem)
    return start, per + (1 if rank < rem else 0)


def route_destination(keys: torch.Tensor, world_size: int) -> torch.Tensor:
    """Owner rank of each row's group key (int32): a multiplicative hash of the key mod
    world, so one cluster's reads land on one rank and ranks get balanced shares."""
    k = keys.to(torch.int64) & 0xFFFFFFFF
    return (((k * 2654435761) & 0xFFFFFFFF) % world_size).to(torch.int32)


def _pack(offsets: torch.Tensor, values: torch.Tensor, dest: torch.Tensor, world_size: int):
    """Rows by destination: (perm, counts[W], byte_counts[W], packed offsets, packed values).
    Device tensors go through rogtk_route_pack (HIP); CPU tensors (gloo rehearsals on
    hosts without a GPU) through the same stable counting sort in torch."""
    n = dest.numel()
    if offsets.is_cuda:
        import ctypes

        from . import _lib
        perm = torch.empty(max(n, 1), dtype=torch.int64, device=offsets.device)
        poff = torch.empty(n + 1, dtype=torch.int64, device=offsets.device)
        total = int(offsets[-1].item()) - int(offsets[0].item()) if n else 0
        pval = torch.empty(max(total, 1), dtype=torch.uint8, device=offsets.device)
        cnt = (ctypes.c_int64 * world_size)()
        bcnt = (ctypes.c_int64 * world_size)()
        _lib.call("rogtk_route_pack", ctypes.c_void_p(offsets.data_ptr()), ctypes.c_void_p(values.data_ptr()),
                  ctypes.c_void_p(dest.data_ptr()), n, world_size, ctypes.c_void_p(perm.data_ptr()), cnt, bcnt,
                  ctypes.c_void_p(poff.data_ptr()), ctypes.c_void_p(pval.data_ptr()), max(total, 1),
                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        return perm[:n], list(cnt), list(bcnt), poff, pval[:total]
    perm = torch.sort(dest.to(torch.int64), stable=True).indices
    lens = offsets[1:] - offsets[:-1]
    counts = torch.bincount(dest.to(torch.int64), minlength=world_size)
    bcounts = torch.zeros(world_size, dtype=torch.int64).index_add_(0, dest.to(torch.int64), lens)
    plens = lens[perm]
    poff = torch.zeros(n + 1, dtype=torch.int64)
    poff[1:] = torch.cumsum(plens, 0)
    starts = offsets[:-1][perm]
    idx = torch.repeat_interleave(starts - poff[:-1], plens) + torch.arange(int(poff[-1]), dtype=torch.int64)
    return perm, counts.tolist(), bcounts.tolist(), poff, values[idx]


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None):
    if dist.get_backend(group) != "nccl" and inp.is_cuda:  # gloo rehearsal with device tensors: stage on host
        host_out = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(host_out, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(host_out)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def route_rows(offsets: torch.Tensor, values: torch.Tensor, keys: torch.Tensor, group=None):
    """One all-to-all that co-locates every group: row i of this rank's string column
    (int64 offsets from 0, uint8 values) with group key keys[i] goes to rank
    route_destination(key). Returns (offsets, values, keys, src_rank, src_row) of the rows
    this rank now owns, ordered by source rank then source row."""
    W = world(group)
    n = keys.numel()
    if not collective(group):
        dev = keys.device
        return (offsets, values, keys, torch.zeros(n, dtype=torch.int32, device=dev),
                torch.arange(n, dtype=torch.int64, device=dev))
    dest = route_destination(keys, W)
    perm, counts, bcounts, poff, pval = _pack(offsets, values, dest, W)
    dev = keys.device
    meta_dev = dev if (dist.get_backend(group) == "nccl") else torch.device("cpu")
    # [rows_d, bytes_d] for each peer d; received as [rows_q, bytes_q] from each peer q
    cnt = torch.tensor([v for d in range(W) for v in (counts[d], bcounts[d])], dtype=torch.int64, device=meta_dev)
    rcnt = torch.empty(2 * W, dtype=torch.int64, device=meta_dev)
    _a2a(rcnt, cnt, None, None, group)
    r = rcnt.view(W, 2).cpu()
    rrows, rbytes = r[:, 0].tolist(), r[:, 1].tolist()
    # lengths, keys, source rows in perm order
    plens = (poff[1:] - poff[:-1])
    out_lens = torch.empty(sum(rrows), dtype=torch.int64, device=dev)
    _a2a(out_lens, plens.contiguous(), rrows, counts, group)
    out_keys = torch.empty(sum(rrows), dtype=keys.dtype, device=dev)
    _a2a(out_keys, keys[perm].contiguous(), rrows, counts, group)
    out_src = torch.empty(sum(rrows), dtype=torch.int64, device=dev)
    _a2a(out_src, perm.contiguous(), rrows, counts, group)
    out_vals = torch.empty(max(sum(rbytes), 1), dtype=torch.uint8, device=dev)
    _a2a(out_vals[:sum(rbytes)], pval.contiguous(), rbytes, bcounts, group)
    out_off = torch.zeros(sum(rrows) + 1, dtype=torch.int64, device=dev)
    out_off[1:] = torch.cumsum(out_lens, 0)
    src_rank = torch.repeat_interleave(torch.arange(W, dtype=torch.int32, device=dev),
                                       torch.tensor(rrows, dtype=torch.int64, device=dev))
    return out_off, out_vals[:sum(rbytes)], out_keys, src_rank, out_src


# ---------------------------------------------------------------------------------------
# Sharded H3 for any UMI length (1..32): clusters of rows spread over ranks, merged with
# all-to-alls (SURVEY.md §8e variant for long UMIs; the north_star's "RCCL all-to-all
# merge"). The device steps are the C-ABI entry points of rogtk_amd/csrc/dist_cluster.hip;
# this function is the exchange plan between them:
#   codes/kind (rows)  -> local distinct codes
#   -> all-to-all by owner = code range -> owned distinct codes -> all-gather: G (sorted)
#   -> masked-key records of the owned codes -> all-to-all by hash(masked key, position)
#   -> clique edges (indices into G) -> all-gather -> connected components on every rank
#   -> rows: cluster id = label of the code's index in G
#   irregular rows: all-gather their strings; exact bytes, or (max_distance 1) Hamming-1
#   edges to each other and to G's codes, merged with the regular clusters.
# Every rank computes the same G, edges and labels, so ids equal the single-GPU ids.
# ---------------------------------------------------------------------------------------

class _HipOps:
    """Device steps through librogtk_hip (the product path; no fallback)."""

    def __init__(self, device):
        self.device = torch.device(device)

    def _stream(self):
        import ctypes
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @staticmethod
    def _p(t):
        import ctypes
        return ctypes.c_void_p(t.data_ptr() if t is not None and t.numel() else 0)

    def long_codes(self, offsets, values, validity, voff, n, L):
        from . import _lib
        codes = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        kind = torch.empty(max(n, 1), dtype=torch.uint8, device=self.device)
        _lib.call("rogtk_long_codes", self._p(offsets), offsets.element_size(), self._p(values),
                  self._p(validity), int(voff), int(n), int(L), self._p(codes), self._p(kind), self._stream())
        return codes[:n], kind[:n]

    def unique(self, codes, kind, L):
        import ctypes
        from . import _lib
        n = codes.numel()
        out = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        m = ctypes.c_int64(0)
        _lib.call("rogtk_unique_codes", self._p(codes), self._p(kind), int(n), int(L), self._p(out),
                  ctypes.byref(m), self._stream())
        return out[:m.value]

    def owner_counts(self, sorted_codes, L, W):
        import ctypes
        from . import _lib
        c = (ctypes.c_int64 * W)()
        _lib.call("rogtk_owner_counts", self._p(sorted_codes), int(sorted_codes.numel()), int(L), int(W), c,
                  self._stream())
        return list(c)

    def masked_records(self, D, L, W):
        import ctypes
        from . import _lib
        total = D.numel() * L
        mk = torch.empty(max(total, 1), dtype=torch.int64, device=self.device)
        pos = torch.empty(max(total, 1), dtype=torch.int32, device=self.device)
        code = torch.empty(max(total, 1), dtype=torch.int64, device=self.device)
        c = (ctypes.c_int64 * W)()
        _lib.call("rogtk_masked_records", self._p(D), int(D.numel()), int(L), int(W), self._p(mk), self._p(pos),
                  self._p(code), c, self._stream())
        return mk[:total], pos[:total], code[:total], list(c)

    def clique_edges(self, mk, pos, code, L, G):
        import ctypes
        from . import _lib
        n = mk.numel()
        E = torch.empty((max(n, 1), 2), dtype=torch.int32, device=self.device)
        m = ctypes.c_int64(0)
        _lib.call("rogtk_clique_edges", self._p(mk), self._p(pos), self._p(code), int(n), int(L), self._p(G),
                  int(G.numel()), self._p(E), ctypes.byref(m), self._stream())
        return E[:m.value]

    def cc_labels(self, nv, E):
        import ctypes
        from . import _lib
        lab = torch.empty(max(nv, 1), dtype=torch.int32, device=self.device)
        k = ctypes.c_int64(0)
        _lib.call("rogtk_cc_labels", int(nv), self._p(E), int(E.shape[0]), self._p(lab), ctypes.byref(k),
                  self._stream())
        return lab[:nv], k.value

    def assign(self, codes, kind, G, labels, cid):
        from . import _lib
        _lib.call("rogtk_assign_codes", self._p(codes), self._p(kind), int(codes.numel()), self._p(G),
                  int(G.numel()), self._p(labels), self._p(cid), self._stream())

    def irregular_merge(self, offsets, values, n, max_len, L, md, G, labels, n_reg):
        """ids of the n gathered irregular strings; labels (per G code) remapped in place."""
        import ctypes
        from . import _lib
        ids = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        k = ctypes.c_int64(0)
        _lib.call("rogtk_irregular_merge", self._p(offsets), self._p(values), int(n), int(max_len), int(L), int(md),
                  self._p(G), int(G.numel()), self._p(labels), int(n_reg), self._p(ids), ctypes.byref(k),
                  self._stream())
        return ids[:n], k.value

    def group_strings(self, offsets, values, n, max_len, base):
        import ctypes
        from . import _lib
        ids = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        g = ctypes.c_int64(0)
        _lib.call("rogtk_group_strings", self._p(offsets), self._p(values), int(n), int(max_len), int(base),
                  self._p(ids), ctypes.byref(g), self._stream())
        return ids[:n], g.value


def _exchange_device(t: torch.Tensor, group) -> torch.device:
    """Where collective buffers live: the tensor's device with nccl (RCCL), the host with gloo."""
    return t.device if dist.get_backend(group) == "nccl" else torch.device("cpu")


def _a2a_var(t: torch.Tensor, send_counts, group=None):
    """Variable all-to-all of the rows of t (grouped by destination rank, send_counts[r]
    rows for rank r); returns the received rows, grouped by source rank."""
    W = world(group)
    if not collective(group):
        return t, [int(send_counts[0])]
    xd = _exchange_device(t, group)
    sc = torch.tensor([int(c) for c in send_counts], dtype=torch.int64, device=xd)
    rc = torch.empty(W, dtype=torch.int64, device=xd)
    dist.all_to_all_single(rc, sc, group=group)
    recv = [int(v) for v in rc.cpu().tolist()]
    out = torch.empty((sum(recv),) + tuple(t.shape[1:]), dtype=t.dtype, device=xd)
    inp = t.to(xd) if t.device != xd else t
    dist.all_to_all_single(out, inp.contiguous(), recv, [int(c) for c in send_counts], group=group)
    return out.to(t.device), recv


def _allgather_var(t: torch.Tensor, group=None):
    """All-gather of variable-length row blocks: the concatenation in rank order, and each
    rank's row count."""
    W = world(group)
    if not collective(group):
        return t, [t.shape[0]]
    xd = _exchange_device(t, group)
    nccl = dist.get_backend(group) == "nccl"

    def gather(out, inp):
        if nccl:
            dist.all_gather_into_tensor(out, inp, group=group)
        else:
            dist.all_gather(list(out.chunk(W)), inp, group=group)

    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=xd)
    ns = torch.empty(W, dtype=torch.int64, device=xd)
    gather(ns, n)
    sizes = [int(v) for v in ns.cpu().tolist()]
    mx = max(max(sizes), 1)
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=xd)
    pad[: t.shape[0]] = t.to(xd)
    full = torch.empty((W * mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=xd)
    gather(full, pad)
    parts = [full[r * mx: r * mx + sizes[r]] for r in range(W)]
    return torch.cat(parts).to(t.device), sizes


def _irregular_strings(offsets: torch.Tensor, values: torch.Tensor, rows: torch.Tensor):
    """(int64 offsets from 0, bytes) of the listed rows (plumbing: gathers bytes)."""
    off = offsets.to(torch.int64)
    starts, lens = off[rows], off[rows + 1] - off[rows]
    poff = torch.zeros(rows.numel() + 1, dtype=torch.int64, device=offsets.device)
    if rows.numel():
        poff[1:] = torch.cumsum(lens, 0)
    total = int(poff[-1].item()) if rows.numel() else 0
    if total == 0:
        return poff, values[:0]
    idx = torch.repeat_interleave(starts - poff[:-1], lens) + torch.arange(total, dtype=torch.int64,
                                                                          device=offsets.device)
    return poff, values[idx]


def umi_cluster_sharded(offsets: torch.Tensor, values: torch.Tensor, n: int, umi_len: int, max_distance: int = 1,
                        validity: torch.Tensor = None, validity_offset: int = 0, group=None, ops=None):
    """H3 cluster ids of this rank's rows of a UMI column sharded over the ranks of
    `group` (int32/int64 Arrow offsets, uint8 values, optional validity bitmap; device
    tensors). Returns (cluster_id int32 [n] (0xFFFFFFFF = null), n_clusters). Spec and
    ids as the single-GPU umi_cluster, for any umi_len 1..32, through
    all-to-alls instead of the 4^L bitmap."""
    if not 1 <= umi_len <= 32:
        raise ValueError("umi_len must be 1..32")
    if max_distance not in (0, 1):
        raise ValueError("max_distance must be 0 or 1")
    ops = ops if ops is not None else _HipOps(offsets.device)
    W = world(group)
    rank = dist.get_rank(group) if W > 1 else 0
    L = umi_len
    codes, kind = ops.long_codes(offsets, values, validity, validity_offset, n, L)
    D = ops.unique(codes, kind, L)
    # owners: contiguous code ranges, so the received runs and G stay sorted by rank
    recv, _ = _a2a_var(D, ops.owner_counts(D, L, W), group)
    O = ops.unique(recv, None, L) if W > 1 else D
    G, _ = _allgather_var(O, group)
    if max_distance == 1 and G.numel() > 1:
        mk, pos, code, cnt = ops.masked_records(O, L, W)
        rmk, _ = _a2a_var(mk, cnt, group)
        rpos, _ = _a2a_var(pos, cnt, group)
        rcode, _ = _a2a_var(code, cnt, group)
        E_local = ops.clique_edges(rmk, rpos, rcode, L, G)
        E, _ = _allgather_var(E_local, group)
        labels, n_reg = ops.cc_labels(G.numel(), E)
    else:
        labels = torch.arange(G.numel(), dtype=torch.int32, device=G.device)
        n_reg = G.numel()
    # irregular rows (N, lowercase, other lengths): their strings are all-gathered; exact
    # bytes (max_distance 0) or Hamming-1 edges to each other and to G's codes, merged with
    # the regular clusters (max_distance 1; labels remapped in place when clusters merge)
    irr = torch.nonzero(kind == 2).flatten()
    poff, pval = _irregular_strings(offsets, values, irr)
    lens = poff[1:] - poff[:-1]
    all_lens, counts = _allgather_var(lens, group)
    all_vals, _ = _allgather_var(pval, group)
    n_total = n_reg
    ids = None
    if all_lens.numel():
        aoff = torch.zeros(all_lens.numel() + 1, dtype=torch.int64, device=all_lens.device)
        aoff[1:] = torch.cumsum(all_lens, 0)
        labels = labels.contiguous()
        ids, n_total = ops.irregular_merge(aoff, all_vals, all_lens.numel(), int(all_lens.max().item()), L,
                                           max_distance, G, labels, n_reg)
    cid = torch.full((max(n, 1),), -1, dtype=torch.int32, device=offsets.device)[:n]
    ops.assign(codes, kind, G, labels, cid)
    if ids is not None and irr.numel():
        start = sum(counts[:rank])
        cid[irr] = ids[start: start + irr.numel()].to(cid.device)
    return cid, int(n_total)
