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


def world(group=None) -> int:
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def gather_bitmaps(local: torch.Tensor, group=None):
    """All-gather one bitmap per rank into a [world * words] tensor (rank-major)."""
    n = world(group)
    if n == 1:
        return local, 1
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
    if W == 1:
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
