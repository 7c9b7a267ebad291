"""Multi-GPU exchange for H3 (one process per GPU, torch.distributed).

Reads shard by record; H1/H2 need no exchange. H3 needs the global set of
distinct UMIs: every rank publishes its 4^L-bit presence bitmap (2 MiB at L=12)
with ONE all-gather (RCCL over xGMI with backend "nccl"; gloo on CPU for tests),
then every rank resolves the same global components redundantly inside
rogtk_cluster_resolve (which ORs the gathered bitmaps while it scans them), so
cluster ids are bit-identical for 1, 2, 4 or 8 GPUs with no second exchange.

An all-gather of N bitmaps moves (N-1)/N * N * 2 MiB per rank; a ring all-reduce
would need a bitwise-OR reduction RCCL does not offer, and a byte-wise MAX on a
4^L-byte table moves 8x the bytes.
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
