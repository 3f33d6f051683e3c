"""Multi-GPU layer: one process per GPU, ``torch.distributed``
(backend ``nccl`` = RCCL on ROCm, over xGMI).

* Decode shards the grid by z-slab: rank r computes ``k in [r*S, min((r+1)*S, N))`` with
  ``S = ceil(N/W)`` for every shape into a local ``[B, S, N, N]`` buffer; ONE
  ``all_gather_into_tensor`` collects ``[W, B, S, N, N]``; because the volume is z-slowest,
  the gathered slabs are already the volume for B == 1 and need one permute for B > 1.
* Sampling and training shard the batch (data parallel); training all-reduces gradients.

The compute of a slab is injected (``compute_slab``) so the partition / reassembly logic is
exercised by CPU ``gloo`` tests with the oracle as the slab function.
"""
from __future__ import annotations

import math
from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def world_and_rank(group=None) -> Tuple[int, int]:
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def slab_bounds(rank: int, world: int, N: int) -> Tuple[int, int, int]:
    """(k0, k1, S): this rank's z-slab [k0, k1) and the padded slab depth S = ceil(N/W)."""
    S = math.ceil(N / world)
    k0 = min(rank * S, N)
    k1 = min(k0 + S, N)
    return k0, k1, S


def decode_sharded(compute_slab: Callable[[int, int, torch.Tensor], None], B: int, N: int,
                   device: torch.device, group=None,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Z-slab sharded decode + all-gather of the full volume ``[B, N, N, N]`` on every rank.

    ``compute_slab(k0, k1, dst)`` fills the contiguous ``dst [B, k1-k0, N, N]``.
    """
    world, rank = world_and_rank(group)
    k0, k1, S = slab_bounds(rank, world, N)
    local = torch.empty(B, S, N, N, device=device, dtype=torch.float32)
    if k1 - k0 == S:
        compute_slab(k0, k1, local)
    else:
        local.zero_()
        if k1 > k0:
            part = torch.empty(B, k1 - k0, N, N, device=device, dtype=torch.float32)
            compute_slab(k0, k1, part)
            local[:, :k1 - k0].copy_(part)
    if world == 1:
        vol = local
    else:
        # output as [W*B, S, N, N] (dim-0 concatenation: the form gloo and RCCL both take)
        gathered = torch.empty(world * B, S, N, N, device=device, dtype=torch.float32)
        dist.all_gather_into_tensor(gathered, local, group=group)
        gathered = gathered.view(world, B, S, N, N)
        if B == 1:
            vol = gathered.view(1, world * S, N, N)
        else:
            vol = gathered.permute(1, 0, 2, 3, 4).reshape(B, world * S, N, N)
    vol = vol[:, :N]
    if out is not None:
        out.copy_(vol)
        return out
    return vol if vol.is_contiguous() else vol.contiguous()


def batch_shard(n: int, rank: int, world: int) -> Tuple[int, int]:
    """[lo, hi) of a batch of n items owned by ``rank`` (contiguous, balanced)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def all_gather_rows(local: torch.Tensor, n: int, group=None) -> torch.Tensor:
    """Reassemble a batch of n rows sharded by ``batch_shard`` (uneven shards allowed):
    pad each shard to ceil(n/W) rows, one ``all_gather_into_tensor``, drop the padding."""
    world, rank = world_and_rank(group)
    if world == 1:
        return local
    per = -(-n // world)
    buf = torch.zeros((per,) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
    buf[:local.shape[0]] = local
    gathered = torch.empty((world * per,) + tuple(local.shape[1:]), device=local.device,
                           dtype=local.dtype)
    dist.all_gather_into_tensor(gathered, buf, group=group)
    rows = []
    for r in range(world):
        a, b = batch_shard(n, r, world)
        rows.append(gathered[r * per:r * per + (b - a)])
    return torch.cat(rows)


def allreduce_mean_(tensors, group=None) -> None:
    """Average gradients over ranks: flatten into one bucket, one all-reduce (RCCL)."""
    _allreduce_(tensors, group, mean=True)


def allreduce_sum_(tensors, group=None) -> None:
    """Sum over ranks in place (one bucket, one all-reduce)."""
    _allreduce_(tensors, group, mean=False)


def _allreduce_(tensors, group, mean: bool) -> None:
    world, _ = world_and_rank(group)
    if world == 1:
        return
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.all_reduce(flat, group=group)
    if mean:
        flat.div_(world)
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n
