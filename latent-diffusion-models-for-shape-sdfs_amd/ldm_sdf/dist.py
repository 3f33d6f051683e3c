"""Multi-GPU layer: one process per GPU, ``torch.distributed``
(backend ``nccl`` = RCCL on ROCm, over xGMI).

* Decode shards the grid by z-slab: rank r computes ``k in [r*S, min((r+1)*S, N))`` with
  ``S = ceil(N/W)`` for every shape into a local ``[B, S, N, N]`` buffer; per shape, one
  ``all_gather_into_tensor(out[b], local[b])`` writes the volume in place (z-slowest, so the
  W slabs in rank order ARE the volume); a group's gathers go out as ONE coalesced collective,
  asynchronously, so they overlap the next group's compute.
* Sampling and training shard the batch (data parallel); training all-reduces gradients.

The compute of a slab is injected (``compute_slab``) so the partition / reassembly logic is
exercised by CPU ``gloo`` tests with the oracle as the slab function.
"""
from __future__ import annotations

import math
import os
import warnings
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist


def init_process_group(backend: str = "nccl", **kw) -> None:
    """``torch.distributed.init_process_group`` with RCCL set to fail fast: an RCCL error or
    timeout on one rank aborts the communicator (``TORCH_NCCL_ASYNC_ERROR_HANDLING=1``, SURVEY
    §5 "Fault/elastic") instead of leaving the other ranks blocked in a collective.  A value the
    caller already exported is kept."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    dist.init_process_group(backend, **kw)


class _Local:
    """``group=LOCAL``: this rank alone, even inside an initialised process group (a rank
    that runs a single-GPU workload while the others wait -- bench.py's rank-0 legs).  Every
    collective of this module is then a no-op, as at world size 1."""

    def __repr__(self) -> str:
        return "ldm_sdf.dist.LOCAL"


LOCAL = _Local()


def world_and_rank(group=None) -> Tuple[int, int]:
    """(world size, rank) of ``group`` (None: the default group once initialised; LOCAL or
    no process group: (1, 0))."""
    if group is LOCAL or not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def slab_bounds(rank: int, world: int, N: int) -> Tuple[int, int, int]:
    """(k0, k1, S): this rank's z-slab [k0, k1) and the padded slab depth S = ceil(N/W)."""
    S = math.ceil(N / world)
    k0 = min(rank * S, N)
    k1 = min(k0 + S, N)
    return k0, k1, S


def shape_groups(B: int, per_group: Optional[int] = None):
    """Consecutive shape ranges ``[(b0, b1), ...]`` the sharded decode computes and gathers
    one after another.  Default: ceil(B/8) shapes per group, so up to 8 groups whose gathers
    overlap the next group's compute."""
    g = max(1, per_group if per_group else -(-B // 8))
    return [(b, min(B, b + g)) for b in range(0, B, g)]


def decode_sharded(compute_slab: Callable[..., None], B: int, N: int,
                   device: torch.device, group=None,
                   out: Optional[torch.Tensor] = None,
                   shapes_per_group: Optional[int] = None) -> torch.Tensor:
    """Z-slab sharded decode + all-gather of the full volume ``[B, N, N, N]`` on every rank.

    ``compute_slab(k0, k1, dst, b0, b1)`` fills the contiguous ``dst [b1-b0, k1-k0, N, N]``
    with shapes ``[b0, b1)``.  Per shape ``b`` the volume ``out[b]`` (z slowest) is exactly the
    W slabs in rank order, so ONE ``all_gather_into_tensor(out[b], local[b])`` assembles it in
    place: no transpose and no second copy.  Shapes go in groups
    (``shape_groups``); each group's gathers are issued as one coalesced asynchronous
    collective (``_gather_group``; RCCL runs it on its own stream) before the next group's
    slabs are computed, so communication overlaps compute.
    When W does not divide N the last slab is zero-padded to S = ceil(N/W) rows and the
    gathered ``[W*S, N, N]`` is trimmed into ``out[b]``.
    """
    world, rank = world_and_rank(group)
    k0, k1, S = slab_bounds(rank, world, N)
    vol = out if out is not None else torch.empty(B, N, N, N, device=device,
                                                  dtype=torch.float32)
    if tuple(vol.shape) != (B, N, N, N) or not vol.is_contiguous():
        raise ValueError("decode_sharded: out must be a contiguous [B, N, N, N] tensor")
    if world == 1:
        for b0, b1 in shape_groups(B, shapes_per_group):
            compute_slab(0, N, vol[b0:b1], b0, b1)
        return vol
    even = S * world == N
    local = torch.empty(B, S, N, N, device=device, dtype=torch.float32)
    pending, staged = [], []
    for b0, b1 in shape_groups(B, shapes_per_group):
        if k1 - k0 == S:
            compute_slab(k0, k1, local[b0:b1], b0, b1)
        else:
            local[b0:b1].zero_()
            if k1 > k0:
                part = torch.empty(b1 - b0, k1 - k0, N, N, device=device, dtype=torch.float32)
                compute_slab(k0, k1, part, b0, b1)
                local[b0:b1, :k1 - k0].copy_(part)
        dsts = []
        for b in range(b0, b1):
            dst = vol[b] if even else torch.empty(world * S, N, N, device=device,
                                                  dtype=torch.float32)
            dsts.append((b, dst))
            if not even:
                staged.append((b, dst))
        pending.append(_gather_group(dsts, local, group))
    for w in pending:
        w.wait()
    for b, dst in staged:
        vol[b].copy_(dst[:N])
    return vol


# How a group's per-shape gathers go out: "coalesced" (one grouped collective through torch's
# coalescing manager, the default) or "per_shape" (one async all_gather_into_tensor per shape).
# The coalescing manager is a private torch API: if entering it raises on this backend, the
# mode falls back to "per_shape" for the rest of the process (same bytes, more launches).
_GATHER_MODE = {"mode": "coalesced"}


def set_gather_mode(mode: str) -> None:
    """Select ``_gather_group``'s form ("coalesced" or "per_shape"); both assemble the same
    volume bit for bit (tests/test_dist_gloo.py)."""
    if mode not in ("coalesced", "per_shape"):
        raise ValueError("gather mode must be 'coalesced' or 'per_shape'")
    _GATHER_MODE["mode"] = mode


def gather_mode() -> str:
    return _GATHER_MODE["mode"]


class _Works:
    """Handles of per-shape async collectives, waited on together."""

    def __init__(self, works):
        self.works = works

    def wait(self) -> None:
        for w in self.works:
            w.wait()


def _gather_group(dsts, local: torch.Tensor, group):
    """One coalesced collective for a group's per-shape gathers: the group's
    ``all_gather_into_tensor(dst_b, local[b])`` calls are issued inside torch's coalescing
    manager, which hands them to the backend as ONE grouped operation (RCCL: one
    ``ncclGroupStart/End`` launch instead of one launch per shape), asynchronously.  If the
    manager cannot be entered (a private API: absent or refused by the backend), the same
    gathers go out as per-shape async collectives (``set_gather_mode``).  Returns the handle
    to wait on."""
    if _GATHER_MODE["mode"] == "coalesced":
        try:
            cm = dist._coalescing_manager(group=group, async_ops=True)
            ctx = cm.__enter__()
        except (AttributeError, NotImplementedError, RuntimeError, TypeError) as e:
            warnings.warn(f"dist: coalesced all-gather unavailable ({e!r}); per-shape gathers "
                          "from now on", RuntimeWarning)
            _GATHER_MODE["mode"] = "per_shape"
        else:
            try:
                for b, dst in dsts:
                    dist.all_gather_into_tensor(dst, local[b], group=group)
            except BaseException:
                cm.__exit__(*__import__("sys").exc_info())
                raise
            cm.__exit__(None, None, None)
            return ctx
    return _Works([dist.all_gather_into_tensor(dst, local[b], group=group, async_op=True)
                   for b, dst in dsts])


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


def allreduce_weighted_(tensors, weight: float, group=None) -> None:
    """``sum_r weight_r * t_r`` in place on every rank (one bucket, one all-reduce): the
    data-parallel gradient of a loss that is a mean over a global batch sharded unevenly --
    rank r passes ``weight = B_r / B`` for gradients of its local mean (train())."""
    _allreduce_(tensors, group, mean=False, pre_scale=weight)


def flat_buffers(shapes: Dict[str, Tuple[int, ...]], device, dtype=torch.float32
                 ) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """One flat buffer and a view of it per named shape, in order, each view starting at a
    16-byte multiple (so the views stay valid operands of the aligned C ABI).  Gradients kept
    in such views are all-reduced as the flat buffer itself: no per-step ``torch.cat`` of 40 MB
    and no copy back (``_allreduce_``)."""
    per = 16 // torch.empty((), dtype=dtype).element_size()
    offs, n = [], 0
    for shp in shapes.values():
        offs.append(n)
        n += -(-math.prod(shp) // per) * per
    flat = torch.zeros(n, device=device, dtype=dtype)
    views = {k: flat[o:o + math.prod(shp)].view(shp)
             for (k, shp), o in zip(shapes.items(), offs)}
    return flat, views


def _flat_base(tensors: List[torch.Tensor]) -> Optional[torch.Tensor]:
    """The 1-D buffer the tensors are consecutive views of (``flat_buffers`` layout, gaps of
    padding allowed), or None."""
    if not tensors:
        return None
    base = tensors[0]._base
    if base is None or base.dim() != 1 or not base.is_contiguous():
        return None
    es = base.element_size()
    start = base.data_ptr()
    pos = 0
    for t in tensors:
        if t._base is not base or not t.is_contiguous():
            return None
        o = (t.data_ptr() - start) // es
        if o < pos or (o - pos) * es >= 16:    # only alignment padding may lie between views
            return None
        pos = o + t.numel()
    return base[:pos]


def _allreduce_(tensors, group, mean: bool, pre_scale: Optional[float] = None) -> None:
    world, _ = world_and_rank(group)
    if world == 1:
        return
    tensors = list(tensors)
    flat = _flat_base(tensors)
    if flat is not None:
        # views of one persistent buffer: reduce it in place (padding between views is zero on
        # every rank and stays zero)
        if pre_scale is not None:
            flat.mul_(pre_scale)
        dist.all_reduce(flat, group=group)
        if mean:
            flat.div_(world)
        return
    flat = torch.cat([t.reshape(-1) for t in tensors])
    if pre_scale is not None:
        flat.mul_(pre_scale)
    dist.all_reduce(flat, group=group)
    if mean:
        flat.div_(world)
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n
