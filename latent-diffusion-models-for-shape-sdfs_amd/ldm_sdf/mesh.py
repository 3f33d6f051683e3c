"""C18: marching cubes on decoded SDF volumes + PLY export.

``marching_cubes`` runs the HIP passes of ``csrc/mc.hip`` (``ldm_mc_count`` ->
read the two counts -> ``ldm_mc_emit``) on the volume where decode left it; conventions and
the generated case table are DESIGN.md §10.  ``write_ply`` writes the binary PLY DeepSDF's
``convert_sdf_samples_to_ply`` writes (host I/O).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _capi as capi
from . import dist as ldist
from .ops import voxel_size


def mc_table() -> Tuple[np.ndarray, np.ndarray]:
    """The library's compile-time generated case table: (tri [256, 16] int8, ntri [256] u8)."""
    tri = np.zeros((256, 16), np.int8)
    ntri = np.zeros(256, np.uint8)
    capi.check(capi.load().ldm_mc_table(tri.ctypes.data, ntri.ctypes.data), "ldm_mc_table")
    return tri, ntri


def marching_cubes(volume: torch.Tensor, level: float = 0.0, bbox=(-1.0, 1.0),
                   ws: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Iso-surface of ``volume [N, N, N]`` (z slowest, as ``decode`` returns it) at ``level``.

    Returns device tensors ``verts [V, 3]`` (x, y, z on the A1 grid over ``bbox``) and
    ``faces [F, 3]`` int32, outward (toward larger values) winding.  One host sync (the two
    counts) sits between the passes.
    """
    capi.require_device(volume)
    if volume.dim() != 3 or len(set(volume.shape)) != 1 or volume.dtype != torch.float32:
        raise capi.LdmError("marching_cubes: volume must be a float32 [N, N, N] tensor")
    volume = volume.contiguous()
    N = volume.shape[0]
    dev = volume.device
    lib = capi.load()
    need = lib.ldm_mc_workspace_bytes(N)
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, device=dev, dtype=torch.uint8)
    counts = torch.empty(2, device=dev, dtype=torch.int32)
    s = capi.stream_handle(dev)
    capi.check(lib.ldm_mc_count(volume.data_ptr(), N, float(level), ws.data_ptr(), ws.numel(),
                                counts.data_ptr(), s), "ldm_mc_count")
    nv, nf = (int(x) for x in counts.cpu())
    verts = torch.empty(max(nv, 1), 3, device=dev, dtype=torch.float32)
    faces = torch.empty(max(nf, 1), 3, device=dev, dtype=torch.int32)
    capi.check(lib.ldm_mc_emit(volume.data_ptr(), N, float(level), voxel_size(N, bbox),
                               float(bbox[0]), ws.data_ptr(), ws.numel(), verts.data_ptr(),
                               faces.data_ptr(), s), "ldm_mc_emit")
    return verts[:nv], faces[:nf]


def marching_cubes_batch(volumes: torch.Tensor, level: float = 0.0, bbox=(-1.0, 1.0),
                         group=None) -> List[Tuple[int, torch.Tensor, torch.Tensor]]:
    """Mesh a batch ``[B, N, N, N]``; with a process group each rank meshes the shapes
    ``b = rank, rank + W, ...`` of the (all-gathered) batch.  Returns (b, verts, faces)."""
    world, rank = ldist.world_and_rank(group)
    ws = torch.empty(capi.load().ldm_mc_workspace_bytes(volumes.shape[-1]),
                     device=volumes.device, dtype=torch.uint8)
    return [(b, *marching_cubes(volumes[b], level, bbox, ws=ws))
            for b in range(rank, volumes.shape[0], world)]


def write_ply(path: str, verts, faces, offset: Optional[Sequence[float]] = None,
              scale: Optional[float] = None) -> None:
    """Binary little-endian PLY (vertex float x, y, z; face ``list uchar int``), as DeepSDF's
    ``convert_sdf_samples_to_ply`` writes it; ``offset``/``scale`` undo a normalisation
    (``p / scale - offset``) when given."""
    v = verts.detach().cpu().numpy() if isinstance(verts, torch.Tensor) else np.asarray(verts)
    f = faces.detach().cpu().numpy() if isinstance(faces, torch.Tensor) else np.asarray(faces)
    v = v.astype("<f4")
    if scale is not None:
        v = v / np.float32(scale)
    if offset is not None:
        v = v - np.asarray(offset, np.float32)
    head = ("ply\nformat binary_little_endian 1.0\n"
            f"element vertex {len(v)}\nproperty float x\nproperty float y\nproperty float z\n"
            f"element face {len(f)}\nproperty list uchar int vertex_indices\nend_header\n")
    rec = np.zeros(len(f), dtype=[("n", "u1"), ("v", "<i4", (3,))])
    rec["n"] = 3
    rec["v"] = f
    with open(path, "wb") as fh:
        fh.write(head.encode("ascii"))
        fh.write(np.ascontiguousarray(v, "<f4").tobytes())
        fh.write(rec.tobytes())
