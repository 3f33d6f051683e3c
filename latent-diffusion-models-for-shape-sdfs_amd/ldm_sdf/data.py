"""C20: DeepSDF data and checkpoint formats.

Host-side I/O only (no device compute).  The formats are those of the DeepSDF code base.

* SDF samples: one ``.npz`` per shape with ``pos`` and ``neg`` arrays of ``[n, 4]`` float rows
  ``(x, y, z, sdf)``, for points outside and inside the surface. Rows whose sdf is NaN are
  dropped on load (DeepSDF ``remove_nans``). A training draw takes ``subsample / 2`` rows
  uniformly with replacement from each half, positives first (DeepSDF
  ``unpack_sdf_samples``).
* Checkpoints:
  * ``ModelParameters/<epoch>.pth``: ``{"epoch": e, "model_state_dict": {"lin{l}.weight",
    "lin{l}.bias"}}``. Weight-norm pairs ``weight_g`` / ``weight_v`` are accepted on load
    (``SDFDecoder.from_state_dict``).
  * ``LatentCodes/<epoch>.pth``: ``{"epoch": e, "latent_codes": {"weight": [n, L]}}``, the
    ``nn.Embedding`` state dict. A bare ``[n, L]`` tensor is accepted too.

Every load goes through loaders that execute nothing from the file:
``numpy.load(allow_pickle=False)`` and ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .models import SDFDecoder

__all__ = ["load_sdf_samples", "unpack_sdf_samples", "SdfSampleSet", "save_model",
           "load_model", "save_latent_codes", "load_latent_codes"]


def _remove_nans(a: np.ndarray) -> np.ndarray:
    return a[~np.isnan(a[:, 3])]


def load_sdf_samples(path: str) -> Tuple[torch.Tensor, torch.Tensor]:
    """(pos [n, 4], neg [m, 4]) float32 CPU tensors from a DeepSDF ``.npz``, NaN rows dropped."""
    with np.load(path, allow_pickle=False) as f:
        if "pos" not in f or "neg" not in f:
            raise ValueError(f"{path}: expected arrays 'pos' and 'neg', got {list(f.keys())}")
        pos, neg = f["pos"], f["neg"]
    for name, a in (("pos", pos), ("neg", neg)):
        if a.ndim != 2 or a.shape[1] != 4:
            raise ValueError(f"{path}: '{name}' must be [n, 4] (x, y, z, sdf), got {a.shape}")
    return (torch.from_numpy(_remove_nans(pos).astype(np.float32)),
            torch.from_numpy(_remove_nans(neg).astype(np.float32)))


def unpack_sdf_samples(pos: torch.Tensor, neg: torch.Tensor, subsample: int,
                       generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """``[subsample, 4]``: ``subsample // 2`` uniform draws with replacement from ``pos`` then
    the same from ``neg`` (an odd ``subsample`` gives the extra row to ``neg``)."""
    if pos.shape[0] == 0 or neg.shape[0] == 0:
        raise ValueError("both sample halves must be non-empty after NaN removal")
    half = subsample // 2
    ip = torch.randint(0, pos.shape[0], (half,), generator=generator, device=pos.device)
    ineg = torch.randint(0, neg.shape[0], (subsample - half,), generator=generator,
                         device=neg.device)
    return torch.cat([pos[ip], neg[ineg]], dim=0)


class SdfSampleSet:
    """All shapes' sample pools in memory, in file order (the latent index = the position)."""

    def __init__(self, paths: Sequence[str]):
        self.paths = list(paths)
        self.pools: List[Tuple[torch.Tensor, torch.Tensor]] = [load_sdf_samples(p)
                                                               for p in self.paths]

    @classmethod
    def from_split(cls, data_source: str, split: Dict[str, Dict[str, List[str]]],
                   subdir: str = "SdfSamples") -> "SdfSampleSet":
        """DeepSDF split JSON layout: ``{dataset: {class: [instance, ...]}}`` under
        ``<data_source>/SdfSamples/<dataset>/<class>/<instance>.npz``."""
        paths = [os.path.join(data_source, subdir, ds, cls_, inst + ".npz")
                 for ds, classes in split.items() for cls_, insts in classes.items()
                 for inst in insts]
        return cls(paths)

    def __len__(self) -> int:
        return len(self.pools)

    def draw(self, samples_per_shape: int, device=None,
             generator: Optional[torch.Generator] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """One DeepSDF draw for every shape: ``xyz [n, P, 3]``, ``sdf [n, P]`` on ``device``.
        This is the input ``train_autodecoder`` subsamples per step."""
        rows = torch.stack([unpack_sdf_samples(p, n, samples_per_shape, generator)
                            for p, n in self.pools])
        rows = rows.to(device) if device is not None else rows
        return rows[..., :3].contiguous(), rows[..., 3].contiguous()


def _ckpt(path: str) -> Dict:
    return torch.load(path, map_location="cpu", weights_only=True)


def save_model(path: str, decoder: SDFDecoder, epoch: int) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save({"epoch": int(epoch), "model_state_dict": decoder.state_dict()}, path)


def load_model(path: str, latent_dim: int, **kw) -> Tuple[SDFDecoder, int]:
    """(decoder, epoch) from a DeepSDF ``ModelParameters`` checkpoint (``module.`` prefixes of
    DataParallel saves are stripped)."""
    ck = _ckpt(path)
    sd = ck["model_state_dict"] if "model_state_dict" in ck else ck
    sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
    return SDFDecoder.from_state_dict(sd, latent_dim, **kw), int(ck.get("epoch", 0))


def save_latent_codes(path: str, latents: torch.Tensor, epoch: int) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save({"epoch": int(epoch),
                "latent_codes": {"weight": latents.detach().to("cpu", torch.float32)}}, path)


def load_latent_codes(path: str) -> Tuple[torch.Tensor, int]:
    """(latents [n, L] fp32 CPU, epoch) from a DeepSDF ``LatentCodes`` checkpoint."""
    ck = _ckpt(path)
    if isinstance(ck, torch.Tensor):
        return ck.float(), 0
    lc = ck["latent_codes"]
    w = lc["weight"] if isinstance(lc, dict) else lc
    if w.dim() == 3:                  # old DeepSDF saves: [n, 1, L]
        w = w.squeeze(1)
    return w.float(), int(ck.get("epoch", 0))
