"""ldm_sdf -- MI355X-native hot path of latent diffusion over DeepSDF shape codes.

Layers: ``api`` (train/sample/decode) -> ``models`` (parameter containers,
packing) -> ``ops`` (one wrapper per C-ABI call) -> ``_capi`` (ctypes) -> ``libldm_sdf.so``
(HIP kernels for gfx950, sources in ``../csrc``).  ``dist`` adds z-slab / batch sharding
over ``torch.distributed`` (RCCL).
"""
from .models import DDPMSchedule, MLPDenoiser, SDFDecoder, decoder_layer_dims  # noqa: F401
from .unet import UNet1DDenoiser  # noqa: F401
from .mesh import marching_cubes, marching_cubes_batch, mc_table, write_ply  # noqa: F401
from .api import (Sampler, TrainState, decode, decode_points, resolve_decode_dtype,  # noqa: F401
                  sample, train, train_step)
from .autodecoder import (AutoDecoderState, autodecoder_train_step,  # noqa: F401
                          train_autodecoder)
from . import ops, dist, pack, data  # noqa: F401
from ._capi import LdmError, load as load_library  # noqa: F401

__version__ = "0.1.0"
