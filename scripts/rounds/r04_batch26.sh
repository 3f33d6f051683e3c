#!/bin/bash
# Round-4 GPU batch 26: 24-bit index products in the UNet conv (v_mul_u32_u24 for v_mul_lo_u32):
# UNet GPU tests, then an interleaved A/B against the previous build (libldm_prev.so) at B = 1, 8.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04q
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_unet.py tests/test_gpu_configs.py > $O/test_gpu.log 2>&1
PREV=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_prev.so
for i in 1 2 3; do
  for B in 1 8; do
    echo "mul24 B=$B" >> $O/ab_mul24.log
    UNET_B=$B UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py 2>/dev/null >> $O/ab_mul24.log
    echo "prev B=$B" >> $O/ab_mul24.log
    LDM_SDF_LIB=$PREV UNET_B=$B UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py 2>/dev/null >> $O/ab_mul24.log
  done
done
echo batch26 done
