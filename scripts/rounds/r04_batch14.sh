#!/bin/bash
# Round-4 GPU batch 14: the launch kernel's contraction geometry preloaded (FastGeo) -- UNet GPU
# tests, step rate at B = 1 / 8, conv stamps.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04p
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread > $O/test_unet.log 2>&1
for i in 1 2; do
  UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py >> $O/unet_once_b1.log 2>&1
  UNET_B=8 UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py >> $O/unet_once_b8.log 2>&1
done
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_stamp.so
LDM_SDF_LIB=$LIB timeout -k 10 120 python -u scripts/stamp_conv.py 1 > $O/stamp_conv_b1.log 2>&1
echo batch14 done
