#!/bin/bash
# Round-4 GPU batch 8: direct conv staging -- UNet GPU tests, step rate (B = 1, 8), A/B against
# the generic staging (dev build, LDM_CONV_FAST), per-launch stamps.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04j
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread > $O/test_unet.log 2>&1
UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py > $O/unet_once_b1.log 2>&1
UNET_B=8 UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py > $O/unet_once_b8.log 2>&1
DEV=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_dev.so
for v in 0 1 0 1; do
  LDM_SDF_LIB=$DEV LDM_CONV_FAST=$v UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py >> $O/ab_fast_b1.log 2>&1
  echo "^ LDM_CONV_FAST=$v" >> $O/ab_fast_b1.log
done
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_stamp.so
LDM_SDF_LIB=$LIB timeout -k 10 120 python -u scripts/stamp_conv.py 1 > $O/stamp_conv_b1.log 2>&1
echo batch8 done
