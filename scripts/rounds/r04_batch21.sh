#!/bin/bash
# Round-4 GPU batch 21: producer-side SiLU twins (ldm_conv1d Ys) -- UNet GPU tests, steps/s at
# B = 1 and B = 8, conv stamps at B = 1.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04w
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_unet.py > $O/test_gpu_unet.log 2>&1
for i in 1 2; do
  UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py >> $O/unet_once_b1.log 2>&1
done
UNET_B=8 UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py >> $O/unet_once_b8.log 2>&1
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_stamp.so
LDM_SDF_LIB=$LIB timeout -k 10 120 python -u scripts/stamp_conv.py 1 > $O/stamp_conv_b1.log 2>&1
echo batch21 done
