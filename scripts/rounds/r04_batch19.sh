#!/bin/bash
# Round-4 GPU batch 19: conv stamps of the final UNet build (B = 1, skip concats as one buffer).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04u
mkdir -p $O
cd $GRAFT_REPO_ROOT
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_stamp.so
LDM_SDF_LIB=$LIB timeout -k 10 120 python -u scripts/stamp_conv.py 1 > $O/stamp_conv_b1.log 2>&1
for i in 1 2; do
  UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py >> $O/unet_once_b1.log 2>&1
done
echo batch19 done
