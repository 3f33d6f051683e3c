#!/bin/bash
# Round-4 GPU batch 10: direct conv staging v2 (one round trip, deferred epilogue operands);
# marching cubes with the block sums folded into classify.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04l
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread > $O/test_unet.log 2>&1
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_stamp.so
LDM_SDF_LIB=$LIB LDM_CONV_FAST=1 timeout -k 10 120 python -u scripts/stamp_conv.py 1 > $O/stamp_conv_b1_direct.log 2>&1
LDM_SDF_LIB=$LIB LDM_CONV_FAST=0 timeout -k 10 120 python -u scripts/stamp_conv.py 1 > $O/stamp_conv_b1_generic.log 2>&1
DEV=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_dev.so
for v in 0 1 0 1; do
  LDM_SDF_LIB=$DEV LDM_CONV_FAST=$v UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py >> $O/ab_fast_b1.log 2>&1
  echo "^ LDM_CONV_FAST=$v" >> $O/ab_fast_b1.log
  LDM_SDF_LIB=$DEV LDM_CONV_FAST=$v UNET_B=8 UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py >> $O/ab_fast_b8.log 2>&1
  echo "^ LDM_CONV_FAST=$v" >> $O/ab_fast_b8.log
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_mc.py -x -q --timeout 120 --timeout-method thread > $O/test_mc.log 2>&1
timeout -k 10 120 python -u scripts/mc_once.py 20 > $O/mc_once.log 2>&1
echo batch10 done
