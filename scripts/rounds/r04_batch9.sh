#!/bin/bash
# Round-4 GPU batch 9: register-held conv stamps, direct vs generic staging.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04k
mkdir -p $O
cd $GRAFT_REPO_ROOT
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_stamp.so
LDM_SDF_LIB=$LIB LDM_CONV_FAST=1 timeout -k 10 120 python -u scripts/stamp_conv.py 1 > $O/stamp_conv_b1_direct.log 2>&1
LDM_SDF_LIB=$LIB LDM_CONV_FAST=0 timeout -k 10 120 python -u scripts/stamp_conv.py 1 > $O/stamp_conv_b1_generic.log 2>&1
echo batch9 done
