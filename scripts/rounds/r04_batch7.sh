#!/bin/bash
# Round-4 GPU batch 7: fine staging stamps of the 18 conv launches (diagnostic build).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04i
mkdir -p $O
cd $GRAFT_REPO_ROOT
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_stamp.so
LDM_SDF_LIB=$LIB timeout -k 10 120 python -u scripts/stamp_conv.py 1 > $O/stamp_conv_b1_fine.log 2>&1
echo batch7 done
