#!/bin/bash
# Round-4 GPU batch 20: direct-staging split stamps (entry, loads issued, data landed, stores).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04v
mkdir -p $O
cd $GRAFT_REPO_ROOT
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_stamp.so
LDM_SDF_LIB=$LIB timeout -k 10 120 python -u scripts/stamp_conv.py 1 > $O/stamp_conv_b1.log 2>&1
echo batch20 done
