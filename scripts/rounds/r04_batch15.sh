#!/bin/bash
# Round-4 GPU batch 15: where a training-step GEMM launch's time goes (GEMM stamps).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04q
mkdir -p $O
cd $GRAFT_REPO_ROOT
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_stamp.so
LDM_SDF_LIB=$LIB timeout -k 10 200 python -u scripts/stamp_gemm.py > $O/stamp_gemm.log 2>&1
echo batch15 done
