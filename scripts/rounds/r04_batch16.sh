#!/bin/bash
# Round-4 GPU batch 16: GEMM epilogue operands loaded before the k-loop (EpiPre) -- GEMM /
# training / auto-decoder GPU tests, A/B of the training step against the build without it,
# GEMM stamps.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04r
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_train_capi.py tests/test_gpu_configs.py tests/test_gpu_autodecoder.py -x -q --timeout 120 --timeout-method thread > $O/test_gemm_train.log 2>&1
NOE=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_noepi.so
for i in 1 2; do
  LDM_SDF_LIB=$NOE TRAIN_STEPS=200 timeout -k 10 120 python -u scripts/train_once.py >> $O/ab_train.log 2>&1
  echo "^ without EpiPre" >> $O/ab_train.log
  TRAIN_STEPS=200 timeout -k 10 120 python -u scripts/train_once.py >> $O/ab_train.log 2>&1
  echo "^ with EpiPre" >> $O/ab_train.log
done
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_stamp.so
LDM_SDF_LIB=$LIB timeout -k 10 200 python -u scripts/stamp_gemm.py > $O/stamp_gemm.log 2>&1
echo batch16 done
