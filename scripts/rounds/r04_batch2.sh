#!/bin/bash
# Round-4 GPU batch 2: decoder variants A/B (split kernel: group base, one-copy layer loop).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04b
mkdir -p $O
cd $GRAFT_REPO_ROOT
LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_dev.so
LDM_SDF_LIB=$LIB AB_VARIANTS=s,s2,s4,s6 timeout -k 10 300 python -u scripts/ab_decoder.py 8 256 5 > $O/ab_decoder_v.log 2>&1
LDM_SDF_LIB=$LIB AB_VARIANTS=s,s4,s6 AB_DTYPES=fp16 timeout -k 10 300 python -u scripts/ab_decoder.py 8 256 3 > $O/ab_decoder_v_fp16.log 2>&1
echo batch2 done
