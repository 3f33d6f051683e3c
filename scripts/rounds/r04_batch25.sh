#!/bin/bash
# Round-4 GPU batch 25: PMC passes (cycles, instruction mix, LDS) over 100 UNet steps at B = 1
# (scripts/unet_once.py), per-kernel summary (profiles/r04p).
set -e
cd $GRAFT_REPO_ROOT
export UNET_STEPS=100 WORKLOAD=scripts/unet_once.py PMC_OUT=$GRAFT_REPO_ROOT/gpurun_out/r04p PASSES="cycles insts lds"
bash scripts/rounds/pmc.sh > gpurun_out/r04p_passes.log 2>&1
python scripts/pmc_by_kernel.py gpurun_out/r04p conv1d > gpurun_out/r04p/summary.txt 2>&1
echo batch25 done
