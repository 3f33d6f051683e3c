#!/bin/bash
# round 3: split-K bound estimate for config 2's GEMM shapes (1024-row padded batch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r03d
o=gpurun_out/r03d/gemm_splitk.log; : > $o
for sh in 1024,1024,2048 1024,1024,1024 1024,1024,4096; do
  for sk in 1 2 4; do
    SHAPE=$sh SPLITK=$sk NO_REF=1 OUT=c TILES=${TILES:-4,24,3,6,14,16,23,26} timeout -k 10 120 python3 scripts/gemm_bench.py >> $o 2>&1 || exit $?
  done
done
SHAPE=1024,1024,2048 SPLITK=1 NO_REF=1 OUT=all TILES=4,24,3,6 timeout -k 10 120 python3 scripts/gemm_bench.py >> $o 2>&1
