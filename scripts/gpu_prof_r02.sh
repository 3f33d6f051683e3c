#!/bin/bash
# Round-2 evidence: rocprof kernel trace of the DEFAULT bench command (the headline line), then
# PMC passes over the config-2 training step and the auto-decoder step (linear_mfma GEMMs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGES="${STAGES:-prof pmc_train pmc_ad}"
for s in $STAGES; do
  case $s in
    prof)
      echo "== rocprof bench (default command)"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run \
          --output-format csv -- python3 bench.py > gpurun_out/prof_bench.log 2>&1 || exit $?
      tail -c 600 gpurun_out/prof_bench.log ;;
    pmc_train)
      echo "== pmc train"
      TRAIN_STEPS=3 WORKLOAD=scripts/train_once.py PMC_OUT=gpurun_out/pmc_train \
        PASSES="cycles insts lds fetch write" bash scripts/pmc.sh || exit $? ;;
    pmc_ad)
      echo "== pmc autodecoder"
      AD_STEPS=1 WORKLOAD=scripts/ad_once.py PMC_OUT=gpurun_out/pmc_ad \
        PASSES="cycles insts fetch write" bash scripts/pmc.sh || exit $? ;;
  esac
done
