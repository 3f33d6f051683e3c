#!/bin/bash
# Round 5: first run of the one-launch training step -> profiles/r05b/: its GPU tests (bitwise
# vs the launch path), the training / GEMM tests after the gemm_tile.h refactor, the A/B of
# both forms at config 2, and a kernel trace of a few DAG steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_dag.py -x -v --timeout 120 \
    --timeout-method thread > $O/pytest_dag.log 2>&1
rc=$?
tail -25 $O/pytest_dag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_capi.py tests/test_gpu_gemm.py \
    tests/test_gpu_configs.py tests/test_gpu_ddpm.py -x -q --timeout 120 --timeout-method thread \
    > $O/pytest_train.log 2>&1 || { tail -30 $O/pytest_train.log; exit 1; }
tail -3 $O/pytest_train.log
timeout -k 10 300 python -u scripts/train_form_ab.py 4 128 > $O/train_ab.log 2>&1 \
    || { tail -20 $O/train_ab.log; exit 1; }
cat $O/train_ab.log
TRAIN_STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o train \
    --output-format csv -- python3 scripts/train_once.py > $O/prof.log 2>&1 \
    || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/train_kernel_stats.csv
head -8 $O/train_kernel_stats.csv
