#!/bin/bash
# Round 5 -> profiles/r05e/: the one-launch training step after the wave-uniform scheduler fix
# (diagnostic step, its GPU tests, the training / GEMM / UNet / DDPM tests, the A/B of both
# forms, a kernel trace of DAG steps), the UNet convs re-pitched for conflict-free fragment
# reads (unet_once B = 1 / 8), and the sampler's per-phase stamps (diagnostic library).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
step diag_m37 60 python -u scripts/dag_diag.py 2000000 37 0
step diag_m1000 60 python -u scripts/dag_diag.py 2000000 1000 0
TAILN=14 step pytest_dag 400 python -u -m pytest tests/test_gpu_train_dag.py -x -v --timeout 120 --timeout-method thread
step pytest_rest 600 python -u -m pytest tests/test_gpu_train_capi.py tests/test_gpu_gemm.py tests/test_gpu_configs.py tests/test_gpu_ddpm.py tests/test_gpu_unet.py tests/test_gpu_autodecoder.py -x -q --timeout 120 --timeout-method thread
step train_ab 300 python -u scripts/train_form_ab.py 4 128
UNET_B=1 step unet_b1 120 python -u scripts/unet_once.py
UNET_B=8 step unet_b8 120 python -u scripts/unet_once.py
TRAIN_STEPS=10 step prof_train 300 rocprofv3 --kernel-trace --stats -d $O/prof -o train --output-format csv -- python3 scripts/train_once.py
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/train_kernel_stats.csv
head -6 $O/train_kernel_stats.csv
LDM_SDF_LIB=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_diag.so TAILN=9 step stamp_sampler 120 python -u scripts/stamp_sampler.py 8
