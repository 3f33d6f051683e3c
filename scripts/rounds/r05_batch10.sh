#!/bin/bash
# Round 5 -> profiles/r05j/: the one-launch step on 128 x 128 GEMM jobs (one workgroup per CU,
# 4-deep ring) and 4-tile AdamW jobs: DAG bitwise tests + the launch-path GEMM / training tests,
# the timeline with all fences / without fences / without release / without acquire (timing
# only), the A/B of both forms; the sampler timed on the product and the diagnostic build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
DIAG=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_diag.so
step diag_m37 60 python -u scripts/dag_diag.py 2000000 37 0
step diag_m1000 60 python -u scripts/dag_diag.py 2000000 1000 0
TAILN=14 step pytest_dag 400 python -u -m pytest tests/test_gpu_train_dag.py -x -v --timeout 120 --timeout-method thread
step pytest_gemm 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_train_capi.py -x -q --timeout 120 --timeout-method thread
LDM_SDF_LIB=$DIAG TAILN=60 step trace_m1000 120 python -u scripts/trace_dag.py 1000 0 $O/trace_m1000.npz
LDM_SDF_LIB=$DIAG TAILN=7 step trace_nofence 120 python -u scripts/trace_dag.py 1000 0x10
LDM_SDF_LIB=$DIAG TAILN=7 step trace_norel 120 python -u scripts/trace_dag.py 1000 0x20
LDM_SDF_LIB=$DIAG TAILN=7 step trace_noacq 120 python -u scripts/trace_dag.py 1000 0x40
step train_ab 300 python -u scripts/train_form_ab.py 4 128
step sampler_product 120 python -u scripts/sampler_time.py
LDM_SDF_LIB=$DIAG step sampler_diag 120 python -u scripts/sampler_time.py
