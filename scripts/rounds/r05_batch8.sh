#!/bin/bash
# Round 5 -> profiles/r05h/: the one-launch step with write-through (sc1) stores throughout, so
# a release has no dirty L2 lines to write back: DAG bitwise tests + the launch-path GEMM /
# training tests (shared epilogue header), then the timeline with all fences, without fences,
# without release, without acquire (timing only), and the A/B of both forms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
DIAG=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_diag.so
TAILN=14 step pytest_dag 400 python -u -m pytest tests/test_gpu_train_dag.py -x -v --timeout 120 --timeout-method thread
step pytest_gemm 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_train_capi.py -x -q --timeout 120 --timeout-method thread
LDM_SDF_LIB=$DIAG TAILN=60 step trace_m1000 120 python -u scripts/trace_dag.py 1000 0 $O/trace_m1000.npz
LDM_SDF_LIB=$DIAG TAILN=7 step trace_nofence 120 python -u scripts/trace_dag.py 1000 0x10
LDM_SDF_LIB=$DIAG TAILN=7 step trace_norel 120 python -u scripts/trace_dag.py 1000 0x20
LDM_SDF_LIB=$DIAG TAILN=7 step trace_noacq 120 python -u scripts/trace_dag.py 1000 0x40
step train_ab 300 python -u scripts/train_form_ab.py 4 128
