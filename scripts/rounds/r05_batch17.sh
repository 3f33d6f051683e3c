#!/bin/bash
# Round 5 -> profiles/r05q/: the 8-wave one-launch step with 128-deep stages for the kgp-2 nodes
# (TILE_K2L) and single-stage prologues (no vmcnt(0) over the whole ring): DAG bitwise tests,
# launch-path GEMM / training tests, timeline, A/B; the product sampler now built with its phase
# stamps: DDPM tests + timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
L=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf
step diag_m37 60 python -u scripts/dag_diag.py 2000000 37 0
TAILN=14 step pytest_dag 400 python -u -m pytest tests/test_gpu_train_dag.py -x -v --timeout 120 --timeout-method thread
step pytest_more 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_train_capi.py tests/test_gpu_ddpm.py -x -q --timeout 120 --timeout-method thread
LDM_SDF_LIB=$L/libldm_diag.so TAILN=60 step trace_m1000 120 python -u scripts/trace_dag.py 1000 0 $O/trace_m1000.npz
step train_ab 300 python -u scripts/train_form_ab.py 4 128
step sampler_product 120 python -u scripts/sampler_time.py
