#!/bin/bash
# Round 5 -> profiles/r05o/: the one-launch step with the weight-gradient products on 128 x 128
# jobs (row nodes classified by role, not by M == batch: at B = 1000 the batch is padded to 1024
# = H, so every dW / dU product had been taken for a row node); DAG bitwise tests, timeline, A/B;
# the sampler: the SL_STAMP kernel linked with the product objects (libldm_slstamp.so) and the
# product kernel linked with the diagnostic build's other objects (libldm_slstale.so) -- where
# does the stamped build's +18 % come from.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05o
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
LDM_SDF_LIB=$L/libldm_diag.so TAILN=60 step trace_m1000 120 python -u scripts/trace_dag.py 1000 0 $O/trace_m1000.npz
step train_ab 300 python -u scripts/train_form_ab.py 4 128
step sampler_product 120 python -u scripts/sampler_time.py
for v in slstamp slstale diag; do
  LDM_SDF_LIB=$L/libldm_$v.so TAILN=3 step sampler_$v 120 python -u scripts/sampler_time.py
done
