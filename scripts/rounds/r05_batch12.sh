#!/bin/bash
# Round 5 -> profiles/r05l/: the one-launch step with a software-pipelined k-loop (fragments of
# stage j + 1 read while stage j's MFMAs run) on 128-row bands (product) and 64-row bands
# (libldm_dag64.so): DAG bitwise tests on both, timeline of the 128 form, A/B of the forms; the
# sampler with the polling waves at issue priority 0 (libldm_slprio<p>.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05l
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
LDM_SDF_LIB=$L/libldm_dag64.so TAILN=14 step pytest_dag64 400 python -u -m pytest tests/test_gpu_train_dag.py -x -v --timeout 120 --timeout-method thread
LDM_SDF_LIB=$L/libldm_diag.so TAILN=60 step trace_m1000 120 python -u scripts/trace_dag.py 1000 0 $O/trace_m1000.npz
LDM_SDF_LIB=$L/libldm_diag.so TAILN=7 step trace_nofence 120 python -u scripts/trace_dag.py 1000 0x10
step train_ab 300 python -u scripts/train_form_ab.py 4 128
LDM_SDF_LIB=$L/libldm_dag64.so AB_FORMS=dag step train_ab_dag64 300 python -u scripts/train_form_ab.py 4 128
step sampler_product 120 python -u scripts/sampler_time.py
for p in 1 3; do
  LDM_SDF_LIB=$L/libldm_slprio$p.so TAILN=3 step sampler_prio$p 120 python -u scripts/sampler_time.py
done
