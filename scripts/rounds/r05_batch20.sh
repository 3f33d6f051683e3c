#!/bin/bash
# Round 5 -> profiles/r05t/: the one-launch step's claim scheduler (a workgroup takes only a
# READY job -- its XCD's chain list first, then the rest -- by CAS on the list head; it never
# holds a job while waiting): DAG bitwise tests (both schedulers), timelines, A/B of the forms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05t
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
step diag_m37_claim 60 python -u scripts/dag_diag.py 2000000 37 0x100
TAILN=16 step pytest_dag 400 python -u -m pytest tests/test_gpu_train_dag.py -x -v --timeout 120 --timeout-method thread
LDM_SDF_LIB=$L/libldm_diag.so TAILN=60 step trace_claim 120 python -u scripts/trace_dag.py 1000 0x100 $O/trace_claim.npz
LDM_SDF_LIB=$L/libldm_diag.so TAILN=8 step trace_queue 120 python -u scripts/trace_dag.py 1000 0
DAG_FLAGS=0x100 step train_ab_claim 300 python -u scripts/train_form_ab.py 6 128
