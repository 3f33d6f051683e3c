#!/bin/bash
# Round 5 -> profiles/r05f/: timeline of the one-launch training step (diagnostic library:
# per-job dequeue / inputs-ready / done stamps) with and without compute, the TrainState
# resume test, and the A/B of both forms on identical random streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
DIAG=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_diag.so
LDM_SDF_LIB=$DIAG TAILN=70 step trace_m1000 120 python -u scripts/trace_dag.py 1000 0 $O/trace_m1000.npz
LDM_SDF_LIB=$DIAG TAILN=12 step trace_nocomp 120 python -u scripts/trace_dag.py 1000 0xF $O/trace_nocomp.npz
LDM_SDF_LIB=$DIAG TAILN=12 step trace_nofence 120 python -u scripts/trace_dag.py 1000 0x1F
step pytest_resume 300 python -u -m pytest tests/test_gpu_train_dag.py -k resume -x -v --timeout 200 --timeout-method thread
step train_ab 300 python -u scripts/train_form_ab.py 4 128
