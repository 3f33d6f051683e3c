#!/bin/bash
# Round 5 -> profiles/r05x/: does workgroup b of the one-launch training step run on XCD b % 8,
# as its queue mapping assumes?  The diagnostic build records each job's XCC_ID (trace_dag.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
L=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf
LDM_SDF_LIB=$L/libldm_diag.so TAILN=60 step trace_m1000 120 python -u scripts/trace_dag.py 1000 0
LDM_SDF_LIB=$L/libldm_diag.so TAILN=60 step trace_m1000_2 120 python -u scripts/trace_dag.py 1000 0
