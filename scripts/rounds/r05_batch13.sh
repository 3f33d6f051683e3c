#!/bin/bash
# Round 5 -> profiles/r05m/: the one-launch step with 64 x 64 jobs for the row (chain) nodes and 128 x 128
# for the weight-gradient products, 64-row bands: DAG bitwise tests, timeline, A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05m
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
LDM_SDF_LIB=$L/libldm_diag.so TAILN=7 step trace_nofence 120 python -u scripts/trace_dag.py 1000 0x10
step train_ab 300 python -u scripts/train_form_ab.py 4 128
# the UNet convs after the round-5 re-pitch: LDS bank conflicts, B = 1
UNET_B=1 PASSES="lds cycles" WORKLOAD=scripts/unet_once.py PMC_OUT=$O/pmc_unet_b1 TAILN=4 step pmc_unet 400 bash scripts/rounds/pmc.sh
python scripts/pmc_by_kernel.py $O/pmc_unet_b1 conv1d > $O/pmc_unet_b1_summary.txt 2>&1; head -12 $O/pmc_unet_b1_summary.txt
