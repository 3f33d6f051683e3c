#!/bin/bash
# Round 5 -> profiles/r05u/: PMC evidence -- the UNet convs after the round-5 re-pitch (LDS bank
# conflicts, waits; 100 steps so the counter pass stays short) and the one-launch training
# step's memory traffic (FETCH_SIZE, L2 hit / miss).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05u
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
UNET_B=1 UNET_STEPS=100 PASSES="lds cycles" WORKLOAD=scripts/unet_once.py PMC_OUT=$O/pmc_unet_b1 TAILN=4 step pmc_unet 400 bash scripts/rounds/pmc.sh
python scripts/pmc_by_kernel.py $O/pmc_unet_b1 conv1d > $O/pmc_unet_b1_summary.txt 2>&1; head -24 $O/pmc_unet_b1_summary.txt
TRAIN_STEPS=20 PASSES="cycles fetch write l2" WORKLOAD=scripts/dag_once.py PMC_OUT=$O/pmc_dag TAILN=4 step pmc_dag 400 bash scripts/rounds/pmc.sh
python scripts/pmc_by_kernel.py $O/pmc_dag train_dag > $O/pmc_dag_summary.txt 2>&1; head -12 $O/pmc_dag_summary.txt
