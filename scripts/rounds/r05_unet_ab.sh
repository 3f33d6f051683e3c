#!/bin/bash
# Round 5 -> profiles/r05v/: the UNet staging-store rotation (window stores rotated per lane,
# bf16 weight halves swapped, reduction rows re-pitched).  GPU UNet tests on the
# new library, then unet_once.py interleaved old (HEAD's unet.hip, libldm_sdf_abold.so) / new at
# B = 1 and B = 8, then the LDS PMC pass on the new library.  Also the one-launch training
# step with the weight-copy operands loaded through the L2 (Node::stat; then the default, now
# ldm_dev_train_dag_flags 0x200) against all-sc1 loads (then 0x200, now the default) and the
# launch path (SKIP_TRAIN=1: UNet only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
OLD=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_sdf_abold.so
TAILN=3 step pytest_unet 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_unet.py
TAILN=3 step pytest_dag 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train_dag.py
if [ -z "${SKIP_TRAIN:-}" ]; then
TAILN=3 step train_ab_plain 300 python -u scripts/train_form_ab.py 4 128
TAILN=3 DAG_FLAGS=0x200 step train_ab_sc1 300 python -u scripts/train_form_ab.py 4 128
TAILN=3 step train_ab_plain2 300 python -u scripts/train_form_ab.py 4 128
fi
for rep in 1 2 3; do
  for b in 1 8; do
    TAILN=1 UNET_B=$b LDM_SDF_LIB=$OLD step ab_old_b${b}_$rep 120 python -u scripts/unet_once.py
    TAILN=1 UNET_B=$b step ab_new_b${b}_$rep 120 python -u scripts/unet_once.py
  done
done
UNET_B=1 UNET_STEPS=100 PASSES="lds cycles" WORKLOAD=scripts/unet_once.py PMC_OUT=$O/pmc_unet_b1 TAILN=4 step pmc_unet 400 bash scripts/rounds/pmc.sh
python scripts/pmc_by_kernel.py $O/pmc_unet_b1 conv1d > $O/pmc_unet_b1_summary.txt 2>&1; head -24 $O/pmc_unet_b1_summary.txt
