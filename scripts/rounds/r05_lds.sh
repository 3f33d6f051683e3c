#!/bin/bash
# Round 5 -> profiles/r05y/: the one-launch training step with deeper LDS rings (159 KiB of LDS:
# TILE_ROW 6 stages, TILE_K2 9; the product's 128 KiB: 5 and 8), libldm_sdf_ablds.so built with
# -DDAG_LDS_KB=159: bitwise tests, then train_form_ab.py interleaved product / deeper.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05y
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
LDS=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_sdf_ablds.so
LDM_SDF_LIB=$LDS TAILN=3 step pytest_dag_lds 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train_dag.py
for rep in 1 2; do
  TAILN=3 step ab_prod_$rep 300 python -u scripts/train_form_ab.py 4 128
  LDM_SDF_LIB=$LDS TAILN=3 step ab_lds_$rep 300 python -u scripts/train_form_ab.py 4 128
done
