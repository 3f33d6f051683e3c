#!/bin/bash
# Round 5 -> profiles/r05w/: which of the three UNet LDS bank-conflict changes costs time
# (the full set measured 3.6 % slower at B = 1 in profiles/r05v while the conflicts fell from
# 0.37-0.54 to 0.08-0.27 of LDS-active cycles).  unet_once.py interleaved over libraries built
# from the same unet.hip with -D UNET_XROT / UNET_WSWAP / UNET_RED_SHIFT: old (HEAD before the
# change), red (reduction re-pitch only), redw (+ weight swap), redx (+ window rotation), full.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
L=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf
for rep in 1 2; do
  for b in 1 8; do
    for v in old red redw redx; do
      TAILN=1 UNET_B=$b LDM_SDF_LIB=$L/libldm_sdf_ab$v.so step ab_${v}_b${b}_$rep 120 python -u scripts/unet_once.py
    done
    TAILN=1 UNET_B=$b step ab_full_b${b}_$rep 120 python -u scripts/unet_once.py
  done
done
