# auto tile rule: AD weight-gradient tile sweep, config-2 training per forced tile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r02l && export TMPDIR=/tmp
for T in 3 14 23 24 20; do
  echo "wg tile $T"; AD_WG_TILE=$T AD_STEPS=3 timeout -k 5 120 python scripts/ad_once.py || exit 1
done > gpurun_out/r02l/ad_tiles.log 2>&1
for T in 0 4 20 24; do
  echo "tile $T"; LDM_GEMM_TILE=$T TRAIN_STEPS=300 timeout -k 5 120 python scripts/train_once.py || exit 1
done > gpurun_out/r02l/train_tiles.log 2>&1
