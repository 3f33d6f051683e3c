# C19 auto-decoder step per tile of the >= 2048-tile launches (LDM_GEMM_TILE_HUGE; 0 = auto)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out
for T in ${TILES:-0 14 3 12 2 9 0}; do
  echo "huge tile $T"; LDM_GEMM_TILE_HUGE=$T AD_STEPS=4 timeout -k 5 120 python scripts/ad_once.py || exit 1
done > gpurun_out/ad_tiles.log 2>&1
