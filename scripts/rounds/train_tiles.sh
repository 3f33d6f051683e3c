# config-2 training step time per forced GEMM tile (LDM_GEMM_TILE; 0 = automatic choice)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out
for T in ${TILES:-0 1 4 5 10 11 13}; do
  echo "tile $T"; LDM_GEMM_TILE=$T TRAIN_STEPS=300 timeout -k 5 120 python scripts/train_once.py || exit 1
done > gpurun_out/train_tiles.log 2>&1
