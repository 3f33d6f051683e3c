# config-2 training: GEMM tile per launch size class (LDM_GEMM_TILE_SMALL/MID/BIG; 0 = auto)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out
for cfg in "0 4 4" "0 4 1" "0 1 1" "0 4 5" "0 4 8" "0 5 5" "0 11 4" "0 4 4"; do
  set -- $cfg
  echo "small $1 mid $2 big $3"
  LDM_GEMM_TILE_SMALL=$1 LDM_GEMM_TILE_MID=$2 LDM_GEMM_TILE_BIG=$3 TRAIN_STEPS=300 timeout -k 5 120 python scripts/train_once.py || exit 1
done > gpurun_out/train_tiles2.log 2>&1
