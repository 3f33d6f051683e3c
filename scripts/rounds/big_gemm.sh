# C19 (auto-decoder) GEMM shapes on ldm_gemm_bf16 per tile vs torch.mm; bf16 sampler deviations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
SHAPE=1048576,512,512 TILES=${TILES:-1,2,3,4,6,7,9,12,14,15} REPS=5 timeout -k 5 120 python scripts/gemm_bench.py > gpurun_out/big_gemm.log 2>&1 || exit 1
SHAPE=512,512,1048576 SPLITK=4 TILES=1,3,4 NO_REF=1 REPS=5 timeout -k 5 120 python scripts/gemm_bench.py >> gpurun_out/big_gemm.log 2>&1 || exit 1
timeout -k 5 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_ddpm.py -k "vs_oracle_rounded" > gpurun_out/bf16_dev.log 2>&1
