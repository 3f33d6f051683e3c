# 128-deep GEMM stages: GPU tests, training shapes and C19 shapes per tile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r02e && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/r02e/test_gemm.log 2>&1 || exit 1
TILES=4,10,20,21,22,23,24,25 NO_REF=1 REPS=50 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/r02e/train_shapes.log 2>&1 || exit 1
SHAPE=1048576,512,512 TILES=4,15,20,21,22,23,25,26 NO_REF=1 REPS=5 timeout -k 10 120 python scripts/gemm_bench.py > gpurun_out/r02e/big.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_autodecoder.py > gpurun_out/r02e/test_ad.log 2>&1 || exit 1
AD_STEPS=3 timeout -k 10 200 python scripts/ad_once.py > gpurun_out/r02e/ad_once.log 2>&1
