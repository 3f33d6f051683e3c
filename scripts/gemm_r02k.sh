# specialised epilogue: GEMM tests, big + training shapes per tile, AD step, config-2 training
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r02k && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_autodecoder.py tests/test_gpu_train_capi.py > gpurun_out/r02k/tests.log 2>&1 || exit 1
SHAPE=1048576,512,512 TILES=3,4,14,15,16,17,18,20,23,26 NO_REF=1 REPS=5 OUT=cb timeout -k 10 120 python scripts/gemm_bench.py > gpurun_out/r02k/big.log 2>&1 || exit 1
TILES=3,4,10,20,21,24 NO_REF=1 REPS=50 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/r02k/train_shapes.log 2>&1 || exit 1
AD_STEPS=3 timeout -k 10 120 python scripts/ad_once.py > gpurun_out/r02k/ad.log 2>&1 || exit 1
TRAIN_STEPS=300 timeout -k 10 120 python scripts/train_once.py > gpurun_out/r02k/train.log 2>&1
