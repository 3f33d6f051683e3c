# register-staged 128-deep variants vs LDS-DMA; AD step with the 64x64 default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r02g && export TMPDIR=/tmp
SHAPE=1024,1024,2048 TILES=4,20,27,28,4,20,27,28 NO_REF=1 REPS=100 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/r02g/train_shapes.log 2>&1 || exit 1
SHAPE=1024,1024,1024 TILES=4,20,27,28 NO_REF=1 REPS=100 timeout -k 10 200 python scripts/gemm_bench.py >> gpurun_out/r02g/train_shapes.log 2>&1 || exit 1
SHAPE=1048576,512,512 TILES=4,15,20,27,28 NO_REF=1 REPS=5 timeout -k 10 120 python scripts/gemm_bench.py > gpurun_out/r02g/big.log 2>&1 || exit 1
AD_STEPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02g/ad -o run --output-format csv -- python3 scripts/ad_once.py > gpurun_out/r02g/ad.log 2>&1
