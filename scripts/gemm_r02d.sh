# new ldm_gemm_bf16 variants (persistent tiles, split-K, RELU_BWD): GPU tests, then the C19
# shapes per tile, hipBLASLt (graph-replayed torch.mm) beside them under rocprofv3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r02d && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/r02d/test_gemm.log 2>&1 || exit 1
SHAPE=1048576,512,512 TILES=4,15,16,17,18 REPS=5 timeout -k 10 120 python scripts/gemm_bench.py > gpurun_out/r02d/big.log 2>&1 || exit 1
SHAPE=1048576,256,512 TILES=4,16,17,18 NO_REF=1 REPS=5 timeout -k 10 120 python scripts/gemm_bench.py >> gpurun_out/r02d/big.log 2>&1 || exit 1
GRAPH_REF=1 TILES=4,16,18 REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02d/blt -o run --output-format csv -- python3 scripts/gemm_bench.py > gpurun_out/r02d/blt.log 2>&1
