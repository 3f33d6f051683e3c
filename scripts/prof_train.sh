# config-2 training step kernel trace (auto GEMM tiles)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r02m && export TMPDIR=/tmp
TRAIN_STEPS=100 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02m/train -o run --output-format csv -- python3 scripts/train_once.py > gpurun_out/r02m/train.log 2>&1
