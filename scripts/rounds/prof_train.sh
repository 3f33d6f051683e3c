# config-2 training step kernel trace (auto GEMM tiles); $1 = output tag (default r02f)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && tag=${1:-r02f} && mkdir -p gpurun_out/$tag && export TMPDIR=/tmp
TRAIN_STEPS=100 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/train -o run --output-format csv -- python3 scripts/train_once.py > gpurun_out/$tag/train.log 2>&1
f=$(ls gpurun_out/$tag/train/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/$tag/train/run_kernel_trace.csv)
python3 scripts/trace_summary.py "$f" "" 24 > gpurun_out/$tag/train_step_trace.txt
