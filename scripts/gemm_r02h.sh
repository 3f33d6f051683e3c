# blocked sample-axis operands: GEMM + AD GPU tests, AD step profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r02h && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_autodecoder.py > gpurun_out/r02h/tests.log 2>&1 || exit 1
AD_STEPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02h/ad -o run --output-format csv -- python3 scripts/ad_once.py > gpurun_out/r02h/ad.log 2>&1
