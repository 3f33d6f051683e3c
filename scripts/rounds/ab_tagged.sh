# replica sampler: tagged-granule hand-offs vs XCD barriers (bit-identity + steps/s), ddpm tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r02n && export TMPDIR=/tmp
for B in 8 1 16; do MODES=replica,replica0,replica,replica0 timeout -k 10 120 python scripts/ab_sample_loop.py $B || exit 1; done > gpurun_out/r02n/ab.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ddpm.py tests/test_gpu_configs.py > gpurun_out/r02n/tests.log 2>&1
