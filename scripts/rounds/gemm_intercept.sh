# GEMM microbench sweeps for the config-2 shapes (row-pitch padding, tiles); logs in gpurun_out/gi
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/gi && export TMPDIR=/tmp
for P in 0 64 128 256; do
  SHAPE=1024,1024,2048 PAD=$P OUT=c TILES=4,5,10,11 NO_REF=1 REPS=200 timeout -k 5 60 python scripts/gemm_bench.py || exit 1
  SHAPE=1024,1024,1024 PAD=$P OUT=c TILES=4,10 NO_REF=1 REPS=200 timeout -k 5 60 python scripts/gemm_bench.py || exit 1
done > gpurun_out/gi/pad.log 2>&1
