# 1M-row forward GEMM: row-pitch padding of the operands (L2 channel spread of the shared W slice)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r02j && export TMPDIR=/tmp
for P in 0 64 8; do
  SHAPE=1048576,512,512 PAD=$P TILES=3,4,15,16,17 NO_REF=1 REPS=5 timeout -k 10 120 python scripts/gemm_bench.py || exit 1
done > gpurun_out/r02j/pad.log 2>&1
