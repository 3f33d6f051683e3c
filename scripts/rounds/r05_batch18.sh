#!/bin/bash
# Round 5 -> profiles/r05r/: the 8-wave one-launch step with the critical tail first in node
# order, the next queue index fetched as a job ends, no drain for unwatched nodes, and U_k's
# AdamW split (p, m, v as soon as its gradient is final; the bf16 copies after dtemb): DAG
# bitwise tests, timeline, A/B; then the round's validation: the whole GPU suite, smoke, the
# default bench and its rocprofv3 kernel-trace summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
L=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf
step diag_m37 60 python -u scripts/dag_diag.py 2000000 37 0
TAILN=14 step pytest_dag 400 python -u -m pytest tests/test_gpu_train_dag.py -x -v --timeout 120 --timeout-method thread
LDM_SDF_LIB=$L/libldm_diag.so TAILN=60 step trace_m1000 120 python -u scripts/trace_dag.py 1000 0 $O/trace_m1000.npz
step train_ab 300 python -u scripts/train_form_ab.py 4 128
TAILN=4 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=2 step bench 600 python -u bench.py
TAILN=3 step rocprof 900 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/bench_kernel_stats.csv
head -12 $O/bench_kernel_stats.csv
