#!/bin/bash
# Round 5 final validation -> profiles/r05z4/: the A/B of the training-step forms, the whole GPU
# suite, smoke, the default bench and the rocprofv3 kernel-trace summary of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05z4
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}

TAILN=4 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=2 step bench 600 python -u bench.py
TAILN=3 step rocprof 900 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/bench_kernel_stats.csv
head -12 $O/bench_kernel_stats.csv
