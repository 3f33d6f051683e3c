#!/bin/bash
# One GPU session: parity tests -> smoke -> short bench -> rocprof kernel stats.
# Stops at the first crash/timeout (exit 124/134/137/139 or signal) so nothing else touches a
# possibly-faulted GPU.  Logs go to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139|13[0-9]|14[0-9]) return 0;; *) return 1;; esac; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return $rc
}
STAGES="${STAGES:-pytest smoke bench prof}"
for s in $STAGES; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread ${PYTEST_ARGS:-} ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 900 python bench.py ${BENCH_ARGS:-} ;;
    micro)  run handoff_latency 120 scripts/microbench/handoff_latency ;;
    prof)   cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
            run rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run \
                --output-format csv -- python3 bench.py ${PROF_ARGS:-} ;;
  esac
done
exit 0
