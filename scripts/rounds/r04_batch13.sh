#!/bin/bash
# Round-4 GPU batch 13 (validation): all GPU tests, smoke, the default bench, and a rocprofv3
# kernel-trace summary of the same bench command (profiles/r04h).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04o
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 $GRAFT_REPO_ROOT/bench.py > $O/bench_rocprof.log 2>&1
echo batch13 done
