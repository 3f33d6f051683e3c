#!/bin/bash
# Round-4 GPU batch 5: launch-start costs (cold data / cold instruction fetch) + GPU tests.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04f
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./scripts/microbench/cold_launch > $O/cold_launch.json 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo batch5 done
