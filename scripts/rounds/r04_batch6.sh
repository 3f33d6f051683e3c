#!/bin/bash
# Round-4 GPU batch 6: first-load latency in a launch chain by writer XCD.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04h
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./scripts/microbench/cold_launch > $O/cold_launch_data.json 2>&1
echo batch6 done
