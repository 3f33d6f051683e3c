#!/bin/bash
# Round-4 GPU batch 1: GPU tests, graph-node and weight-stream microbenchmarks, the default bench,
# the marching-cubes kernel profile, the decoder group-base A/B and a UNet step trace.
# Every GPU step has its own time limit; the first failure ends the script.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04a
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 ./scripts/microbench/graph_chain_latency > $O/graph_node_latency.json 2>&1
timeout -k 10 120 ./scripts/microbench/weight_stream > $O/weight_stream.json 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
LDM_SDF_LIB=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_dev.so AB_VARIANTS=s,s2,s,s2 timeout -k 10 200 python -u scripts/ab_decoder.py 8 256 4 > $O/ab_decoder_groupbase.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_mc -o mc -- python3 $GRAFT_REPO_ROOT/scripts/mc_once.py 20 > $O/mc_once.log 2>&1
UNET_STEPS=50 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_unet -o unet -- python3 $GRAFT_REPO_ROOT/scripts/unet_once.py > $O/unet_once.log 2>&1
echo batch1 done
