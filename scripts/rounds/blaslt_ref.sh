# hipBLASLt (torch.mm replayed from a hipGraph) on the training / C19 GEMM shapes, with its
# kernel names and durations from rocprofv3 (the tile configuration is in the name)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/blt && export TMPDIR=/tmp
GRAPH_REF=1 BIG=1 TILES=4,10 REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/blt -o run --output-format csv -- python3 scripts/gemm_bench.py > gpurun_out/blt/bench.log 2>&1
