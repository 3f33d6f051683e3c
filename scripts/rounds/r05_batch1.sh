#!/bin/bash
# Round 5, first GPU call -> profiles/r05a/: GPU tests + smoke after the hygiene/ABI-7 changes,
# the default bench (new decode_b1 leg, config-3 split), and a fresh decoder PMC at
# B = 64 x 256^3 on the default split kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -c 600 $O/bench.log
DEC_B=64 DEC_R=1 PASSES="cycles insts lds" PMC_OUT=$O/pmc_b64 bash scripts/rounds/pmc.sh \
    > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python scripts/pmc_by_kernel.py $O/pmc_b64 dec_fs > $O/pmc_b64_summary.txt 2>&1
cat $O/pmc_b64_summary.txt | head -20
