#!/bin/bash
# Round 5 -> profiles/r05n/: the one-launch step with fence-free hand-offs (sc1 stores AND sc1
# loads of every handed-off byte, one workgroup per CU: the MI355X guide's table row 1): DAG
# bitwise tests + launch-path GEMM / training tests (shared headers), timeline with and without
# the release/acquire form (flag 0x80), A/B of the forms; the sampler with every stamp mark
# (libldm_slmarks31.so), s_sleep naps at the marks (naps31) and before the polls only (naps16).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05n
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
step pytest_gemm 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_train_capi.py -x -q --timeout 120 --timeout-method thread
LDM_SDF_LIB=$L/libldm_diag.so TAILN=60 step trace_m1000 120 python -u scripts/trace_dag.py 1000 0 $O/trace_m1000.npz
LDM_SDF_LIB=$L/libldm_diag.so TAILN=7 step trace_fences 120 python -u scripts/trace_dag.py 1000 0x80
step train_ab 300 python -u scripts/train_form_ab.py 4 128
step sampler_product 120 python -u scripts/sampler_time.py
for v in marks31 naps31 naps16; do
  LDM_SDF_LIB=$L/libldm_sl$v.so TAILN=3 step sampler_$v 120 python -u scripts/sampler_time.py
done
