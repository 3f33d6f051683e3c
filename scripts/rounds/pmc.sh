#!/bin/bash
# PMC passes over the decoder workload (scripts/decode_once.py).  One counter group per
# rocprofv3 run (no trace domains with --pmc).  Output: gpurun_out/pmc/<pass>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
WORKLOAD=${WORKLOAD:-scripts/decode_once.py}
mkdir -p $OUT
declare -A P
P[cycles]="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_WAVES"
P[insts]="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
P[lds]="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_UNALIGNED_STALL"
P[fetch]="FETCH_SIZE"
P[write]="WRITE_SIZE"
P[ea]="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
P[l2]="TCC_HIT_sum TCC_MISS_sum"
for name in ${PASSES:-cycles insts lds fetch write ea l2}; do
  echo "== pass $name: ${P[$name]}"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${P[$name]} -d $OUT/$name -o run \
      --output-format csv -- python3 $WORKLOAD > $OUT/$name.log 2>&1
  rc=$?
  echo "   rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/$name.log; exit $rc;; esac
done
