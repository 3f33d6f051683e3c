set -u
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_gemm}
mkdir -p $OUT
for name in ${PASSES:-cycles insts lds l2 ta}; do
  case $name in
    cycles) C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_WAVES";;
    insts) C="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE";;
    lds) C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_UNALIGNED_STALL";;
    l2) C="TCC_HIT_sum TCC_MISS_sum";;
    ta) C="TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE";;
  esac
  SHAPE=${SHAPE:-1024,1024,2048} TILES=${TILES:-1,10} NO_REF=1 REPS=20 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $OUT/$name -o run --output-format csv -- python3 scripts/gemm_bench.py > $OUT/$name.log 2>&1 || exit $?
done
