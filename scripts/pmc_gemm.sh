set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_gemm
for name in cycles insts lds; do
  case $name in
    cycles) C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_WAVES";;
    insts) C="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE";;
    lds) C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_UNALIGNED_STALL";;
  esac
  SHAPE=1024,1024,2048 TILES=1,5,6 NO_REF=1 REPS=20 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_gemm/$name -o run --output-format csv -- python3 scripts/gemm_bench.py > gpurun_out/pmc_gemm/$name.log 2>&1 || exit $?
done
SHAPE=1024,1024,2048 TILES=1,5,6 NO_REF=1 REPS=20 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_gemm/trace -o run --output-format csv -- python3 scripts/gemm_bench.py > gpurun_out/pmc_gemm/trace.log 2>&1
