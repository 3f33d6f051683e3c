# PMC: ldm_gemm_bf16 (tiles 4 / 20 / 24) beside hipBLASLt (graph-replayed torch.mm) on the
# config-2 block GEMM 1024x1024x2048; then the C19 bf16 step under rocprofv3 --kernel-trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r02f && export TMPDIR=/tmp
OUT=gpurun_out/r02f
for name in cycles insts lds l2 ta tcp; do
  case $name in
    cycles) C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_WAVES";;
    insts) C="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE";;
    lds) C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM";;
    l2) C="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum";;
    ta) C="TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE";;
    tcp) C="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum";;
  esac
  GRAPH_REF=1 SHAPE=1024,1024,2048 TILES=4,20,24 REPS=20 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $OUT/pmc/$name -o run --output-format csv -- python3 scripts/gemm_bench.py > $OUT/$name.log 2>&1 || exit $?
done
AD_STEPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ad -o run --output-format csv -- python3 scripts/ad_once.py > $OUT/ad.log 2>&1
