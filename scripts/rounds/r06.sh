#!/bin/bash
# Round 6 GPU calls, one batch per argument (bash scripts/rounds/r06.sh <batch> <outdir>); every
# step runs under its own time limit and the batch stops at the first failure.  Output goes to
# gpurun_out/<outdir>/; the logs that back a DESIGN.md statement are copied to profiles/<outdir>/.
#   guards   the one-launch / data-parallel training tests, the whole GPU suite and smoke
#   debug    the same training tests and the GEMM tests against the DEBUG=1 library
#            (LDM_DASSERT bounds traps, wt_store.h extents), then the whole GPU suite on it
#   bench    the default bench and the rocprofv3 kernel-trace summary of the same command
#   sampler  the sampler build A/B (scripts/sampler_time.py against each library in $SL_LIBS)
#   decoder  the decoder part stamps (scripts/stamp_split.py on each FS_STAMP library in $FS_LIBS)
#   multirank  bench.py --gpus 2 with both ranks on cuda:0 over gloo (the N > 1 control flow)
#   adam     AdamW tile A/B over the libraries in $AD_LIBS (kernel time, config-2 step)
#   dlib     decoder build A/B over the libraries in $DEC_LIBS (scripts/decode_time.py)
#   mc       marching-cubes build A/B over the libraries in $MC_LIBS (+ tests with MC_TESTS=1)
#   unet     UNet build A/B over the libraries in $UNET_LIBS (+ tests with UNET_TESTS=1)
#   mregs    scripts/microbench/mfma_regs (a k-step's speed vs the registers of its operands)
#   lds      scripts/microbench/lds_half_latency (LDS read latency / stream below vs above 64 KiB)
#            and scripts/microbench/acc_range (a k-step on each of two live accumulator sets)
#   first    config 3's first call in a fresh process, with a kernel + HIP API trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
B=${1:?batch}
O=gpurun_out/${2:?outdir}
mkdir -p $O
step() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc $rc"; tail -${TAILN:-6} $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
LIB=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
case $B in
  guards)
    TAILN=4 step dag_product 400 $PYT tests/test_gpu_train_dag.py tests/test_gpu_train_dp.py
    TAILN=4 step pytest_gpu 900 $PYT tests -m gpu
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
    ;;
  debug)
    LDM_SDF_LIB=$LIB/libldm_sdf_debug.so TAILN=4 step dag_debug 600 $PYT tests/test_gpu_train_dag.py tests/test_gpu_train_dp.py
    LDM_SDF_LIB=$LIB/libldm_sdf_debug.so TAILN=4 step gemm_debug 600 $PYT tests/test_gpu_gemm.py tests/test_gpu_train_capi.py
    LDM_SDF_LIB=$LIB/libldm_sdf_debug.so TAILN=4 step pytest_gpu_debug 900 $PYT tests -m gpu -k "not test_native_library_is_loaded"
    ;;
  bench)
    TAILN=2 step bench 600 python -u bench.py
    TAILN=3 step rocprof 900 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py
    find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/bench_kernel_stats.csv
    head -12 $O/bench_kernel_stats.csv
    ;;
  sampler)
    [ -n "${SL_TESTS:-}" ] && TAILN=3 step sampler_tests 600 $PYT tests/test_gpu_ddpm.py tests/test_sampler_codegen.py
    for L in ${SL_LIBS:?}; do
      LDM_SDF_LIB=$LIB/$L TAILN=3 step sampler_${L%.so} 300 python -u scripts/sampler_time.py
    done
    ;;
  decoder)
    for L in ${FS_LIBS:?}; do
      LDM_SDF_LIB=$LIB/$L TAILN=70 step stamp_${L%.so} 300 python -u scripts/stamp_split.py
    done
    ;;
  multirank)
    # the N > 1 flow of bench.py (z-slab gathers, rank-0 legs, barriers) rehearsed on one GPU:
    # 2 ranks on cuda:0 over gloo (timings meaningless: both ranks share the device)
    LDM_BENCH_BACKEND=gloo LDM_BENCH_TRACE=1 LDM_BENCH_WATCHDOG=150 TAILN=40 step bench_gloo2 300 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu --no-ddpm --no-config5 --train-steps 5 --ad-steps 1
    LDM_BENCH_BACKEND=gloo LDM_BENCH_TRACE=1 LDM_BENCH_WATCHDOG=170 TAILN=40 step bench_gloo2_all 300 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu --train-steps 5 --ad-steps 1
    ;;
  adam)
    # the AdamW tile A/B: correctness first, then kernel time and the config-2 step per library
    TAILN=3 step adam_tests 400 $PYT tests/test_gpu_train_capi.py tests/test_gpu_train_dag.py
    for rep in 1 2; do
      for L in ${AD_LIBS:?}; do
        LDM_SDF_LIB=$LIB/$L TAILN=1 step adamw_${L%.so}_$rep 120 python -u scripts/adamw_time.py
        LDM_SDF_LIB=$LIB/$L TAILN=3 step train_${L%.so}_$rep 300 python -u scripts/train_form_ab.py 3 128
      done
    done
    ;;
  dlib)
    # decoder build A/B: scripts/decode_time.py per library in $DEC_LIBS, alternating
    [ -n "${DEC_TESTS:-}" ] && TAILN=3 step dec_tests 600 $PYT tests/test_gpu_decoder.py tests/test_gpu_configs.py
    for rep in 1 2 3; do
      for L in ${DEC_LIBS:?}; do
        LDM_SDF_LIB=$LIB/$L TAILN=1 step dec_${L%.so}_$rep 120 python -u scripts/decode_time.py 8 256 5
      done
    done
    ;;
  mc)
    # marching-cubes build A/B: wall time per mesh and the rocprof kernel stats, per library
    [ -n "${MC_TESTS:-}" ] && TAILN=3 step mc_tests 300 $PYT tests/test_gpu_mc.py
    for rep in 1 2; do
      for L in ${MC_LIBS:?}; do
        LDM_SDF_LIB=$LIB/$L TAILN=1 step mc_${L%.so}_$rep 120 python -u scripts/mc_once.py 50
        LDM_SDF_LIB=$LIB/$L TAILN=1 step mcprof_${L%.so}_$rep 300 rocprofv3 --kernel-trace --stats -d $O/mcprof_${L%.so}_$rep -o mc --output-format csv -- python3 scripts/mc_once.py 50
        find $O/mcprof_${L%.so}_$rep -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/mc_kernel_stats_${L%.so}_$rep.csv
      done
    done
    ;;
  unet)
    # UNet build A/B: steps/s at B = 1 and B = 8 and the sample's hash, per library
    [ -n "${UNET_TESTS:-}" ] && TAILN=3 step unet_tests 600 $PYT tests/test_gpu_unet.py
    for rep in 1 2; do
      for L in ${UNET_LIBS:?}; do
        LDM_SDF_LIB=$LIB/$L UNET_REPS=3 TAILN=3 step unet_${L%.so}_$rep 120 python -u scripts/unet_once.py
        LDM_SDF_LIB=$LIB/$L UNET_REPS=2 UNET_B=8 TAILN=2 step unet8_${L%.so}_$rep 120 python -u scripts/unet_once.py
      done
    done
    ;;
  dagab)
    # one-launch training step A/B (timing) over the libraries in $DAG_LIBS, alternating
    for rep in 1 2; do
      for L in ${DAG_LIBS:?}; do
        LDM_SDF_LIB=$LIB/$L AB_FORMS=dag TAILN=2 step dag_${L%.so}_$rep 300 python -u scripts/train_form_ab.py 3 128
      done
    done
    ;;
  mregs)
    TAILN=30 step mfma_regs 120 ./scripts/microbench/mfma_regs
    TAILN=28 step loop_replay 120 ./scripts/microbench/loop_replay
    ;;
  lds)
    TAILN=14 step lds_half 120 ./scripts/microbench/lds_half_latency
    TAILN=4 step acc_range 120 ./scripts/microbench/acc_range
    ;;
  first)
    TAILN=20 step first_call 300 python -u scripts/config3_first_call.py
    TAILN=3 step first_trace 600 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $O/first -o first --output-format csv -- python3 scripts/config3_first_call.py
    ;;
  *) echo "unknown batch $B"; exit 2 ;;
esac
