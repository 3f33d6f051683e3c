export TMPDIR=/tmp; O=gpurun_out/tv1; mkdir -p $O; L=$PWD/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_train_dag.py tests/test_gpu_autodecoder.py > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do for lib in libldm_base.so libldm_sdf.so; do
  for o in adfwd adbwd; do LDM_SDF_LIB=$L/$lib OUT=$o SHAPE=1048576,512,512 TILES=15,15 REPS=5 NO_REF=1 timeout -k 10 200 python scripts/gemm_bench.py >> $O/bench_$lib.log 2>&1 || exit 1; done
  LDM_SDF_LIB=$L/$lib AD_STEPS=3 timeout -k 10 300 python scripts/ad_once.py >> $O/ad_$lib.log 2>&1 || exit 1
  LDM_SDF_LIB=$L/$lib AB_FORMS=launches timeout -k 10 300 python scripts/train_form_ab.py 3 128 >> $O/train_$lib.log 2>&1 || exit 1
done; done
