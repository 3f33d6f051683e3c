#!/bin/bash
# Timing ablations of the quarter decoder kernel (diagnostic: the ablated builds compute wrong
# values).  Builds libldm_abl<m>.so per mask m (decoder_q.hip QABL bits), then times each in
# its own process with scripts/ab_decoder.py (variant "q").
#   build (CPU):  scripts/ablate_decoder.sh build "1 2 4 8"
#   run (GPU):    scripts/ablate_decoder.sh run "0 1 2 4 8"   (a name such as "prev" runs
#                 libldm_prev.so: scripts/build_rev.sh builds a committed revision's library)
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
CS="$ROOT/latent-diffusion-models-for-shape-sdfs_amd/csrc"
PK="$ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf"
cmd=$1; masks=$2
for m in $masks; do
  if [ "$cmd" = build ]; then
    [ "$m" = 0 ] && continue
    make -s -C "$CS" -j8 BUILD=build_abl$m OUT="$PK/libldm_abl$m.so" \
      HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function -DQABL=$m"
  else
    case $m in 0) lib="$PK/libldm_sdf.so";; [0-9]*) lib="$PK/libldm_abl$m.so";; *) lib="$PK/libldm_$m.so";; esac
    echo "== QABL=$m"
    LDM_SDF_LIB="$lib" AB_VARIANTS=q timeout -k 10 200 python "$ROOT/scripts/ab_decoder.py" ${AB_B:-4} 256 ${AB_R:-3}
  fi
done
