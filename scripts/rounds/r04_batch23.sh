#!/bin/bash
# Round-4 GPU batch 23: A/B of the direct staging's argument pin (product build vs -DLDM_CONV_PIN=0),
# interleaved, UNet steps/s at B = 1 and B = 8.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04y
mkdir -p $O
cd $GRAFT_REPO_ROOT
NOPIN=$GRAFT_REPO_ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_nopin.so
for i in 1 2 3; do
  for B in 1 8; do
    echo "pin B=$B" >> $O/ab_pin.log
    UNET_B=$B UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py 2>/dev/null >> $O/ab_pin.log
    echo "nopin B=$B" >> $O/ab_pin.log
    LDM_SDF_LIB=$NOPIN UNET_B=$B UNET_STEPS=1000 timeout -k 10 120 python -u scripts/unet_once.py 2>/dev/null >> $O/ab_pin.log
  done
done
echo batch23 done
