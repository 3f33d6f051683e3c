#!/bin/bash
# Build libldm_<name>.so from a committed revision of csrc/ (for same-box A/B timing with
# scripts/ablate_decoder.sh run "0 <name> 0 <name>").   usage: scripts/rounds/build_rev.sh <rev> <name>
set -eu
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
rev=$1; name=$2
tmp=$(mktemp -d /tmp/ldm_rev.XXXX)
mkdir -p "$tmp/csrc" "$tmp/include"
git -C "$ROOT" archive "$rev" latent-diffusion-models-for-shape-sdfs_amd/csrc include | tar -x -C "$tmp"
make -s -C "$tmp/latent-diffusion-models-for-shape-sdfs_amd/csrc" -j8 \
  OUT="$ROOT/latent-diffusion-models-for-shape-sdfs_amd/ldm_sdf/libldm_$name.so"
rm -rf "$tmp"
