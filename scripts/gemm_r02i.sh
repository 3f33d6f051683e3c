# C19 step per weight-gradient tile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r02i && export TMPDIR=/tmp
for T in 3 4 14 23 2; do
  echo "wg tile $T"; AD_WG_TILE=$T AD_STEPS=2 timeout -k 10 120 python scripts/ad_once.py || exit 1
done > gpurun_out/r02i/ad_tiles.log 2>&1
AD_STEPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02i/ad -o run --output-format csv -- python3 scripts/ad_once.py > gpurun_out/r02i/ad.log 2>&1
