# Round 6: with the two-launch binning the default, its grid cap (bg1/bg4,
# default 8 workgroups per CU) and entries per thread (bp2/bp8, default 4)
# re-checked on the config-3 mix, 1M x 100 B and append.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
VARIANTS="bg4 bg1 bp2 bp8" CASES="--config entries;--config entries --entry-size 100;--config append" \
  REPS=3 STEPS=20 TAG=r06/${1:-binknobs}/ab bash tools/gpu_ab.sh || exit 1
