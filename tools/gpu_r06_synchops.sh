# Round 6: the sync search's validation hops (default 6) against 4, 5, 8 on
# the replay sweep after the part-size change.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
VARIANTS="sh4 sh5 sh8" CASES="--config replay --value-len 64;--config replay --value-len 256;--config replay --value-len 1024;--config replay --value-len 2048;--config replay --value-len 8192" \
  REPS=2 STEPS=10 TAG=r06/${1:-synchops}/ab bash tools/gpu_ab.sh || exit 1
