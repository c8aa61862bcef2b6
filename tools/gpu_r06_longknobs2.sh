# Round 6: the long-phase re-check, second pass: role split off (sp0), octet
# cost 6 (oc6) and both, on every table workload.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
VARIANTS="sp0 oc6 sp0oc6" CASES="--config entries;--config entries --entry-size 1024;--config entries --entry-size 4096;--config entries --entry-size 100;--config append;--config replay" \
  REPS=3 STEPS=20 TAG=r06/${1:-longknobs2}/ab bash tools/gpu_ab.sh || exit 1
