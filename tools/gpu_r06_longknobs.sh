# Round 6: the long phase's scheduling knobs re-checked on the final tree for
# the config-3 mix and 1M x 1 KiB: role split off (sp0),
# age skew 0 / 60 (default 140), octet cost 2 / 6 (default 4), kappa 192
# (default 256).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
VARIANTS="sp0 sk0 sk60 oc2 oc6 kap192" CASES="--config entries;--config entries --entry-size 1024" \
  REPS=3 STEPS=20 TAG=r06/${1:-longknobs}/ab bash tools/gpu_ab.sh || exit 1
