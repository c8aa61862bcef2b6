# Round 6: same-box A/B of the small-entry binning choices -- one-launch
# k_bin_one (base) vs the two-launch count + scatter (bo0), the speculative
# tiny pass off (spec0), the role split off (sp0) -- on the config-3 sizes and
# the concurrency shape.  Variants: python -m ramcloud_amd.build --variants bo0 spec0 sp0
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
VARIANTS="${VARIANTS:-bo0 spec0 sp0}" \
CASES="${CASES:---config entries --entry-size 100;--config entries;--config entries --entry-size 1024;--config entries --entry-size 4096;--config append;--config entries --contexts 2;--config entries --contexts 8}" \
REPS=${REPS:-3} TAG=${1:-r06/binab} bash tools/gpu_ab.sh
