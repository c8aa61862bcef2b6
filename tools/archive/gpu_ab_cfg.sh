# A/B of library builds over several bench configurations, alternating builds
# (3 reps).  Each CONFIGS item is "name:bench args" with '+' for spaces.
#   TAG=x VARIANTS="evrec" CONFIGS="c2:--steps+20 c3:--config+entries" bash tools/gpu_ab_cfg.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abcfg}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
fi
for rep in 1 2 3; do
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  for c in $CONFIGS; do
    n=${c%%:*}; a=${c#*:}; a=${a//+/ }
    RAMCRC_LIB=$L timeout -k 10 150 python bench.py $a --no-cpu-baseline >> $O/${v}_$n.jsonl 2>> $O/$v.err || exit 1
  done
done
done
