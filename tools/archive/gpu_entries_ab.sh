# A/B of libramcrc variants on the entries path: kernel trace of the entries
# bench at SIZES (0 = the config-3 mix) per variant, then (PARITY=v) the GPU
# entries parity tests against that variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-entab}
mkdir -p $O
if [ -n "$PARITY" ]; then
  RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_$PARITY.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "entr or batch or tiny" --timeout 240 --timeout-method thread > $O/parity_$PARITY.log 2>&1 || exit 1
fi
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  for sz in $SIZES; do
  for n in ${ENTRIES:-1000000}; do
    RAMCRC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_${sz}_$n -o t -- python3 bench.py --config entries --entries $n --entry-size $sz --steps 10 --warmup 2 --no-cpu-baseline > $O/${v}_${sz}_$n.json 2> $O/${v}_${sz}_$n.err || exit 1
  done
  done
done
