# Round 4: binning of replay batches (40M / 4M / 0.5M records): the whole GPU
# suite, then an A/B of the default build against variants on replay 64 B,
# 1 KiB and 8 KiB values, with kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04/bincount}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1 || exit 1
for rep in 1 2; do
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  for vl in 64 1024 8192; do
    RAMCRC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${v}_${vl}_$rep" -o t -- python3 bench.py --config replay --value-len $vl --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/${v}_${vl}_$rep.json" 2> "$OUT/${v}_${vl}_$rep.err" || exit 1
    find "$OUT/${v}_${vl}_$rep" -type f ! -name '*kernel_stats.csv' -delete
  done
done
done
