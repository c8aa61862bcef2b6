# Round 4: count-pass loads in flight on replay batches (40M / 4M records):
# A/B of the default build against variants, replay 64 B and 1 KiB, with traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04/bincount}
mkdir -p "$OUT"
RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_cpf1.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_segments.py tests/test_gpu_recovery.py > "$OUT/pytest_cpf1.log" 2>&1 || exit 1
for rep in 1 2; do
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  for vl in 64 1024; do
    RAMCRC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${v}_${vl}_$rep" -o t -- python3 bench.py --config replay --value-len $vl --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/${v}_${vl}_$rep.json" 2> "$OUT/${v}_${vl}_$rep.err" || exit 1
    find "$OUT/${v}_${vl}_$rep" -type f ! -name '*kernel_stats.csv' -delete
  done
done
done
