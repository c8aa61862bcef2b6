# Round 4: replay across the RecoverSegmentBenchmark value sweep, walk part
# size forced to 2^15 .. 2^18, plus kernel traces at 8 KiB values.
set -o pipefail
OUT=gpurun_out/${1:-r04/parts}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 64 128 256 512 1024 2048 4096 8192; do
  for ps in 15 16 17 18; do
    if [ $v -le 256 ] && [ $ps -eq 18 ]; then continue; fi
    if [ $v -ge 2048 ] && [ $ps -eq 15 ]; then continue; fi
    timeout -k 10 120 python bench.py --config replay --value-len $v --walk-part-shift $ps --no-cpu-baseline --steps 10 --warmup 2 > "$OUT/replay_${v}_ps${ps}.json" 2> "$OUT/replay_${v}_ps${ps}.err" || exit 1
    echo "$v $ps $(tail -c 300 $OUT/replay_${v}_ps${ps}.json | grep -o '"ms_per_step": [0-9.]*')"
  done
done
for ps in 16 17 18; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o r8192_ps$ps -- python bench.py --config replay --value-len 8192 --walk-part-shift $ps --no-cpu-baseline --steps 10 > "$OUT/prof_8192_ps$ps.json" 2> "$OUT/prof_8192_ps$ps.err" || exit 1
done
