# Round 4: larger walk parts (2^19, 2^20) for 2 .. 8 KiB values.
set -o pipefail
OUT=gpurun_out/${1:-r04/parts2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 2048 4096 8192; do
  for ps in 18 19 20; do
    timeout -k 10 120 python bench.py --config replay --value-len $v --walk-part-shift $ps --no-cpu-baseline --steps 10 --warmup 2 > "$OUT/replay_${v}_ps${ps}.json" 2> "$OUT/replay_${v}_ps${ps}.err" || exit 1
  done
done
