# Round 6: replay value-sweep lines with the CPU baseline and the object-CRC
# check against the oracle.
set -o pipefail
OUT=gpurun_out/${1:-r06/replaylines}
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in ${VALUES:-64 128 256 512 1024 2048 8192}; do
  timeout -k 10 200 python bench.py --config replay --value-len $v > "$OUT/replay_$v.json" 2> "$OUT/replay_$v.err" || exit 1
done
