# Round 4: GPU suite, then the RecoverSegmentBenchmark value sweep (replay),
# the entries lines and one replay trace per end of the sweep.
set -o pipefail
OUT=gpurun_out/${1:-r04/replay}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1 || exit 1
for v in 64 128 256 512 1024 2048 8192; do
  timeout -k 10 120 python bench.py --config replay --value-len $v --no-cpu-baseline > "$OUT/replay_$v.json" 2> "$OUT/replay_$v.err" || exit 1
done
for sz in 0 100 160 1024; do
  timeout -k 10 200 python bench.py --config entries --entry-size $sz --no-cpu-baseline > "$OUT/c3_$sz.json" 2> "$OUT/c3_$sz.err" || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o r64 -- python bench.py --config replay --value-len 64 --no-cpu-baseline --steps 10 > "$OUT/prof_r64.json" 2> "$OUT/prof_r64.err" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o r1024 -- python bench.py --config replay --value-len 1024 --no-cpu-baseline --steps 10 > "$OUT/prof_r1024.json" 2> "$OUT/prof_r1024.err" || exit 1
