# Round 4: multi-window tiny phase (bins 2..kTinyK): full GPU suite, then
# entries / replay lines at the sizes it serves.
set -o pipefail
OUT=gpurun_out/${1:-r04/tinyk}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1 || exit 1
for sz in 100 160 300 500 1024; do
  timeout -k 10 200 python bench.py --config entries --entry-size $sz --no-cpu-baseline > "$OUT/c3_$sz.json" 2> "$OUT/c3_$sz.err" || exit 1
done
timeout -k 10 200 python bench.py --config entries --no-cpu-baseline > "$OUT/c3_mix.json" 2> "$OUT/c3_mix.err" || exit 1
for v in 64 128 256 512 1024; do
  timeout -k 10 120 python bench.py --config replay --value-len $v --no-cpu-baseline > "$OUT/replay_$v.json" 2> "$OUT/replay_$v.err" || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o r128 -- python bench.py --config replay --value-len 128 --no-cpu-baseline --steps 10 > "$OUT/prof_r128.json" 2> "$OUT/prof_r128.err" || exit 1
