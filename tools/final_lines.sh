# The round's final tree on one GPU: the GPU suite, smoke, every bench line
# DESIGN.md quotes (sections 5-7) and the rocprofv3 kernel traces its kernel
# times come from.  Every step under its own time limit.  In two calls when
# one would pass gpurun's limit: PART=a (suite, smoke, segments, entries,
# append, stream), PART=b (replay sweep, contexts, traces); default both.
#     PART=a bash tools/final_lines.sh [OUT]      (default gpurun_out/final)
set -o pipefail
OUT=gpurun_out/${1:-final}
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
PART=${PART:-ab}
if [[ $PART == *a* ]]; then
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
timeout -k 10 300 python bench.py --config recovery > "$OUT/recovery.json" 2> "$OUT/recovery.err" || exit 1
for sz in 0 100 1024 4096; do
  timeout -k 10 200 python bench.py --config entries --entry-size $sz > "$OUT/c3_$sz.json" 2> "$OUT/c3_$sz.err" || exit 1
done
timeout -k 10 200 python bench.py --config append > "$OUT/append.json" 2> "$OUT/append.err" || exit 1
timeout -k 10 300 python bench.py --config stream > "$OUT/stream.json" 2> "$OUT/stream.err" || exit 1
fi
if [[ $PART == *b* ]]; then
for v in 64 128 256 512 1024 2048 3072 4096 8192; do
  timeout -k 10 200 python bench.py --config replay --value-len $v > "$OUT/replay_$v.json" 2> "$OUT/replay_$v.err" || exit 1
done
timeout -k 10 200 python bench.py --config replay > "$OUT/replay.json" 2> "$OUT/replay.err" || exit 1
# the reference's concurrency shape (RecoverSegmentBenchmark's replay threads)
for K in ${KS:-1 4 16}; do
  timeout -k 10 300 python bench.py --config entries --contexts $K > "$OUT/ctx_entries_k$K.json" 2> "$OUT/ctx_entries_k$K.err" || exit 1
  timeout -k 10 300 python bench.py --config replay --value-len 64 --contexts $K --steps 10 > "$OUT/ctx_replay64_k$K.json" 2> "$OUT/ctx_replay64_k$K.err" || exit 1
done
P="rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof"
timeout -k 10 200 $P -o c2 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/prof_c2.json" 2> "$OUT/prof_c2.err" || exit 1
timeout -k 10 200 $P -o c3 -- python3 bench.py --config entries --steps 20 --no-cpu-baseline > "$OUT/prof_c3.json" 2> "$OUT/prof_c3.err" || exit 1
timeout -k 10 200 $P -o c3_100 -- python3 bench.py --config entries --entry-size 100 --steps 20 --no-cpu-baseline > "$OUT/prof_c3_100.json" 2> "$OUT/prof_c3_100.err" || exit 1
timeout -k 10 200 $P -o append -- python3 bench.py --config append --steps 20 --no-cpu-baseline > "$OUT/prof_append.json" 2> "$OUT/prof_append.err" || exit 1
timeout -k 10 300 $P -o replay -- python3 bench.py --config replay --steps 10 --no-cpu-baseline > "$OUT/prof_replay.json" 2> "$OUT/prof_replay.err" || exit 1
timeout -k 10 300 $P -o replay64 -- python3 bench.py --config replay --value-len 64 --steps 10 --no-cpu-baseline > "$OUT/prof_replay64.json" 2> "$OUT/prof_replay64.err" || exit 1
timeout -k 10 300 $P -o replay128 -- python3 bench.py --config replay --value-len 128 --steps 10 --no-cpu-baseline > "$OUT/prof_replay128.json" 2> "$OUT/prof_replay128.err" || exit 1
fi
python tools/lines_summary.py "$OUT"/*.json > "$OUT/lines.txt" 2>&1
