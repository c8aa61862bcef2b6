# Round 4: the ordered-stream path (RAMCRC_ORDERED; records mode for replay)
# -- parity first, then the lines (ordered and binned) and kernel traces.
set -o pipefail
OUT=gpurun_out/${1:-r04/stream}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ordered.py tests/test_gpu_write_path.py tests/test_gpu_segments.py tests/test_gpu_segment_ref.py tests/test_gpu_certify.py tests/test_gpu_recovery.py > "$OUT/pytest_ordered.log" 2>&1 || exit 1
for cfg in "mix:" "100:--entry-size 100" "1024:--entry-size 1024" "4096:--entry-size 4096"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 200 python bench.py --config entries $a --no-cpu-baseline > "$OUT/c3_${name}_ordered.json" 2> "$OUT/c3_${name}_ordered.err" || exit 1
done
timeout -k 10 200 python bench.py --config entries --order any --no-cpu-baseline > "$OUT/c3_mix_binned.json" 2> "$OUT/c3_mix_binned.err" || exit 1
timeout -k 10 200 python bench.py --config append --no-cpu-baseline > "$OUT/append_ordered.json" 2> "$OUT/append_ordered.err" || exit 1
timeout -k 10 200 python bench.py --config append --order any --no-cpu-baseline > "$OUT/append_binned.json" 2> "$OUT/append_binned.err" || exit 1
for v in 1024 64 8192; do
  timeout -k 10 300 python bench.py --config replay --value-len $v --no-cpu-baseline > "$OUT/replay_$v.json" 2> "$OUT/replay_$v.err" || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c3 -- python bench.py --config entries --no-cpu-baseline --steps 10 > "$OUT/prof_c3.json" 2> "$OUT/prof_c3.err" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c3_100 -- python bench.py --config entries --entry-size 100 --no-cpu-baseline --steps 10 > "$OUT/prof_c3_100.json" 2> "$OUT/prof_c3_100.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o replay -- python bench.py --config replay --no-cpu-baseline --steps 10 > "$OUT/prof_replay.json" 2> "$OUT/prof_replay.err" || exit 1
