# Round 4: walk part size chosen per batch (k_walk_probe): parity of the
# walk tests, then the RecoverSegmentBenchmark value sweep and a trace.
set -o pipefail
OUT=gpurun_out/${1:-r04/adapt}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_segments.py tests/test_gpu_segment_ref.py tests/test_gpu_certify.py tests/test_gpu_recovery.py > "$OUT/pytest_walk.log" 2>&1 || exit 1
for v in 64 128 256 512 1024 2048 4096 8192; do
  timeout -k 10 120 python bench.py --config replay --value-len $v --no-cpu-baseline > "$OUT/replay_$v.json" 2> "$OUT/replay_$v.err" || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o replay8192 -- python bench.py --config replay --value-len 8192 --no-cpu-baseline --steps 10 > "$OUT/prof_8192.json" 2> "$OUT/prof_8192.err" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o replay64 -- python bench.py --config replay --value-len 64 --no-cpu-baseline --steps 10 > "$OUT/prof_64.json" 2> "$OUT/prof_64.err" || exit 1
