# Round 6: the walk's pool block map reset per call (the repeated-call fix):
# walk / replay / certify tests incl. the repeated-call regression test, then
# the replay half of the final lines, then the part-size A/B (p17 = the probe
# may pick 128 KiB parts) at 2 and 3 KiB values.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/${1:-final2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_replay_fused.py tests/test_gpu_segments.py tests/test_gpu_segment_ref.py tests/test_gpu_certify.py \
    -m gpu > $O/pytest_walk.log 2>&1 || exit 1
PART=b bash tools/final_lines.sh r06/${1:-final2} || exit 1
VARIANTS="p17" CASES="--config replay --value-len 2048;--config replay --value-len 3072;--config replay --value-len 1536" \
  REPS=2 STEPS=10 TAG=r06/${1:-final2}/ab_p17 bash tools/gpu_ab.sh || exit 1
