# Round 6: the part walk's read-ahead (a per-lane register buffer of 8 / 16 /
# 32 16-byte units, RAMCRC_PEEK_UNITS; removed after this A/B, 15-40 % slower):
# walk / replay / certify tests, replay A/B against off (pk0), a 64 B trace.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/${1:-peek}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_replay_fused.py tests/test_gpu_segments.py tests/test_gpu_segment_ref.py tests/test_gpu_certify.py \
    -m gpu > $O/pytest.log 2>&1 || exit 1
VARIANTS="pk0 pk8" CASES="--config replay --value-len 64;--config replay --value-len 128;--config replay --value-len 256;--config replay --value-len 1024" \
  REPS=2 STEPS=10 TAG=r06/${1:-peek}/ab bash tools/gpu_ab.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r64 -- \
    python3 bench.py --config replay --value-len 64 --steps 10 --no-cpu-baseline > $O/prof64.json 2>> $O/err.txt || exit 1
