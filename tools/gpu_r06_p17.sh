# Round 6: the probe no longer picks 128 KiB parts (RAMCRC_SKIP_P17): walk /
# replay / certify tests on the tree, replay A/B against p17 (the old choice)
# at 1 / 2 / 4 KiB values, and the 2 KiB replay line with its CPU baseline.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/${1:-p17}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_replay_fused.py tests/test_gpu_segments.py tests/test_gpu_segment_ref.py tests/test_gpu_certify.py \
    -m gpu > $O/pytest.log 2>&1 || exit 1
VARIANTS="p17" CASES="--config replay --value-len 1024;--config replay --value-len 2048;--config replay --value-len 4096;--config replay --value-len 1536;--config replay --value-len 2560" \
  REPS=2 STEPS=10 TAG=r06/${1:-p17}/ab bash tools/gpu_ab.sh || exit 1
timeout -k 10 200 python bench.py --config replay --value-len 2048 > $O/replay_2048.json 2> $O/replay_2048.err || exit 1
