# Round 6, one call: walk/replay tests on the tree, replay A/B of the
# adaptive sync stage (sada0 = always 7 KiB) over the value sweep, a trace
# of the 64 B replay.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/combo3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_replay_fused.py \
    tests/test_gpu_segments.py tests/test_gpu_segment_ref.py tests/test_gpu_certify.py -m gpu > $O/pytest.log 2>&1 || exit 1
VARIANTS="sada0" CASES="--config replay --value-len 64;--config replay --value-len 128;--config replay --value-len 256;--config replay --value-len 512;--config replay --value-len 1024" \
  REPS=3 STEPS=10 TAG=r06/combo3/ab bash tools/gpu_ab.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r64 -- \
    python3 bench.py --config replay --value-len 64 --steps 10 --no-cpu-baseline > $O/prof64.json 2>> $O/err.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r128 -- \
    python3 bench.py --config replay --value-len 128 --steps 10 --no-cpu-baseline > $O/prof128.json 2>> $O/err.txt || exit 1
