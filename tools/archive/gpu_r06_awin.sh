# Round 6: A with staged windows (awin, k_walk_partsw) against A: walk / replay
# tests and a 64 B trace under awin, replay A/B.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/${1:-awin}
mkdir -p $O
RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_awin.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_replay_fused.py tests/test_gpu_segments.py tests/test_gpu_segment_ref.py tests/test_gpu_certify.py \
    -m gpu > $O/pytest.log 2>&1 || exit 1
VARIANTS="awin" CASES="--config replay --value-len 64;--config replay --value-len 128;--config replay --value-len 100" \
  REPS=2 STEPS=10 TAG=r06/${1:-awin}/ab bash tools/gpu_ab.sh || exit 1
RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_awin.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r64 -- \
    python3 bench.py --config replay --value-len 64 --steps 10 --no-cpu-baseline > $O/prof64.json 2>> $O/err.txt || exit 1
