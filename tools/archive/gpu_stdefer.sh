# Stored-checksum loads joined at use (records mode): segment/replay parity,
# then a replay A/B against HEAD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-stdefer}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_segments.py tests/test_gpu_parity.py tests/test_gpu_write_path.py tests/test_gpu_recovery.py > $O/pytest.log 2>&1 || exit 1
VARIANTS="head" CASES="--config replay;--config replay --value-len 300;--config replay --value-len 64;--config entries" REPS=3 TAG=${TAG:-stdefer}/ab bash tools/gpu_ab.sh
