# Sync stage 7 KiB as the default: walk/replay/certificate parity, then the
# replay A/B against the 9 KiB stage.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-sync7}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_segments.py tests/test_gpu_certify.py tests/test_gpu_recovery.py tests/test_shard.py > $O/pytest.log 2>&1 || exit 1
VARIANTS="ss9" CASES="--config replay;--config replay --value-len 64;--config replay --value-len 8192;--config replay --value-len 300" REPS=3 TAG=${TAG:-sync7}/ab bash tools/gpu_ab.sh
