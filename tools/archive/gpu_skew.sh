# Age skew per mode: small-entry parity, then the A/B against skew 80 everywhere.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-skew}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_binning.py tests/test_gpu_write_path.py tests/test_gpu_segments.py \
    > $O/pytest.log 2>&1 || exit 1
VARIANTS="sk80" CASES="--config entries;--config entries --entry-size 1024;--config entries --entry-size 4096;--config replay" REPS=3 TAG=${TAG:-skew}/ab bash tools/gpu_ab.sh
