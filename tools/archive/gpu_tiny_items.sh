# Tiny-round-aware workgroup shares: parity of the small-entry kernels,
# stamps with and without, A/B of kTinyItems.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ti}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_binning.py tests/test_gpu_write_path.py tests/test_gpu_segments.py \
    > $O/pytest.log 2>&1 || exit 1
for v in stamps_ti0 stamps; do
  RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_$v.so timeout -k 10 120 python tools/stamps.py >> $O/$v.txt 2>&1 || exit 1
done
VARIANTS="head ti0 te0" CASES="--config entries;--config replay;--config entries --entry-size 100" REPS=3 TAG=${TAG:-ti}/ab bash tools/gpu_ab.sh || exit 1
