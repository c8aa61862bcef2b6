# Tiny rounds to the oldest waves first: small-entry parity, stamps with and
# without, A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tage}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_binning.py tests/test_gpu_write_path.py tests/test_gpu_segments.py \
    > $O/pytest.log 2>&1 || exit 1
for v in stamps_tage0 stamps; do
  for s in 100 0; do
    RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_$v.so timeout -k 10 120 python tools/stamps.py --entry-size $s >> $O/$v.txt 2>&1 || exit 1
  done
done
VARIANTS="tage0" CASES="--config entries --entry-size 100;--config entries;--config replay --value-len 64" REPS=3 TAG=${TAG:-tage}/ab bash tools/gpu_ab.sh
