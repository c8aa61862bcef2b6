# Long phase work split: parity on the working tree, A/B of the split modes
# against HEAD, phase stamps of the static and the stealing split.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-long4}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_binning.py tests/test_gpu_write_path.py tests/test_gpu_segments.py \
    > $O/pytest.log 2>&1 || exit 1
for v in ${STAMPS:-stamps_st0 stamps}; do
  for s in 0 1024 4096; do
    RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_$v.so timeout -k 10 120 python tools/stamps.py --entry-size $s >> $O/$v.txt 2>&1 || exit 1
  done
done
VARIANTS="${VARIANTS:-head st0 st2h}" CASES="${CASES:---config entries;--config entries --entry-size 1024;--config entries --entry-size 4096;--config replay}" \
    REPS=${REPS:-3} TAG=${TAG:-long4}/ab bash tools/gpu_ab.sh || exit 1
