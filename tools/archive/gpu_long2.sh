# Long phase v2: parity of the small-entry kernels on the working tree, the
# A/B against HEAD, then k_entries phase stamps (probe build).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-long2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_binning.py tests/test_gpu_write_path.py tests/test_gpu_segments.py \
    > $O/pytest.log 2>&1 || exit 1
VARIANTS="${VARIANTS:-head}" CASES="${CASES:---config entries;--config entries --entry-size 1024;--config entries --entry-size 4096;--config replay;--config entries --entry-size 100}" \
    REPS=${REPS:-3} TAG=${TAG:-long2}/ab bash tools/gpu_ab.sh || exit 1
for s in 0 1024 4096 100; do
  RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_stamps.so timeout -k 10 120 python tools/stamps.py --entry-size $s >> $O/stamps.txt 2>&1 || exit 1
done
