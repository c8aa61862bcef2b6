# Long-phase changes: parity of the small-entry kernels on the working tree,
# then an interleaved A/B against HEAD (tools/build_rev.sh HEAD head).
#   TAG=r03/long1 bash tools/gpu_long_ab.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-long1}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_binning.py tests/test_gpu_write_path.py tests/test_gpu_segments.py \
    > $O/pytest.log 2>&1 || exit 1
VARIANTS="${VARIANTS:-head}" CASES="${CASES:---config entries;--config entries --entry-size 1024;--config entries --entry-size 4096;--config replay;--config entries --entry-size 100}" \
    REPS=${REPS:-3} TAG=${TAG:-long1}/ab bash tools/gpu_ab.sh
