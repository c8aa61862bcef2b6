# Round 6: the replay walk variants -- dense batches in 32 KiB parts with
# 32-record LDS runs (dense15), the LDS runs alone (lrec32), verify-in-walk off
# (vf0) -- checked by the walk / replay GPU tests under each, then timed
# against the product library on the RecoverSegmentBenchmark value sweep.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r06/walkab}
mkdir -p $O
for v in ${CHECK:-dense15}; do
  RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
      --timeout-method thread tests/test_gpu_segments.py tests/test_gpu_replay_fused.py tests/test_gpu_segment_ref.py \
      -m gpu > $O/pytest_$v.log 2>&1 || exit 1
done
VARIANTS="${VARIANTS:-dense15 lrec32 vf0}" \
CASES="${CASES:---config replay --value-len 64;--config replay --value-len 128;--config replay --value-len 1024;--config replay --value-len 8192}" \
REPS=${REPS:-2} STEPS=10 TAG=${1:-r06/walkab}/ab bash tools/gpu_ab.sh
