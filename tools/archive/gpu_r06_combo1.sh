# Round 6, one call: the walk variants' GPU tests, the replay A/B of the
# k_walk_copyv CRC forms and the dense part shift, and the binning A/B.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/combo1
mkdir -p $O
CHECK="vcrc1 vcrc2 dense15a" bash -c 'for v in $CHECK; do
  RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
      --timeout-method thread tests/test_gpu_segments.py tests/test_gpu_replay_fused.py tests/test_gpu_segment_ref.py \
      -m gpu > '$O'/pytest_$v.log 2>&1 || exit 1; done' || exit 1
VARIANTS="vcrc1 vcrc2 vcrc2r8 vrep8 dense15 dense15a sada" CASES="--config replay --value-len 64;--config replay --value-len 128" \
  REPS=2 STEPS=10 TAG=r06/combo1/walkab bash tools/gpu_ab.sh || exit 1
VARIANTS="bo0 spec0 sp0" CASES="--config entries --entry-size 100;--config entries;--config entries --entry-size 1024;--config entries --contexts 2;--config entries --contexts 8" \
  REPS=2 TAG=r06/combo1/binab bash tools/gpu_ab.sh || exit 1
