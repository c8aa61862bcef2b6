# Round 6, one call: the whole GPU suite on the two-launch binning default,
# and the replay A/B of the tree-shaped VALU CRC forms.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/combo2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || exit 1
for v in vcrc1 vcrc2; do
  RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
      --timeout-method thread tests/test_gpu_replay_fused.py -m gpu > $O/pytest_$v.log 2>&1 || exit 1
done
VARIANTS="vcrc1 vcrc2 sada" CASES="--config replay --value-len 64;--config replay --value-len 128" \
  REPS=2 STEPS=10 TAG=r06/combo2/walkab bash tools/gpu_ab.sh || exit 1
