# Round 6, one call: binning/parity tests (the two-window table direct path),
# the nibble-table variant's replay tests, and A/Bs: nibble tables (vnib) on
# replay 64 / 128 B, the direct multi-window path (dm0 = off) on 160 / 200 B
# table batches.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/combo4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binning.py \
    tests/test_gpu_parity.py -m gpu > $O/pytest.log 2>&1 || exit 1
RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_vnib.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_replay_fused.py -m gpu > $O/pytest_vnib.log 2>&1 || exit 1
VARIANTS="vnib" CASES="--config replay --value-len 64;--config replay --value-len 128" \
  REPS=3 STEPS=10 TAG=r06/combo4/ab_vnib bash tools/gpu_ab.sh || exit 1
VARIANTS="dm0" CASES="--config entries --entry-size 160;--config entries --entry-size 200;--config entries" \
  REPS=3 TAG=r06/combo4/ab_dm bash tools/gpu_ab.sh || exit 1
