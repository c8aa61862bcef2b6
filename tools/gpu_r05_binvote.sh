# Round 5: k_bin_one vote/abort + guarded scatter -- binning tests, then the
# cost of the guarded scatter (base vs rs0 = no guard, bo0 = two launches).
set -o pipefail
O=gpurun_out/r05/binvote
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
    tests/test_gpu_binning.py > $O/pytest_binning.log 2>&1 || { tail -30 $O/pytest_binning.log; exit 1; }
tail -3 $O/pytest_binning.log
grep -h "rescues" $O/pytest_binning.log
VARIANTS="rs0 bo0" CASES="--config entries;--config entries --entry-size 100;--config append" \
    REPS=3 STEPS=20 TAG=r05/binvote/ab bash tools/gpu_ab.sh || exit 1
python tools/ab_summary.py gpurun_out/r05/binvote/ab 2>&1 | tail -20
