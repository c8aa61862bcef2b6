# Round 5: k_entries role split (tiny and long phases on separate workgroups)
# vs sp0 (phases in sequence), and the tiny window weight kappa (128/256/512).
set -o pipefail
O=gpurun_out/r05/split
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_binning.py tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_write_path.py \
    tests/test_gpu_replay_fused.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VARIANTS="sp0 kap192 kap320" CASES="--config entries;--config append;--config entries --entry-size 1024;--config entries --entry-size 4096" \
    REPS=3 STEPS=20 TAG=r05/split/ab2 bash tools/gpu_ab.sh || exit 1
python tools/ab_summary.py gpurun_out/r05/split/ab2
