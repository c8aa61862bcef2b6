# Round 5: long phase = static age-weighted shares for the first DYN_STATIC %
# of each workgroup's range, then deque claims and steals (base 75 %; ds50,
# ds90; ld0 = fully static), bin lookups cached per bin.
set -o pipefail
O=gpurun_out/r05/deque2
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_binning.py tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_write_path.py \
    tests/test_gpu_replay_fused.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_stamps.so timeout -k 10 200 python tools/stamps.py --save $O/mix.npy > $O/stamps_mix.txt 2>&1 || exit 1
VARIANTS="ld0 ds50 ds90" CASES="--config entries;--config entries --entry-size 1024;--config entries --entry-size 4096;--config append;--config replay" \
    REPS=2 STEPS=20 TAG=r05/deque2/ab bash tools/gpu_ab.sh || exit 1
head -22 $O/stamps_mix.txt
python tools/ab_summary.py gpurun_out/r05/deque2/ab
