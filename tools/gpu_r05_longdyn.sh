# Round 5: dynamic long-phase octet claims -- parity first, then A/B against
# static shares (ld0) and the phase stamps of the new order.
set -o pipefail
O=gpurun_out/r05/longdyn
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_binning.py tests/test_gpu_segments.py tests/test_gpu_write_path.py tests/test_gpu_replay_fused.py tests/test_gpu_segment_ref.py \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=ramcloud_amd/lib/variants/libramcrc_stamps.so
RAMCRC_LIB=$L timeout -k 10 200 python tools/stamps.py --save $O/mix.npy > $O/stamps_mix.txt 2>&1 || exit 1
cat $O/stamps_mix.txt
VARIANTS="ld0 tg0 hm0" CASES="--config entries;--config entries --entry-size 100;--config entries --entry-size 1024;--config entries --entry-size 4096;--config append;--config replay;--config replay --value-len 64" \
    REPS=3 STEPS=20 TAG=r05/longdyn/ab bash tools/gpu_ab.sh || exit 1
python tools/ab_summary.py gpurun_out/r05/longdyn/ab
