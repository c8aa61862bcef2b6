# Round 5: dynamic long-phase octet claims, generated tiny tables, DPP group
# XOR, fused replay -- parity first, then same-box A/B (ld0 = static shares,
# tg0 = copied tiny table, hm0 = ds_swizzle group XOR) and the phase stamps.
set -o pipefail
O=gpurun_out/r05/longdyn
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_binning.py tests/test_gpu_segments.py tests/test_gpu_write_path.py \
    tests/test_gpu_replay_fused.py tests/test_gpu_segment_ref.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=ramcloud_amd/lib/variants/libramcrc_stamps.so
RAMCRC_LIB=$L timeout -k 10 200 python tools/stamps.py --save $O/mix.npy > $O/stamps_mix.txt 2>&1 || exit 1
cat $O/stamps_mix.txt
VARIANTS="ld0" CASES="--config entries;--config entries --entry-size 1024;--config entries --entry-size 4096;--config append;--config replay" \
    REPS=2 STEPS=20 TAG=r05/longdyn/ab_long bash tools/gpu_ab.sh || exit 1
python tools/ab_summary.py gpurun_out/r05/longdyn/ab_long
VARIANTS="tg0 hm0" CASES="--config entries;--config entries --entry-size 100;--config replay --value-len 64" \
    REPS=2 STEPS=20 TAG=r05/longdyn/ab_tiny bash tools/gpu_ab.sh || exit 1
python tools/ab_summary.py gpurun_out/r05/longdyn/ab_tiny
VARIANTS="wp0" CASES="--config replay --value-len 64;--config replay;--config replay --value-len 8192" \
    REPS=2 STEPS=10 TAG=r05/longdyn/ab_walk bash tools/gpu_ab.sh || exit 1
python tools/ab_summary.py gpurun_out/r05/longdyn/ab_walk
