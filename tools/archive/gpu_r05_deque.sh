# Round 5: long phase as per-workgroup deques with stealing (vs ld0 static),
# the guarded scatter's grid cap (vs rw0 = a workgroup per tile), and a trace
# of the fused replay at 64-byte values.
set -o pipefail
O=gpurun_out/r05/deque
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_binning.py tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_write_path.py \
    tests/test_gpu_replay_fused.py tests/test_gpu_segment_ref.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_stamps.so timeout -k 10 200 python tools/stamps.py --save $O/mix.npy > $O/stamps_mix.txt 2>&1 || exit 1
VARIANTS="ld0" CASES="--config entries;--config entries --entry-size 1024;--config entries --entry-size 4096;--config append;--config replay" \
    REPS=2 STEPS=20 TAG=r05/deque/ab_long bash tools/gpu_ab.sh || exit 1
VARIANTS="rw0" CASES="--config entries --entry-size 100;--config entries" \
    REPS=2 STEPS=20 TAG=r05/deque/ab_rescue bash tools/gpu_ab.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o replay64 -- \
    python3 bench.py --config replay --value-len 64 --steps 10 --no-cpu-baseline > $O/replay64.json 2> $O/replay64.err || exit 1
cat $O/stamps_mix.txt | head -20
python tools/ab_summary.py gpurun_out/r05/deque/ab_long
python tools/ab_summary.py gpurun_out/r05/deque/ab_rescue
