# Round 5: the replay summary read once per wave in k_walk_copy (no 32K
# same-address atomics): GPU replay/segment tests, then the replay traces.
set -o pipefail
OUT=gpurun_out/r05/${TAG:-replayfix}
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_segments.py tests/test_gpu_replay_fused.py tests/test_gpu_segment_ref.py tests/test_gpu_certify.py \
    > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
P="rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof"
timeout -k 10 300 $P -o replay -- python3 bench.py --config replay --steps 10 --no-cpu-baseline > $OUT/prof_replay.json 2> $OUT/prof_replay.err || exit 1
timeout -k 10 300 $P -o replay64 -- python3 bench.py --config replay --value-len 64 --steps 10 --no-cpu-baseline > $OUT/prof_replay64.json 2> $OUT/prof_replay64.err || exit 1
for v in 64 1024 8192; do
  timeout -k 10 200 python3 bench.py --config replay --value-len $v --steps 10 --no-cpu-baseline > $OUT/replay_$v.json 2> $OUT/replay_$v.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$OUT/replay_$v.json')); print($v, d['value'], d['ms_per_step'])"
done
