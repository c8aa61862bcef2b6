# New-feature GPU pass: write-path + segment parity tests, the replay and
# append configs, and a kernel trace of the replay config (walk vs verify).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${ROUND:-r01}/replay
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config replay --steps 10 --warmup 2 > $O/replay.json 2> $O/replay.err || exit 1
timeout -k 10 300 python bench.py --config replay --value-len 64 --replay-nseg 256 --steps 5 --warmup 1 --no-cpu-baseline > $O/replay64.json 2> $O/replay64.err || exit 1
timeout -k 10 300 python bench.py --config append --steps 10 --warmup 2 > $O/append.json 2> $O/append.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o replay \
    -- python3 bench.py --config replay --steps 5 --warmup 1 --no-cpu-baseline > $O/trace_replay.json 2> $O/trace.err || exit 1
