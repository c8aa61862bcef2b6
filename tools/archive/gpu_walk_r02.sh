# Parallel segment walk: GPU walk/verify parity tests, then the replay bench
# with the parallel and the serial walker, and a kernel trace of the former.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-walk1}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_recovery.py -x -v --timeout 300 --timeout-method thread > $O/pytest_seg.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config replay --steps 6 --warmup 2 --no-cpu-baseline > $O/replay_par.json 2> $O/replay_par.err || exit 1
timeout -k 10 300 python bench.py --config replay --serial-walk --steps 6 --warmup 2 --no-cpu-baseline > $O/replay_ser.json 2> $O/replay_ser.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_replay -o t -- python3 bench.py --config replay --steps 6 --warmup 2 --no-cpu-baseline > $O/trace_replay.json 2> $O/trace_replay.err || exit 1
