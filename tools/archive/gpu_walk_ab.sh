# Segment-walk parity (default library) and a replay A/B of the working tree
# against HEAD (tools/build_rev.sh HEAD head) with kernel traces.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-walk1}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_segments.py tests/test_gpu_certify.py tests/test_gpu_recovery.py > $O/pytest.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/tr_new -o run -- python3 bench.py --config replay --value-len 64 --steps 5 --warmup 2 --no-cpu-baseline > $O/tr_new.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/tr_new1k -o run -- python3 bench.py --config replay --steps 5 --warmup 2 --no-cpu-baseline > $O/tr_new1k.log 2>&1 &&
VARIANTS="${VARIANTS:-head}" CASES="--config replay;--config replay --value-len 64" REPS=3 TAG=${TAG:-walk1}/ab bash tools/gpu_ab.sh
