# Walk A's speculative prefetch: segment parity, then a replay A/B against
# the build without it, with kernel traces of both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-spec}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_segments.py tests/test_gpu_certify.py tests/test_gpu_recovery.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_spec -o run -- python3 bench.py --config replay --steps 5 --warmup 2 --no-cpu-baseline > $O/tr_spec.log 2>&1 || exit 1
RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_nospec.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_nospec -o run -- python3 bench.py --config replay --steps 5 --warmup 2 --no-cpu-baseline > $O/tr_nospec.log 2>&1 || exit 1
VARIANTS="nospec" CASES="--config replay;--config replay --value-len 64;--config replay --value-len 8192" REPS=3 TAG=${TAG:-spec}/ab bash tools/gpu_ab.sh
