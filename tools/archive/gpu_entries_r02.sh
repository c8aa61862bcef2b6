# Entries path: parity tests, then per-size and mix benches with a kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ent}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_write_path.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for sz in 0 100 1024 4096; do
  timeout -k 10 300 python bench.py --config entries --entry-size $sz --steps 10 --warmup 2 --no-cpu-baseline > $O/e$sz.json 2> $O/e$sz.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 bench.py --config entries --steps 10 --warmup 2 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || exit 1
