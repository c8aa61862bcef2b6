# Entries path after a kernel change: GPU parity tests, then the per-size and
# Zipf-mix benches (each step under its own limit; the first failure ends it).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ec}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for s in 1024 4096 0; do
  timeout -k 10 120 python bench.py --config entries --entry-size $s --steps 10 --warmup 2 > $O/size_$s.json 2> $O/size_$s.err || exit 1
done
timeout -k 10 200 python bench.py --config replay --steps 10 --warmup 2 --no-cpu-baseline > $O/replay.json 2> $O/replay.err || exit 1
timeout -k 10 200 python bench.py --config append --steps 10 --warmup 2 > $O/append.json 2> $O/append.err || exit 1
