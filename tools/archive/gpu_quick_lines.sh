# Quick bench lines (no profiler): config 2, config 3 mix and 100 B, replay.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-quick}
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 300 python bench.py --config entries --steps 10 --warmup 2 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 300 python bench.py --config entries --entry-size 100 --steps 10 --warmup 2 --no-cpu-baseline > $O/c3_100.json 2> $O/c3_100.err || exit 1
timeout -k 10 300 python bench.py --config replay --steps 10 --warmup 2 --no-cpu-baseline > $O/replay.json 2> $O/replay.err || exit 1
