# Round 5: kernel trace of the 128 B-value replay (the weakest point of the
# RecoverSegmentBenchmark sweep) and of 1M x 160 B table entries.
set -o pipefail
OUT=gpurun_out/r05/replay128
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof"
timeout -k 10 300 $P -o replay128 -- python3 bench.py --config replay --value-len 128 --steps 10 --no-cpu-baseline > $OUT/replay128.json 2> $OUT/replay128.err || exit 1
timeout -k 10 300 $P -o e160 -- python3 bench.py --config entries --entry-size 160 --steps 20 --no-cpu-baseline > $OUT/e160.json 2> $OUT/e160.err || exit 1
