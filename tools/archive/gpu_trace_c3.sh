# Kernel trace + stats of the config-3 benches (mix and 1M x 100 B) on the
# default build.   TAG=x bash tools/gpu_trace_c3.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tracec3}
mkdir -p $O
for sz in 0 100; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$sz -o t \
      -- python3 bench.py --config entries --entry-size $sz --steps 10 --warmup 2 --no-cpu-baseline > $O/trace_$sz.json 2> $O/trace_$sz.err || exit 1
done
