# Round 3: bench lines of every config on this tree (CPU baselines on the
# reference's intelCrc32C, T threads), then rocprofv3 kernel traces of the
# config-3 mix, 100 B entries, config 4 at N=1 and replay.  Each step has its
# own time limit; the first failure ends the script.
#   TAG=r03lines bash tools/gpu_r03_lines.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03lines}
mkdir -p $O
line() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit 1
}
trace() {
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n -o bench \
      -- python3 bench.py "$@" --no-cpu-baseline > $O/trace_$n.json 2> $O/trace_$n.err || exit 1
}
line entries --config entries --steps 10 --warmup 2
line entries100 --config entries --entry-size 100 --steps 10 --warmup 2
line recovery --config recovery --steps 10 --warmup 2
line replay --config replay --steps 10 --warmup 2
line append --config append --steps 10 --warmup 2
trace c3 --config entries --steps 10 --warmup 2
trace c3_100 --config entries --entry-size 100 --steps 10 --warmup 2
trace c4 --config recovery --steps 10 --warmup 2
trace replay --config replay --steps 10 --warmup 2
