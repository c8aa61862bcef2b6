# Final-tree profiles: rocprofv3 kernel trace + stats and a FETCH_SIZE pass for
# each bench line whose roofline.traffic is read from profiles/pmc (config 2,
# config 4 at N=1, config 3 mix and 100 B), plus a kernel trace of the replay
# bench.  One pass per run, each under its own time limit.
#   TAG=r02final bash tools/gpu_profile_final.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02final}
mkdir -p $O
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n -o bench \
      -- python3 bench.py "$@" --no-cpu-baseline > $O/trace_$n.json 2> $O/trace_$n.err || exit 1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$n -o pmc \
      -- python3 bench.py "$@" --no-cpu-baseline > $O/pmc_$n.json 2> $O/pmc_$n.err || exit 1
}
run c2 --steps 20 --warmup 3
run c4 --config recovery --steps 10 --warmup 2
run c3 --config entries --steps 10 --warmup 2
run c3_100 --config entries --entry-size 100 --steps 10 --warmup 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_replay -o bench \
    -- python3 bench.py --config replay --steps 10 --warmup 2 --no-cpu-baseline > $O/trace_replay.json 2> $O/trace_replay.err || exit 1
