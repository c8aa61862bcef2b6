# rocprofv3 kernel-trace/stats and FETCH_SIZE passes for the bench lines
# (config 2 default, config 4 at N=1, config 3).  One pass per run; every run
# under its own time limit; the first failure ends the script.
#   TAG=r02c bash tools/gpu_profile_r02.sh   -> gpurun_out/$TAG/{trace,pmc}_{c2,c4,c3}
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02c}
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
