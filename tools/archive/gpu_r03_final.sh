# Round 3, committed tree: GPU suite, smoke, the default bench line, bench
# lines of every config (reference CPU baselines), rocprofv3 kernel traces
# and FETCH_SIZE passes of the small-entry workloads.  Each step has its own
# time limit; the first failure ends the script.
#   TAG=r03/final1 bash tools/gpu_r03_final.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03final}
mkdir -p $O
python -c "import ramcloud_amd.ramcrc as r; print(r.lib().ramcrc_build_info().decode())" > $O/build_info.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
line() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit 1
}
trace() {
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n -o bench \
      -- python3 bench.py "$@" --no-cpu-baseline > $O/trace_$n.json 2> $O/trace_$n.err || exit 1
}
pmc() {
  local n=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$n -o p \
      -- python3 bench.py "$@" --no-cpu-baseline > $O/pmc_$n.json 2> $O/pmc_$n.err || exit 1
}
line entries --config entries --steps 10 --warmup 2
line entries100 --config entries --entry-size 100 --steps 10 --warmup 2
line entries1k --config entries --entry-size 1024 --steps 10 --warmup 2
line recovery --config recovery --steps 10 --warmup 2
line replay --config replay --steps 10 --warmup 2
line replay64 --config replay --value-len 64 --steps 5 --warmup 2
line append --config append --steps 10 --warmup 2
trace c2 --steps 20 --warmup 3
trace c3 --config entries --steps 10 --warmup 2
trace c3_100 --config entries --entry-size 100 --steps 10 --warmup 2
trace replay --config replay --steps 10 --warmup 2
pmc c3 --config entries --steps 10 --warmup 2
pmc c3_100 --config entries --entry-size 100 --steps 10 --warmup 2
