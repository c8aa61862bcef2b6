# FETCH_SIZE passes (one counter pass per run, nothing else collected) of
# every workload whose bench line reports roofline.traffic.  Afterwards, on
# the build host:  python tools/final_pmc_digest.py OUT  -> profiles/pmc/*.json
#     bash tools/final_pmc.sh [OUT]      (default gpurun_out/pmc)
set -o pipefail
OUT=gpurun_out/${1:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name, bench arguments...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/$n" -o p -- \
      python3 bench.py "$@" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/$n.json" 2> "$OUT/$n.err"
}
if [ -n "$EXTRA" ]; then   # only the replay sizes added in round 6
  for v in 512 2048 3072 4096; do run replay$v --config replay --value-len $v || exit 1; done
  exit 0
fi
run c2 || exit 1
run c4 --config recovery --no-t1 || exit 1
run mix --config entries || exit 1
run e100 --config entries --entry-size 100 || exit 1
run append --config append || exit 1
run replay --config replay || exit 1
run replay64 --config replay --value-len 64 || exit 1
run replay128 --config replay --value-len 128 || exit 1
run replay256 --config replay --value-len 256 || exit 1
run replay8192 --config replay --value-len 8192 || exit 1
run e1024 --config entries --entry-size 1024 || exit 1
run e4096 --config entries --entry-size 4096 || exit 1
