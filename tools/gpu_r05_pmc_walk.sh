# Round 5: HBM traffic of the walk kernels on the 64 B-value replay
# (FETCH_SIZE and WRITE_SIZE, one counter per pass).
set -o pipefail
OUT=gpurun_out/r05/pmc_walk
mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$OUT/$c" -o p -- \
      python3 bench.py --config replay --value-len 64 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$c.json" 2> "$OUT/$c.err" || exit 1
done
