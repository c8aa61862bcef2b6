# Round 6: HBM traffic of every kernel of the replay step on the final tree
# (FETCH_SIZE and WRITE_SIZE, one counter per pass) at 64 B and 128 B values.
set -o pipefail
OUT=gpurun_out/r06/pmc_step
mkdir -p $OUT
export TMPDIR=/tmp
for v in 64 128; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$OUT/v${v}_$c" -o p -- \
        python3 bench.py --config replay --value-len $v --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/v${v}_$c.json" 2> "$OUT/v${v}_$c.err" || exit 1
  done
done
