# Round 4: FETCH_SIZE passes (one counter pass each) for the entries and
# append lines, on the current tree; plus 40M x 96 B entries (steady-state
# tiny phase) for comparison with the replay's records-mode tiny phase.
set -o pipefail
OUT=gpurun_out/${1:-r04/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/mix" -o p -- python3 bench.py --config entries --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/mix.json" 2> "$OUT/mix.err" || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/e100" -o p -- python3 bench.py --config entries --entry-size 100 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/e100.json" 2> "$OUT/e100.err" || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/append" -o p -- python3 bench.py --config append --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/append.json" 2> "$OUT/append.err" || exit 1
timeout -k 10 120 python3 bench.py --config entries --entries 40000000 --entry-size 96 --steps 10 --no-cpu-baseline > "$OUT/e96_40m.json" 2> "$OUT/e96_40m.err" || exit 1
