# Round 5: where the long phase's cycles go (1M x 1 KiB entries and the
# config-3 mix): VALU / LDS instruction counts, busy and wait cycles of
# k_entries, one counter pass per run.
set -o pipefail
OUT=gpurun_out/r05/pmc_long
mkdir -p $OUT
export TMPDIR=/tmp
run() {   # name, counters, bench arguments...
  local n=$1 c=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$OUT/$n" -o p -- \
      python3 bench.py "$@" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/$n.json" 2> "$OUT/$n.err"
}
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
C2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"
run k1_a "$C1" --config entries --entry-size 1024 || exit 1
run k1_b "$C2" --config entries --entry-size 1024 || exit 1
run mix_a "$C1" --config entries || exit 1
run mix_b "$C2" --config entries || exit 1
run t100_a "$C1" --config entries --entry-size 100 || exit 1
run t100_b "$C2" --config entries --entry-size 100 || exit 1
ls $OUT
