# Round 4: counters of the steady-state tiny phase (40M x 96 B entries), one
# pass per counter group; then the k_walk_copy unroll A/B on replay 64 B.
set -o pipefail
OUT=gpurun_out/${1:-r04/tinypmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d "$OUT/a" -o p -- python3 bench.py --config entries --entries 40000000 --entry-size 96 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> "$OUT/a.err" || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY --output-format csv -d "$OUT/b" -o p -- python3 bench.py --config entries --entries 40000000 --entry-size 96 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> "$OUT/b.err" || exit 1
VARIANTS="cu2 cu8" CASES="--config replay --value-len 64" REPS=2 TAG=r04/ab_copy bash tools/gpu_ab.sh || exit 1
