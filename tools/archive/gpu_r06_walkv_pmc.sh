# Round 6: SQ counters of the fused part walk (walkv variant) at 64 B values.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/${1:-walkvpmc}
mkdir -p $O/pmc
RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_walkv.so timeout -s KILL 150 rocprofv3 \
    --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_WAVES \
    --output-format csv -d $O/pmc/sq -o p -- \
    python3 bench.py --config replay --value-len 64 --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_sq.json 2>> $O/err.txt || exit 1
python tools/pmc_kernels.py $O/pmc/* > $O/pmc_summary.txt 2>&1
