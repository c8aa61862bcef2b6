# PMC passes (one counter group per pass) for the entries path; sizes as args (0 = mixed).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/epm
for s in "$@"; do
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/epm/a_$s -o p -- python3 bench.py --config entries --entry-size $s --steps 2 --warmup 1 > /dev/null 2> gpurun_out/epm/a_$s.err || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/epm/b_$s -o p -- python3 bench.py --config entries --entry-size $s --steps 2 --warmup 1 > /dev/null 2> gpurun_out/epm/b_$s.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/epm/t_$s -o p -- python3 bench.py --config entries --entry-size $s --steps 5 --warmup 1 > /dev/null 2> gpurun_out/epm/t_$s.err || exit 1
done
