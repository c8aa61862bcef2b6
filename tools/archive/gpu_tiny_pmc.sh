# Extra PMC passes on the entries path (instruction cache, LDS detail).  Args: entry sizes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tpm
for s in "$@"; do
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/tpm/c_$s -o p -- python3 bench.py --config entries --entry-size $s --steps 2 --warmup 1 > /dev/null 2> gpurun_out/tpm/c_$s.err || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL --output-format csv -d gpurun_out/tpm/d_$s -o p -- python3 bench.py --config entries --entry-size $s --steps 2 --warmup 1 > /dev/null 2> gpurun_out/tpm/d_$s.err || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d gpurun_out/tpm/e_$s -o p -- python3 bench.py --config entries --entry-size $s --steps 2 --warmup 1 > /dev/null 2> gpurun_out/tpm/e_$s.err || exit 1
done
