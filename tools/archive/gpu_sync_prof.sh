# Kernel traces of the replay config (base library and the searly variant) and
# one SQ counter pass over the walk kernels.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sync2
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/base -o run -- python3 bench.py --config replay --steps 5 --warmup 2 --no-cpu-baseline > $O/base.log 2>&1 &&
RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_searly.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/searly -o run -- python3 bench.py --config replay --steps 5 --warmup 2 --no-cpu-baseline > $O/searly.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/v64 -o run -- python3 bench.py --config replay --value-len 64 --steps 5 --warmup 2 --no-cpu-baseline > $O/v64.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --kernel-include-regex "k_walk|k_entries|k_bin" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES -d $O/pmc -o run -- python3 bench.py --config replay --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc.log 2>&1
