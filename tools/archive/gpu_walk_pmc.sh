# PMC passes for the walk kernels (replay config), one counter group per pass.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-walkpmc}
mkdir -p $O
B="python3 bench.py --config replay --replay-nseg 256 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d $O/a -o p -- $B > /dev/null 2> $O/a.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/b -o p -- $B > /dev/null 2> $O/b.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c -o p -- $B > /dev/null 2> $O/c.err || exit 1
python tools/pmc_kernels.py $O/a $O/b $O/c > $O/summary.txt
