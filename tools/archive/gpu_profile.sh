# rocprofv3 kernel-trace/stats pass and separate PMC passes for the bench.
set -o pipefail
export TMPDIR=/tmp
R=${ROUND:-r01}
mkdir -p gpurun_out/prof_$R
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R/trace -o bench \
    -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$R/trace_bench.json 2> gpurun_out/prof_$R/trace.err && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_$R/pmc_fetch -o pmc \
    -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$R/pmc_fetch_bench.json 2> gpurun_out/prof_$R/pmc_fetch.err && \
timeout -k 10 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof_$R/pmc_lds -o pmc \
    -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$R/pmc_lds_bench.json 2> gpurun_out/prof_$R/pmc_lds.err
