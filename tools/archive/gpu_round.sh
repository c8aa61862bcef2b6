# One GPU call: parity tests, smoke, the headline bench, the secondary configs,
# then the rocprofv3 kernel-trace pass and the PMC passes of the headline bench.
# Every GPU step has its own time limit; the first failure ends the script.
#   ROUND=r01 CONFIGS="entries replay" bash tools/gpu_round.sh
set -o pipefail
export TMPDIR=/tmp
R=${ROUND:-r01}
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
for c in ${CONFIGS:-entries entries_batch stream recovery}; do
  case $c in
    entries) args="--config entries --steps 10 --warmup 2" ;;
    entries_batch) args="--config entries --path batch --steps 10 --warmup 2" ;;
    stream) args="--config stream --nseg 256 --steps 3" ;;
    recovery) args="--config recovery --nseg-total 2048 --steps 10 --warmup 2 --no-cpu-baseline" ;;
    *) args="--config $c --steps 10 --warmup 2" ;;
  esac
  timeout -k 10 300 python bench.py $args > $O/$c.json 2> $O/$c.err || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench \
    -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc \
    -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_fetch_bench.json 2> $O/pmc_fetch.err || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_lds -o pmc \
    -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_lds_bench.json 2> $O/pmc_lds.err || exit 1
