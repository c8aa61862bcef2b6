# Round 6: the part walk's LDS record rows rotated per lane: walk/replay tests,
# replay A/B against lrot0 (a knob removed afterwards; its build was wrong,
# so the A/B is void) and the LDS bank-conflict pass (pmc_summary.txt).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/${1:-lrot}
mkdir -p $O/pmc
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_replay_fused.py tests/test_gpu_segments.py tests/test_gpu_segment_ref.py \
    -m gpu > $O/pytest.log 2>&1 || exit 1
VARIANTS="lrot0" CASES="--config replay --value-len 64;--config replay --value-len 128;--config replay --value-len 1024" \
  REPS=3 STEPS=10 TAG=r06/${1:-lrot}/ab bash tools/gpu_ab.sh || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
    --output-format csv -d $O/pmc/lds -o p -- \
    python3 bench.py --config replay --value-len 64 --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_lds.json 2>> $O/err.txt || exit 1
python tools/pmc_kernels.py $O/pmc/* > $O/pmc_summary.txt 2>&1
