# Round 6: verify-in-walk (k_walk_copyv) -- the walk/replay GPU tests, the
# replay lines at 64 / 128 / 1024 B values with the mode on and off, a kernel
# trace at 64 B, and per-kernel PMC passes (HBM traffic, LDS bank conflicts).
#   bash tools/gpu_r06_viw.sh OUT
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/${1:-viw}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_replay_fused.py \
    tests/test_gpu_segments.py tests/test_gpu_segment_ref.py -m gpu > $O/pytest.log 2>&1 || exit 1
for v in ${VALUES:-64 128 1024}; do
  for m in 1 0; do
    timeout -k 10 200 python bench.py --config replay --value-len $v --verify-in-walk $m --no-cpu-baseline \
        >> $O/replay_$v.jsonl 2>> $O/err.txt || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r64 -- \
    python3 bench.py --config replay --value-len 64 --steps 10 --no-cpu-baseline > $O/prof64.json 2>> $O/err.txt || exit 1
if [ "${PMC:-1}" = 1 ]; then
  for c in FETCH_SIZE WRITE_SIZE "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"; do
    tag=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$O/pmc/$tag" -o p -- \
        python3 bench.py --config replay --value-len 64 --steps 3 --warmup 1 --no-cpu-baseline > "$O/pmc_$tag.json" 2>> $O/err.txt || exit 1
  done
  python tools/pmc_kernels.py $O/pmc/* > $O/pmc_summary.txt 2>&1
fi
