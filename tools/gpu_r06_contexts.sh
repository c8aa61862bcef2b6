# Round 6: the reference's concurrency shape: K contexts /
# host threads on one GPU, K in {1, 2, 4, 8, 16}, for the config-3 mix and
# replay at 64 B and 1 KiB values; plus (optionally) the GPU suite first.
#   SUITE=1 bash tools/gpu_r06_contexts.sh OUT
set -o pipefail
OUT=gpurun_out/${1:-r06/contexts}
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ "${SUITE:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1 || exit 1
fi
for K in ${KS:-1 2 4 8 16}; do
  timeout -k 10 300 python bench.py --config entries --contexts $K --steps ${STEPS:-20} > "$OUT/entries_k$K.json" 2> "$OUT/entries_k$K.err" || exit 1
  for v in ${VALUES:-64 1024}; do
    timeout -k 10 300 python bench.py --config replay --value-len $v --contexts $K --steps ${RSTEPS:-10} > "$OUT/replay${v}_k$K.json" 2> "$OUT/replay${v}_k$K.err" || exit 1
  done
done
