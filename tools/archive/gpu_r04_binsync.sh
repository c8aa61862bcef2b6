# Round 4: k_bin_one variants (A/B by step time) and kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04/binsync}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_binning.py > "$OUT/pytest_bin.log" 2>&1 || exit 1
TAG=${1:-r04/binsync}/ab VARIANTS="bo0 bsp4" SIZES="0 100" bash tools/gpu_variant_ab.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c3 -- python bench.py --config entries --entry-size 0 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_c3.json" 2> "$OUT/prof_c3.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c3_100 -- python bench.py --config entries --entry-size 100 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_c3_100.json" 2> "$OUT/prof_c3_100.err" || exit 1
