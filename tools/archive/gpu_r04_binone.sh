# Round 4: one-launch binning (k_bin_one) -- binning/parity tests, the whole
# GPU suite, a same-box A/B against the two-launch build (bo0) and the
# 32-unit poll sleep (bsp32) on the entries configs and the append workload,
# and kernel traces of the config-3 mix and 100-byte entries.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04/binone}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_binning.py tests/test_gpu_parity.py > "$OUT/pytest_bin.log" 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1 || exit 1
TAG=${1:-r04/binone}/ab VARIANTS="bo0 bsp32" SIZES="0 100 1024 4096" bash tools/gpu_variant_ab.sh || exit 1
for rep in 1 2; do
for v in base bo0; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  RAMCRC_LIB=$L timeout -k 10 300 python bench.py --config append --steps 10 --warmup 2 --no-cpu-baseline >> "$OUT/ab/${v}_append.jsonl" 2> "$OUT/ab/${v}_append.err" || exit 1
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c3 -- python bench.py --config entries --entry-size 0 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_c3.json" 2> "$OUT/prof_c3.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c3_100 -- python bench.py --config entries --entry-size 100 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_c3_100.json" 2> "$OUT/prof_c3_100.err" || exit 1
