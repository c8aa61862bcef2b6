# Round 4: slot-major wave ids in the tiny phases (tiny_wave) -- parity, then a
# same-box A/B against the workgroup-major mapping (tcm0) on tiny-heavy
# entries and replay batches.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04/tcm}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_binning.py tests/test_gpu_parity.py tests/test_gpu_segments.py > "$OUT/pytest.log" 2>&1 || exit 1
TAG=${1:-r04/tcm}/ab VARIANTS="tcm0" SIZES="100 160 0" bash tools/gpu_variant_ab.sh || exit 1
for rep in 1 2; do
for v in base tcm0; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  for vl in 64 128; do
    RAMCRC_LIB=$L timeout -k 10 300 python bench.py --config replay --value-len $vl --steps 10 --warmup 2 --no-cpu-baseline >> "$OUT/ab/${v}_replay$vl.jsonl" 2> "$OUT/ab/${v}_replay.err" || exit 1
  done
done
done
