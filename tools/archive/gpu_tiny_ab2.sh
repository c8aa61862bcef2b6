# Tiny-phase A/B: entry parity tests on the default build, then the entries
# bench (100 B and the config-3 mix) alternating the default build and the
# variants named in VARIANTS (built by ramcloud_amd.build.build_variants).
#   TAG=x VARIANTS="notrim" bash tools/gpu_tiny_ab2.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tinyab2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_write_path.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for rep in 1 2 3; do
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  for sz in ${SIZES:-100 0}; do
    RAMCRC_LIB=$L timeout -k 10 120 python bench.py --config entries --entry-size $sz --steps 20 --warmup 3 --no-cpu-baseline >> $O/${v}_$sz.jsonl 2>> $O/$v.err || exit 1
  done
done
done
