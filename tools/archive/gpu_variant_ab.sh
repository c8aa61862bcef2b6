# A/B of libramcrc build variants on entries benches: VARIANTS="a b" SIZES="1024 0"
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-vab}
mkdir -p $O
for rep in 1 2; do
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  for sz in $SIZES; do
    RAMCRC_LIB=$L timeout -k 10 300 python bench.py --config entries --entry-size $sz --steps 10 --warmup 2 --no-cpu-baseline >> $O/${v}_$sz.jsonl 2> $O/$v.err || exit 1
  done
done
done
