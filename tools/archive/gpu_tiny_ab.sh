set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tinyab}
mkdir -p $O
for v in base tinymask base tinymask; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  for sz in 100 0; do
    RAMCRC_LIB=$L timeout -k 10 300 python bench.py --config entries --entry-size $sz --steps 10 --warmup 2 --no-cpu-baseline >> $O/${v}_$sz.jsonl 2> $O/$v.err || exit 1
  done
done
