# Entries A/B within one box, alternating base and variants twice; kernel
# trace per run.  VARIANTS="a b" SIZES="100 0"
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-entab}
mkdir -p $O
for rep in 1 2; do
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  for sz in $SIZES; do
    RAMCRC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_${sz}_$rep -o t -- python3 bench.py --config entries --entry-size $sz --steps 10 --warmup 2 --no-cpu-baseline > $O/${v}_${sz}_$rep.json 2> $O/${v}_${sz}_$rep.err || exit 1
  done
done
done
