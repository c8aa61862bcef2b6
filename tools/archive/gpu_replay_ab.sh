# Replay A/B within one box: base and each variant, twice, alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-replayab}
mkdir -p $O
for rep in 1 2; do
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  RAMCRC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$rep -o t -- python3 bench.py --config replay --steps 10 --warmup 2 --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit 1
done
done
