# A/B of the walk's sync-search variants: kernel trace of the replay bench per
# libramcrc variant (VARIANTS="sh4 sp16 ..."), walk kernels' averages compared.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-syncab}
mkdir -p $O
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  RAMCRC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o t -- python3 bench.py --config replay --steps 6 --warmup 2 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || exit 1
done
