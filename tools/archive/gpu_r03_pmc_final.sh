# End-of-round PMC passes of k_entries on 1M x 1 KiB entries and the config-3
# mix, and phase stamps of the final tree (probe build).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03pmc}
mkdir -p $O
BENCH="--config entries --entry-size 1024 --steps 2 --warmup 1" TAG=${TAG:-r03pmc}/e1k bash tools/gpu_pmc.sh || exit 1
BENCH="--config entries --steps 2 --warmup 1" TAG=${TAG:-r03pmc}/mix bash tools/gpu_pmc.sh || exit 1
for s in 0 1024 4096; do
  RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_stamps.so timeout -k 10 120 python tools/stamps.py --entry-size $s >> $O/stamps.txt 2>&1 || exit 1
done
