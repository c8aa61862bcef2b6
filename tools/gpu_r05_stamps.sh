# Round 5: k_entries phase stamps (mix, 1 KiB, 4 KiB) and the guarded
# scatter's cost after its one-load vote read (base vs rs0).
set -o pipefail
O=gpurun_out/r05/stamps
mkdir -p $O
L=ramcloud_amd/lib/variants/libramcrc_stamps.so
RAMCRC_LIB=$L timeout -k 10 200 python tools/stamps.py --save $O/mix.npy > $O/stamps_mix.txt 2>&1 || exit 1
RAMCRC_LIB=$L timeout -k 10 200 python tools/stamps.py --entry-size 1024 --save $O/1k.npy > $O/stamps_1k.txt 2>&1 || exit 1
RAMCRC_LIB=$L timeout -k 10 200 python tools/stamps.py --entry-size 4096 --save $O/4k.npy > $O/stamps_4k.txt 2>&1 || exit 1
cat $O/stamps_mix.txt
VARIANTS="rs0" CASES="--config entries --entry-size 100;--config entries" REPS=3 STEPS=20 TAG=r05/stamps/ab bash tools/gpu_ab.sh || exit 1
python tools/ab_summary.py gpurun_out/r05/stamps/ab
