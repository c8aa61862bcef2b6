# Round 5, final tree: k_entries phase stamps on 1M x 100 B entries and the
# config-3 mix (where the tiny phase's time goes after the VALU cuts).
set -o pipefail
O=gpurun_out/r05/stamps2
mkdir -p $O
L=ramcloud_amd/lib/variants/libramcrc_stamps.so
RAMCRC_LIB=$L timeout -k 10 200 python tools/stamps.py --entry-size 100 --save $O/e100.npy > $O/stamps_100.txt 2>&1 || exit 1
RAMCRC_LIB=$L timeout -k 10 200 python tools/stamps.py --save $O/mix.npy > $O/stamps_mix.txt 2>&1 || exit 1
cat $O/stamps_100.txt
