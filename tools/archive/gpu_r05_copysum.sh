# Round 5: cost of the replay summary inside k_walk_copy (cs0 = a timing
# probe without it) on the 64 B-value replay, with traces of both.
set -o pipefail
OUT=gpurun_out/r05/copysum
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof"
timeout -k 10 300 $P -o base -- python3 bench.py --config replay --value-len 64 --steps 10 --no-cpu-baseline > $OUT/prof_base.json 2> $OUT/prof_base.err || exit 1
RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_cs0.so timeout -k 10 300 $P -o cs0 -- python3 bench.py --config replay --value-len 64 --steps 10 --no-cpu-baseline > $OUT/prof_cs0.json 2> $OUT/prof_cs0.err || exit 1
grep -h k_walk_copy $OUT/prof/*kernel_stats.csv
