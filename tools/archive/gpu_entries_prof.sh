# Entries path (config 3): per-size benches, a kernel trace per size, and a
# FETCH_SIZE pass of the Zipf mix (HBM traffic of the scan kernels).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${ROUND:-r01}/entries
mkdir -p $O
for s in 100 1024 4096 0; do
  timeout -k 10 120 python bench.py --config entries --entry-size $s --steps 10 --warmup 2 > $O/size_$s.json 2> $O/size_$s.err || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$s -o p \
      -- python3 bench.py --config entries --entry-size $s --steps 10 --warmup 2 > /dev/null 2> $O/t_$s.err || exit 1
done
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p \
    -- python3 bench.py --config entries --steps 5 --warmup 1 > $O/pmc_fetch_bench.json 2> $O/pmc_fetch.err || exit 1
