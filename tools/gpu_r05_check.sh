# Round 5: the GPU suite, the config-4 line (cpu_baseline) and traces of the
# 100-byte-entry binning, one launch vs two.
set -o pipefail
O=gpurun_out/r05/check
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --config recovery --steps 10 --warmup 2 > $O/recovery.json 2> $O/recovery.err || exit 1
cat $O/recovery.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base bo0; do
  if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
  RAMCRC_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- \
      python bench.py --config entries --entry-size 100 --steps 20 --warmup 3 --no-cpu-baseline \
      > $O/c3_100_$v.json 2> $O/prof_$v.err || exit 1
done
find $O -name "*kernel_stats.csv" | head
