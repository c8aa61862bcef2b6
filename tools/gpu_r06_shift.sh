# Round 6: replay at 2 KiB values ran slower than at 1 KiB (2.93 vs 3.29 TB/s):
# the part size the probe picks (128 KiB) against forced 64 / 256 KiB, and
# the 1 KiB and 4 KiB lines beside it; a kernel trace of the 2 KiB step.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06/${1:-shift}
mkdir -p $O
VS=${VS:-1024 2048 4096}
SS=${SS:-0 15 16 17 18}
for rep in 1 2; do
  for v in $VS; do
    for s in $SS; do
      a=""; [ $s != 0 ] && a="--walk-part-shift $s"
      timeout -k 10 200 python bench.py --config replay --value-len $v $a --steps 10 --warmup 2 --no-cpu-baseline \
          >> $O/v${v}_s$s.jsonl 2>> $O/err.txt || exit 1
    done
  done
done
[ -n "$NOPROF" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r2048 -- \
    python3 bench.py --config replay --value-len 2048 --steps 10 --no-cpu-baseline > $O/prof2048.json 2>> $O/err.txt || exit 1
