# Round 5: k_walk_fix's per-segment record (RAMCRC_WALK_DEBUG build) on the
# 128 B- and 64 B-value replays: which segments leave the fast path, and why.
set -o pipefail
OUT=gpurun_out/r05/walkdbg
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in 128 64; do
  RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_walkdbg.so timeout -k 10 200 python3 bench.py --config replay --value-len $v \
      --steps 1 --warmup 0 --no-cpu-baseline > $OUT/replay$v.log 2> $OUT/replay$v.err || exit 1
  grep -c fixdbg $OUT/replay$v.log || true
  grep fixsum $OUT/replay$v.log | head -3 || true
done
