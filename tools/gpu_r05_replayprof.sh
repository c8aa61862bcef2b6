# Round 5: kernel traces of the replay lines (1 KiB and 64 B values) on the
# current tree, to place the 1 KiB step's growth since round 4.
set -o pipefail
OUT=gpurun_out/r05/replayprof
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof"
timeout -k 10 300 $P -o replay -- python3 bench.py --config replay --steps 10 --no-cpu-baseline > $OUT/prof_replay.json 2> $OUT/prof_replay.err || exit 1
timeout -k 10 300 $P -o replay64 -- python3 bench.py --config replay --value-len 64 --steps 10 --no-cpu-baseline > $OUT/prof_replay64.json 2> $OUT/prof_replay64.err || exit 1
timeout -k 10 200 python3 bench.py --config replay --steps 10 --no-cpu-baseline > $OUT/replay.json 2> $OUT/replay.err || exit 1
cat $OUT/replay.json
