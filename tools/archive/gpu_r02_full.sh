# Full GPU suite + smoke + bench lines (default, recovery N=1, entries, replay serial/pipelined).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --config recovery --steps 10 --warmup 2 > $O/recovery.json 2> $O/recovery.err || exit 1
timeout -k 10 300 python bench.py --config entries --steps 10 --warmup 2 > $O/entries.json 2> $O/entries.err || exit 1
timeout -k 10 300 python bench.py --config replay --steps 10 --warmup 2 > $O/replay.json 2> $O/replay.err || exit 1
timeout -k 10 300 python bench.py --config replay --walk-cus 128 --steps 10 --warmup 2 --no-cpu-baseline > $O/replay_pipe.json 2> $O/replay_pipe.err || exit 1
timeout -k 10 300 python bench.py --config replay --value-len 64 --replay-nseg 256 --steps 4 --warmup 1 --no-cpu-baseline > $O/replay64.json 2> $O/replay64.err || exit 1
timeout -k 10 300 python bench.py --config stream --nseg 256 --steps 3 > $O/stream.json 2> $O/stream.err || exit 1
timeout -k 10 300 python bench.py --config append --steps 10 --warmup 2 > $O/append.json 2> $O/append.err || exit 1
