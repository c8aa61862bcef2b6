# Round-2 GPU call: the GPU suite, smoke, the default bench line and the
# config-4 / config-3 lines.  Every GPU step has its own time limit; the first
# failure ends the script.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --config recovery --steps 10 --warmup 2 > $O/recovery.json 2> $O/recovery.err || exit 1
timeout -k 10 300 python bench.py --config entries --steps 10 --warmup 2 > $O/entries.json 2> $O/entries.err || exit 1
