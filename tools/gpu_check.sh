set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err && \
timeout -k 10 300 python bench.py --config recovery --nseg-total 256 --steps 20 --no-cpu-baseline > gpurun_out/recovery256.json 2> gpurun_out/recovery256.err && \
timeout -k 10 300 python bench.py --config entries --steps 10 --warmup 2 > gpurun_out/entries.json 2> gpurun_out/entries.err
