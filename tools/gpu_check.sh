set -o pipefail
mkdir -p gpurun_out
(nproc; lscpu | head -20; rocm-smi --showproductname) > gpurun_out/host_info.txt 2>&1 || true
timeout -k 10 700 python -m pytest tests -m gpu -x -q  > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
