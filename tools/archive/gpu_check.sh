set -o pipefail
mkdir -p gpurun_out/ep
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit 1
for s in 100 1024 4096 0; do
  timeout -k 10 120 python bench.py --config entries --entry-size $s --steps 10 --warmup 2 > gpurun_out/ep/size_$s.json 2> gpurun_out/ep/size_$s.err || exit 1
done
timeout -k 10 120 python bench.py --config entries --path batch --steps 10 --warmup 2 > gpurun_out/ep/batch.json 2> gpurun_out/ep/batch.err
