# A/B the k_chunks tuning variants on the headline config (interleaved, 2 rounds).
set -o pipefail
mkdir -p gpurun_out/var
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/var/pytest_gpu.log 2>&1 || exit 1
for round in 1 2; do
  for v in ramcloud_amd/lib/variants/*.so; do
    n=$(basename $v .so)
    RAMCRC_LIB=$PWD/$v timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/var/${n}_$round.json 2> gpurun_out/var/${n}_$round.err || exit 1
  done
done
