set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/te
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/te/mix -o p -- python3 bench.py --config entries --steps 10 --warmup 2 > gpurun_out/te/mix.json 2> gpurun_out/te/mix.err
