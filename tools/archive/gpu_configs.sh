# Secondary configs: C3 entries (both paths), C5 streaming, C4 recovery on 1 GPU.
set -o pipefail
mkdir -p gpurun_out/cfg
timeout -k 10 300 python bench.py --config entries --path entries --steps 5 --warmup 1 > gpurun_out/cfg/entries.json 2> gpurun_out/cfg/entries.err && \
timeout -k 10 300 python bench.py --config entries --path batch --steps 5 --warmup 1 > gpurun_out/cfg/entries_batch.json 2> gpurun_out/cfg/entries_batch.err && \
timeout -k 10 300 python bench.py --config stream --nseg 256 --steps 3 > gpurun_out/cfg/stream.json 2> gpurun_out/cfg/stream.err && \
timeout -k 10 300 python bench.py --config recovery --nseg-total 2048 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/cfg/recovery.json 2> gpurun_out/cfg/recovery.err
