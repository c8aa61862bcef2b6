set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ep
for s in 100 1024 4096 0; do
  timeout -k 10 120 python bench.py --config entries --entry-size $s --steps 5 --warmup 1 > gpurun_out/ep/size_$s.json 2> gpurun_out/ep/size_$s.err || exit 1
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/ep/pmc -o p -- python3 bench.py --config entries --steps 2 --warmup 1 > /dev/null 2> gpurun_out/ep/pmc.err
