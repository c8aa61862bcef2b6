# A/B of libramcrc build variants on one box, interleaved: for each rep, the
# base library and every variant run every case.  Cases are bench.py argument
# strings separated by ';'.
#   VARIANTS="a b" CASES="--config entries;--config entries --entry-size 100" REPS=3 TAG=ab1 \
#       bash tools/gpu_ab.sh
# -> gpurun_out/$TAG/<variant>_<case#>.jsonl (summarise with tools/ab_summary.py)
set -o pipefail
O=gpurun_out/${TAG:-ab}
mkdir -p $O
IFS=';' read -r -a CS <<< "${CASES:---config entries}"
for rep in $(seq 1 ${REPS:-2}); do
  for v in base $VARIANTS; do
    if [ $v = base ]; then L=""; else L=ramcloud_amd/lib/variants/libramcrc_$v.so; fi
    for i in "${!CS[@]}"; do
      RAMCRC_LIB=$L timeout -k 10 200 python bench.py ${CS[$i]} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
          >> $O/${v}_$i.jsonl 2>> $O/${v}.err || exit 1
    done
  done
done
echo "${CASES}" > $O/cases.txt
