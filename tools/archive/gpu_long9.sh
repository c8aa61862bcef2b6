# The flat-stream long phase (static split): whole GPU suite + smoke on the
# working tree, A/B against HEAD and the work-stealing variants, phase stamps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-long9}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
for s in 0 1024 4096; do
  RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_stamps.so timeout -k 10 120 python tools/stamps.py --entry-size $s >> $O/stamps.txt 2>&1 || exit 1
done
VARIANTS="${VARIANTS:-head st2 st2_sn4 st2_cpw1 st2_cpw2}" CASES="${CASES:---config entries;--config entries --entry-size 1024;--config entries --entry-size 4096;--config replay}" \
    REPS=${REPS:-2} TAG=${TAG:-long9}/ab bash tools/gpu_ab.sh || exit 1
