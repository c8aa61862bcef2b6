# Round 5: tiny-phase VALU cuts -- v_med3 tail clamp (md0 = the old
# max/add/min) and pf0 (no register prefetch of the next round's windows:
# loads go straight into the spent buffer, 40 copies and 6 VGPRs fewer).
set -o pipefail
O=gpurun_out/r05/tinyva
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_binning.py tests/test_gpu_parity.py tests/test_gpu_segments.py \
    tests/test_gpu_replay_fused.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VARIANTS="${VARIANTS:-md0 pf0}" CASES="${CASES:---config entries --entry-size 100;--config entries;--config replay --value-len 64;--config append}" \
    REPS=${REPS:-3} STEPS=20 TAG=${TAG:-r05/tinyva/ab} bash tools/gpu_ab.sh || exit 1
python tools/ab_summary.py gpurun_out/${TAG:-r05/tinyva/ab}
