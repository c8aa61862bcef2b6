# Round 3: the binning diagnostic and robustness tests first, then the whole
# GPU suite, smoke and the default bench line on this tree (library built
# here, shipped prebuilt).
set -o pipefail
OUT=gpurun_out/${1:-r03}
mkdir -p "$OUT"
python -c "import ramcloud_amd.ramcrc as r; print(r.lib().ramcrc_build_info().decode())" > "$OUT/build_info.txt" 2>&1 || exit 1
timeout -k 10 150 python tools/diag_plan_skip.py 12 plain > "$OUT/diag.txt" 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_binning.py tests/test_gpu_certify.py > "$OUT/pytest_new.log" 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
