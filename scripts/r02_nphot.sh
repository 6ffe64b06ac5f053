#!/bin/bash
# NoPartitioning probe variants: parity of the cooperative probe, then C4 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
PHJ_NP_HOT=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "np or nopart or NP or C4 or c1 or seeded" > gpurun_out/pytest_np.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_np.log; exit 1; }
tail -2 gpurun_out/pytest_np.log
run() {
  env "$@" timeout -k 10 200 python bench.py --config c4 --no-traffic --no-cpu-baseline --steps 10 > gpurun_out/b.json 2> gpurun_out/b.err || { echo "bench failed $*"; tail -5 gpurun_out/b.err; exit 2; }
  python3 -c "import json;b=json.load(open('gpurun_out/b.json'));k=b['kernels_ms'];print('$*', round(b['ms_per_step'],4), b['correct'], k.get('np.build'), k.get('np.probe'))"
}
run PHJ_NP_HOT=0 PHJ_NP_COOP=0
run PHJ_NP_HOT=0 PHJ_NP_COOP=1
run PHJ_NP_HOT=0 PHJ_NP_COOP=1 PHJ_NP_ITEMS=8
run PHJ_NP_HOT=0 PHJ_NP_DIAG=4
run PHJ_NP_HOT=1
run PHJ_NP_HOT=0 PHJ_NP_COOP=1 PHJ_NP_RATIO_DUMMY=1
echo ok
