#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
PHJ_P1_TABLE=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_p1t.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_p1t.log; exit 1; }
tail -1 gpurun_out/pytest_p1t.log
run() {
  env ${1//,/ } timeout -k 10 200 python bench.py ${@:2} --no-traffic --no-cpu-baseline --steps 20 > gpurun_out/b.json 2> gpurun_out/b.err || { echo "bench failed $*"; tail -5 gpurun_out/b.err; exit 2; }
  python3 -c "import json;b=json.load(open('gpurun_out/b.json'));k=b['kernels_ms'];print('$*', round(b['ms_per_step'],4), b['correct'], {a:round(v,3) for a,v in k.items() if not a.startswith('R.')})"
}
run PHJ_P1_TABLE=0
run PHJ_P1_TABLE=1
run PHJ_P1_TABLE=0 --config c5
run PHJ_P1_TABLE=1 --config c5
echo ok
