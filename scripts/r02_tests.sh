#!/bin/bash
# New GPU tests (full size, schedules) + the C2 bench with the three CPU legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_schedules.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_new.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_new.log; exit 1; }
tail -3 gpurun_out/pytest_new.log
timeout -k 10 400 python bench.py --verbose --no-traffic > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench failed"; tail -5 gpurun_out/bench_c2.err; exit 2; }
cut -c1-300 gpurun_out/bench_c2.json
echo ok
