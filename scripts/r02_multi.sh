#!/bin/bash
# Multi-device contexts on one GPU (local members, RCCL world of one), CLI, then the bench at N=1 and --exchange.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_cli.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_multi.log; exit 1; }
tail -3 gpurun_out/pytest_multi.log
timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench failed"; tail -20 gpurun_out/bench_c2.err; exit 2; }
cut -c1-400 gpurun_out/bench_c2.json
timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --exchange > gpurun_out/bench_x.json 2> gpurun_out/bench_x.err || { echo "bench exchange failed"; tail -20 gpurun_out/bench_x.err; exit 3; }
cut -c1-400 gpurun_out/bench_x.json
timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --exchange --config c4 > gpurun_out/bench_x4.json 2> gpurun_out/bench_x4.err || { echo "bench exchange c4 failed"; tail -20 gpurun_out/bench_x4.err; exit 4; }
cut -c1-400 gpurun_out/bench_x4.json
echo ok
