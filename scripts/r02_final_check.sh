#!/bin/bash
# Whole GPU suite, then C2 with hash codes (default) and without (A/B, same box).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic > gpurun_out/bench_c2_hc.json 2> gpurun_out/bench_c2_hc.err || { echo "bench failed"; tail -5 gpurun_out/bench_c2_hc.err; exit 2; }
PHJ_P1_HCODE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic > gpurun_out/bench_c2_nohc.json 2> gpurun_out/bench_c2_nohc.err || { echo "bench0 failed"; exit 3; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic > gpurun_out/bench_c2_hc2.json 2>> gpurun_out/bench_c2_hc.err || { echo "bench2 failed"; exit 4; }
PHJ_P1_HOME=2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic > gpurun_out/bench_c2_home2.json 2> gpurun_out/bench_c2_home2.err || { echo "bench home2 failed"; exit 5; }
timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/rehearse.jsonl 2> gpurun_out/rehearse.err || { echo "rehearse failed"; exit 6; }
cut -c1-90 gpurun_out/rehearse.jsonl
for f in gpurun_out/bench_c2_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['correct'], d['kernels_ms'])"; done
echo ok
