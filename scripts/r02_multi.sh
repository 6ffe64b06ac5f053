#!/bin/bash
# Multi-device contexts on one GPU (local members, RCCL world of one), CLI, exchange bench, W rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_multi.log; exit 1; }
tail -1 gpurun_out/pytest_multi.log
timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --exchange > gpurun_out/bench_x.json 2> gpurun_out/bench_x.err || { echo "bench exchange failed"; tail -20 gpurun_out/bench_x.err; exit 3; }
python3 -c "import json;b=json.load(open('gpurun_out/bench_x.json'));print('exchange c2', round(b['ms_per_step'],4), b['correct'], b['exchange_ms'])"
timeout -k 10 400 python scripts/rehearse_world.py > gpurun_out/rehearse.jsonl 2> gpurun_out/rehearse.err || { echo "rehearse failed"; tail -20 gpurun_out/rehearse.err; exit 4; }
cut -c1-400 gpurun_out/rehearse.jsonl
echo ok
