#!/bin/bash
# Chunked pass-1 variants: parity of every schedule touching it, then A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_schedules.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "P1_VAR or fullsize or c2 or c5" > gpurun_out/pytest_p1var.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_p1var.log; exit 1; }
tail -1 gpurun_out/pytest_p1var.log
bash scripts/ab.sh "PHJ_P1_VAR=0" "" "PHJ_P1_VAR=1" "PHJ_P1_VAR=0" ""
