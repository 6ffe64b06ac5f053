#!/bin/bash
# Keys-only chunked pass 1: full GPU suite, then A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash scripts/ab.sh "PHJ_P1_KO=0" "" "PHJ_P1_KO=0" "" || exit 1
CFG=c5 bash scripts/ab.sh "PHJ_P1_KO=0" ""
