#!/bin/bash
# Private-chain pass 1: full GPU suite, then A/B against the shared chains.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash scripts/ab.sh "PHJ_P1_PRIV=0" "" "PHJ_P1_PRIV=0" ""
