#!/bin/bash
# Round end on one box: the whole GPU suite, then the round profiles (bench lines, rocprof, rehearsal).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash scripts/round_profiles.sh
