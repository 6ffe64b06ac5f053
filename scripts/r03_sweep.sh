#!/bin/bash
# The reference's generate.sh sweep (-p 32..8192 and NoPartitioning, both skews) on the current build, CPU columns too.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 1000 python scripts/sweep.py --skew 1.05 1.25 --gpus 1 --cpu --cpu-threads 15 --out gpurun_out/r03_sweep_cli > gpurun_out/sweep.log 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/sweep.log; exit 1; }
cat gpurun_out/r03_sweep_cli_*.dat
