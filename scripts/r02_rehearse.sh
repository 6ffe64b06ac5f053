#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python scripts/rehearse_world.py > gpurun_out/rehearse.jsonl 2> gpurun_out/rehearse.err || { echo "rehearse failed"; tail -20 gpurun_out/rehearse.err; exit 4; }
cut -c1-500 gpurun_out/rehearse.jsonl
