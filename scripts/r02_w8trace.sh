#!/bin/bash
# Kernel timeline of one rehearsed W=8 member step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/w8trace" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/rehearse_world.py" --worlds 8 --steps 5 > "$GRAFT_REPO_ROOT/gpurun_out/w8trace.log" 2>&1) || { echo "rocprof failed"; tail -5 gpurun_out/w8trace.log; exit 3; }
python3 scripts/trace_summary.py gpurun_out/w8trace --step-kernel k_probe_p1 > gpurun_out/w8trace.txt 2>&1
tail -60 gpurun_out/w8trace.txt
