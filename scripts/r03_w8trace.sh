#!/bin/bash
# Kernel timelines: one rehearsed W=8 member step and one C2 step (rocprofv3 kernel trace).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/w8trace" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/rehearse_world.py" --worlds 8 --steps 5 > "$GRAFT_REPO_ROOT/gpurun_out/w8trace.log" 2>&1) || { echo "rocprof w8 failed"; tail -5 gpurun_out/w8trace.log; exit 3; }
python3 scripts/trace_summary.py gpurun_out/w8trace --step-kernel k_probe_ht > gpurun_out/w8trace.txt 2>&1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/c2trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > "$GRAFT_REPO_ROOT/gpurun_out/c2trace.log" 2>&1) || { echo "rocprof c2 failed"; tail -5 gpurun_out/c2trace.log; exit 4; }
python3 scripts/trace_summary.py gpurun_out/c2trace --step-kernel k_probe_ht > gpurun_out/c2trace.txt 2>&1
echo ok
