#!/bin/bash
# Kernel timeline of a few C2 steps (rocprofv3 kernel trace) at PHJ_P1_WPC2=2 and 4:
# when does R's chain run beside S's persistent pass 1?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 2 4; do
  (cd /tmp && PHJ_P1_WPC2=$w timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace_w$w -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $GRAFT_REPO_ROOT/gpurun_out/trace_w$w.log 2>&1) || { echo "trace $w failed"; tail -5 gpurun_out/trace_w$w.log; exit 1; }
done
echo ok
