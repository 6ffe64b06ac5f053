#!/bin/bash
# A/B the W = 1..8 rehearsal of two library builds on one box: the current
# partitionedhashjoin_amd/libphj_hip.so against partitionedhashjoin_amd/libphj_hip_prev.so,
# which must be built beforehand (e.g. `git stash; make lib; cp ...so ..._prev.so; git stash pop; make lib`).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_fullsize_group.py -x -q --timeout 300 --timeout-method thread > gpurun_out/reh_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/reh_tests.log; exit 1; }
tail -2 gpurun_out/reh_tests.log
for k in 1 2; do
  PHJ_LIB=partitionedhashjoin_amd/libphj_hip_prev.so timeout -k 10 200 python scripts/rehearse_world.py --worlds 8 4 > gpurun_out/reh_prev$k.jsonl 2>/dev/null || exit 2
  echo prev; cut -c1-90 gpurun_out/reh_prev$k.jsonl
  timeout -k 10 200 python scripts/rehearse_world.py --worlds 8 4 > gpurun_out/reh_new$k.jsonl 2>/dev/null || exit 3
  echo new; cut -c1-90 gpurun_out/reh_new$k.jsonl
done
