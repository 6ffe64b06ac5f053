#!/bin/bash
# Member tables + probe in d1 ranges (PHJ_FILL_SPLIT): group tests, rehearsal A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_fullsize_group.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/split_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/split_pytest.log; exit 1; }
tail -2 gpurun_out/split_pytest.log
for env in "PHJ_FILL_SPLIT=1" "PHJ_FILL_SPLIT=2" "PHJ_FILL_SPLIT=4" "PHJ_FILL_SPLIT=1" "PHJ_FILL_SPLIT=2" "PHJ_FILL_SPLIT=4"; do
  env $env timeout -k 10 300 python scripts/rehearse_world.py --worlds 1 8 > gpurun_out/split_$env.jsonl 2> gpurun_out/split.err || { echo "rehearse failed"; tail -5 gpurun_out/split.err; exit 5; }
  echo $env; cut -c1-60 gpurun_out/split_$env.jsonl
done
echo ok
