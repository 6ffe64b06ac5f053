#!/bin/bash
# CU-split streams (PHJ_CU_SPLIT) and the ungrouped probe over hash codes, C2 A/B on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_schedules.py -x -q --timeout 200 --timeout-method thread -k "CU_SPLIT or default" > gpurun_out/pytest_split.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_split.log; exit 1; }
tail -1 gpurun_out/pytest_split.log
for v in 0 4 8 2 0 4; do
  PHJ_CU_SPLIT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic > gpurun_out/ab_split$v.json 2>> gpurun_out/ab.err || { echo "split $v failed"; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/ab_split$v.json')); k=d['kernels_ms']; print('split $v', round(d['ms_per_step'],4), d['correct'], k['S.p1.scatter'], k['build'], k['probe'])"
done
PHJ_P1_GRP=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic > gpurun_out/ab_grp0.json 2>> gpurun_out/ab.err || { echo "grp0 failed"; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/ab_grp0.json')); k=d['kernels_ms']; print('grp0', round(d['ms_per_step'],4), d['correct'], k['S.p1.scatter'], k['probe'])"
echo ok
