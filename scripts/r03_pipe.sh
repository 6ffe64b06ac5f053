#!/bin/bash
# Probe-side pass 1 in row ranges, each probed beside the next range's pass 1 (PHJ_PIPE): schedule tests, C2/C5 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_schedules.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "PIPE or default or fullsize or count" > gpurun_out/pipe_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pipe_pytest.log; exit 1; }
tail -2 gpurun_out/pipe_pytest.log
for cfg in c2 c5; do
for env in "PHJ_PIPE=1" "PHJ_PIPE=2" "PHJ_PIPE=4" "PHJ_PIPE=6" "PHJ_PIPE=1" "PHJ_PIPE=4"; do
  tag=${cfg}_$(echo $env | tr ' =' '_-')
  env $env timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-traffic --steps 10 > gpurun_out/pp_$tag.json 2> gpurun_out/pp_$tag.err || { echo "bench $env failed"; tail -5 gpurun_out/pp_$tag.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/pp_$tag.json')); print('$cfg $env', round(d['ms_per_step'],3), d['correct'], {k: round(v,3) for k,v in d['kernels_ms'].items()})"
done
done
echo ok
