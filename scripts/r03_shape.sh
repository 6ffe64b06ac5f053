#!/bin/bash
# On-chip probe workgroup shape (PHJ_PROBE_SHAPE 0 = 1024 x 4, 1 = 512 x 8): parity, C2/C5 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_schedules.py -m gpu -x -q --timeout 300 --timeout-method thread -k "SHAPE or default" > gpurun_out/shape_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/shape_pytest.log; exit 1; }
tail -2 gpurun_out/shape_pytest.log
for cfg in c2 c5; do
for env in "PHJ_PROBE_SHAPE=0" "PHJ_PROBE_SHAPE=1" "PHJ_PROBE_SHAPE=0" "PHJ_PROBE_SHAPE=1"; do
  tag=${cfg}_$(echo $env | tr ' =' '_-')
  env $env timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-traffic --steps 10 > gpurun_out/sh_$tag.json 2> gpurun_out/sh_$tag.err || { echo "bench $env failed"; tail -5 gpurun_out/sh_$tag.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/sh_$tag.json')); print('$cfg $env', round(d['ms_per_step'],3), d['correct'], {k: round(v,3) for k,v in d['kernels_ms'].items()})"
done
done
for env in "PHJ_PROBE_SHAPE=0" "PHJ_PROBE_SHAPE=1"; do
  env $env timeout -k 10 300 python scripts/rehearse_world.py --worlds 8 > gpurun_out/sh_rehearse_$env.jsonl 2> gpurun_out/sh_rehearse.err || { echo "rehearse failed"; exit 5; }
  echo $env; cut -c1-60 gpurun_out/sh_rehearse_$env.jsonl
done
echo ok
