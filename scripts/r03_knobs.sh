#!/bin/bash
# After the lighter R chain: pass-1 grid (PHJ_P1_WPC2) A/B at C2/C5, and the
# rehearsal with event timers off (device time without the per-kernel markers).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in c2 c5; do
for env in "PHJ_P1_WPC2=2" "PHJ_P1_WPC2=3" "PHJ_P1_WPC2=4" "PHJ_P1_WPC2=2" "PHJ_P1_WPC2=3" "PHJ_P1_WPC2=4"; do
  tag=${cfg}_$(echo $env | tr ' =' '_-')
  env $env timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-traffic --steps 10 > gpurun_out/kn_$tag.json 2> gpurun_out/kn_$tag.err || { echo "bench $env failed"; tail -5 gpurun_out/kn_$tag.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/kn_$tag.json')); print('$cfg $env', round(d['ms_per_step'],3), d['correct'], {k: round(v,3) for k,v in d['kernels_ms'].items()})"
done
done
PHJ_TIMERS=0 timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/kn_rehearse_notimers.jsonl 2> gpurun_out/kn_rehearse.err || { echo "rehearse failed"; tail -5 gpurun_out/kn_rehearse.err; exit 5; }
cut -c1-100 gpurun_out/kn_rehearse_notimers.jsonl
echo ok
