#!/bin/bash
# Keys-only pass-1 workgroups per CU (PHJ_P1_WPC2 = 2x; 0 = every LDS slot, the old grid): C2 / C5 steps
# and the per-rank W rehearsal, one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --steps 30 > gpurun_out/ab_cur.json 2>> gpurun_out/ab.err || { echo "$* failed"; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/ab_cur.json')); k=d['kernels_ms']; print('$*', round(d['ms_per_step'],4), d['correct'], 'S.p1', k['S.p1.scatter'], 'R.p1.hist', k['R.p1.hist'], 'build', k['build'], 'probe', k['probe'])"
}
for v in 0 3 2 4 3 0 2; do run PHJ_P1_WPC2=$v; done

for v in 0 3; do
  PHJ_P1_WPC2=$v timeout -k 10 200 python scripts/rehearse_world.py > gpurun_out/reh_wpc$v.jsonl 2> gpurun_out/reh.err || { echo "rehearse failed"; exit 3; }
  echo "rehearse wpc2=$v"; cut -c1-60 gpurun_out/reh_wpc$v.jsonl
done
echo ok
