#!/bin/bash
# Knobs beside the 1.5-workgroups-per-CU pass 1: aux stream priority, tiles per shard, C2, one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --steps 30 > gpurun_out/ab_cur.json 2>> gpurun_out/ab.err || { echo "$* failed"; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/ab_cur.json')); k=d['kernels_ms']; print('$*', round(d['ms_per_step'],4), d['correct'], 'S.p1', k['S.p1.scatter'], 'R.p2.scatter', k['R.p2.scatter'], 'build', k['build'], 'probe', k['probe'])"
}
run X=0
run PHJ_AUX_PRIO=1
run PHJ_P1_KO_TPS=512
run PHJ_P1_KO_TPS=2048
run PHJ_NT_LOAD=0
run PHJ_AUX_PRIO=1
run X=0
echo ok
