#!/bin/bash
# S pass-1 persistent grid (PHJ_P1_SLOTS per shard; default 48 = 3 per CU at 16 shards) and the
# aux stream's priority: does leaving CU slots free let R's chain overlap S's pass 1? C2, one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --steps 30 > gpurun_out/ab_cur.json 2>> gpurun_out/ab.err || { echo "$* failed"; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/ab_cur.json')); k=d['kernels_ms']; print('$*', round(d['ms_per_step'],4), d['correct'], 'S.p1', k['S.p1.scatter'], 'R.p1.hist', k['R.p1.hist'], 'build', k['build'], 'probe', k['probe'])"
}
run X=0
run PHJ_P1_SLOTS=32
run PHJ_P1_SLOTS=40
run PHJ_AUX_PRIO=1
run PHJ_AUX_PRIO=1 PHJ_P1_SLOTS=32
run PHJ_P1_SLOTS=24
run X=0
echo ok
