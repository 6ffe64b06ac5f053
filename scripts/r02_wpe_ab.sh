#!/bin/bash
# On-chip probe over hash codes at 6 vs 8 waves per SIMD (PHJ_P1_WPE), C2, one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --steps 30 > gpurun_out/ab_cur.json 2>> gpurun_out/ab.err || { echo "$* failed"; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/ab_cur.json')); k=d['kernels_ms']; print('$*', round(d['ms_per_step'],4), d['correct'], 'S.p1', k['S.p1.scatter'], 'probe', k['probe'])"
}
run PHJ_P1_WPE=6
run PHJ_P1_WPE=8
run PHJ_P1_WPE=6
run PHJ_P1_WPE=8
echo ok
