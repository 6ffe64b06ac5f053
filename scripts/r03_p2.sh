#!/bin/bash
# R's pass 2 in one launch (k_ht_p2) + closed-form table slots + S-first member step:
# GPU suite, C2/C4/C5 A/B against the three-kernel pass 2, W rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/p2_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/p2_pytest.log; exit 1; }
tail -2 gpurun_out/p2_pytest.log
for cfg in c2 c5 c4; do
for env in "PHJ_HT_P2=0" "PHJ_HT_P2=1" "PHJ_HT_P2=0" "PHJ_HT_P2=1"; do
  tag=${cfg}_$(echo $env | tr ' =' '_-')
  env $env timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-traffic --steps 10 > gpurun_out/p2_$tag.json 2> gpurun_out/p2_$tag.err || { echo "bench $env failed"; tail -5 gpurun_out/p2_$tag.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/p2_$tag.json')); print('$cfg $env', round(d['ms_per_step'],3), d['correct'], {k: round(v,3) for k,v in d['kernels_ms'].items()})"
done
done
for env in "PHJ_HT_P2=0" "PHJ_HT_P2=1"; do
  env $env timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/p2_rehearse_$env.jsonl 2> gpurun_out/p2_rehearse.err || { echo "rehearse failed"; tail -5 gpurun_out/p2_rehearse.err; exit 5; }
  echo $env; cut -c1-100 gpurun_out/p2_rehearse_$env.jsonl
done
bash scripts/r03_w8trace.sh
echo ok
