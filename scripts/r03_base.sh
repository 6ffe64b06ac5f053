#!/bin/bash
# Round-3 starting point on one box: C2/C4/C5 bench lines + W=1..8 rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for c in c2 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-traffic > gpurun_out/base_$c.json 2> gpurun_out/base_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/base_$c.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/base_$c.json')); print('$c', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'])"
done
timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/base_rehearse.jsonl 2> gpurun_out/base_rehearse.err || { echo "rehearse failed"; tail -5 gpurun_out/base_rehearse.err; exit 6; }
cut -c1-200 gpurun_out/base_rehearse.jsonl
echo ok
