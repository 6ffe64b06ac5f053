#!/bin/bash
# Code-table join (phj_table.h): parity subset, then C2/C5 bench, W=1..8 rehearsal,
# then the counter calibration + probe PMC (scripts/r03_pmc.sh's passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py > gpurun_out/ht_pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/ht_pytest.log; exit 1; }
tail -2 gpurun_out/ht_pytest.log
for c in c2 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-traffic > gpurun_out/ht_$c.json 2> gpurun_out/ht_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/ht_$c.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/ht_$c.json')); print('$c', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'])"
done
timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/ht_rehearse.jsonl 2> gpurun_out/ht_rehearse.err || { echo "rehearse failed"; tail -5 gpurun_out/ht_rehearse.err; exit 6; }
cut -c1-400 gpurun_out/ht_rehearse.jsonl
bash scripts/r03_pmc.sh
