#!/bin/bash
# NoPartitioning over region code tables (PHJ_NP_CT=1) vs 64-B key buckets: GPU suite, C4 benches, probe PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/np_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/np_pytest.log; exit 1; }
tail -2 gpurun_out/np_pytest.log
for env in "PHJ_NP_CT=0" "PHJ_NP_CT=1" "PHJ_NP_CT=0" "PHJ_NP_CT=1"; do
  tag=$(echo $env | tr ' =' '_-')
  env $env timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 10 > gpurun_out/np_$tag.json 2> gpurun_out/np_$tag.err || { echo "bench $env failed"; tail -5 gpurun_out/np_$tag.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/np_$tag.json')); print('$env', round(d['ms_per_step'],3), d['correct'], {k: round(v,3) for k,v in d['kernels_ms'].items()}, d['roofline'].get('traffic'))"
done
echo ok
