#!/bin/bash
# On-chip probe: grouped (k_probe_ht) vs streaming (k_probe_stream, PHJ_PROBE_STREAM 1/2/3 = 256/512/1024 threads).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in c2 c5; do
for env in "PHJ_P1_PIPE=0 PHJ_P1_WPC2=2" "PHJ_P1_PIPE=1 PHJ_P1_WPC2=2" "PHJ_P1_PIPE=1 PHJ_P1_WPC2=3" "PHJ_P1_PIPE=1 PHJ_P1_WPC2=4" "PHJ_P1_PIPE=0 PHJ_P1_WPC2=4" "PHJ_P1_PIPE=0 PHJ_P1_WPC2=2"; do
  tag=${cfg}_$(echo $env | tr ' =' '_-')
  env $env timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-traffic --steps 10 > gpurun_out/pd_$tag.json 2> gpurun_out/pd_$tag.err || { echo "bench $env failed"; tail -5 gpurun_out/pd_$tag.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/pd_$tag.json')); print('$cfg $env', round(d['ms_per_step'],3), d['correct'], {k: round(v,3) for k,v in d['kernels_ms'].items()})"
done
done
echo ok
