#!/bin/bash
# Rehearsal per world size with the S pass-1 grid at 1/2, 1 and 1.5 workgroups per CU (PHJ_P1_WPC2=1/2/3).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for env in "PHJ_P1_WPC2=2" "PHJ_P1_WPC2=1" "PHJ_P1_WPC2=3" "PHJ_P1_WPC2=2" "PHJ_P1_WPC2=1" "PHJ_P1_WPC2=3"; do
  env $env timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/ww_$env.jsonl 2> gpurun_out/ww.err || { echo "rehearse failed"; tail -5 gpurun_out/ww.err; exit 5; }
  echo $env; python3 -c "
import json
for l in open('gpurun_out/ww_$env.jsonl'):
    d=json.loads(l); k=d['kernels_ms']; print(d['world'], d['rank0_device_ms'], k['S.p1.scatter'], k['R.p1.hist'], k['R.p2.scatter'], k['build'], k['exchange'], k['probe'])"
done
echo ok
