#!/bin/bash
# Per-rank rehearsal (W = 1, 2, 4, 8) under two pass-1 variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  env $v timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/rehearse_ab.jsonl 2> gpurun_out/rehearse_ab.err || { echo "rehearse failed"; tail -5 gpurun_out/rehearse_ab.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/rehearse_ab.jsonl'):
    d=json.loads(l); k=d['kernels_ms']
    print(d['world'], d['rank0_device_ms'], d['matches_rank0'], k)
"
done
