#!/bin/bash
# A/B the per-rank W rehearsal over tuning environments: scripts/ab_rehearse.sh "8" "ENV=.." "ENV=.." ...
set -o pipefail
mkdir -p gpurun_out
worlds=$1; shift
for v in "$@"; do
  env $v timeout -k 10 200 python scripts/rehearse_world.py --worlds $worlds > gpurun_out/abr.jsonl 2> gpurun_out/abr.err || { echo "$v failed"; tail -5 gpurun_out/abr.err; exit 3; }
  python - "$v" <<'PY'
import json, sys
for l in open("gpurun_out/abr.jsonl"):
    d = json.loads(l); k = d["kernels_ms"]
    print(f"{sys.argv[1] or 'default':24s} W={d['world']} {d['ms_per_step']:.4f} ms " +
          " ".join(f"{n}={k[n]:.3f}" for n in k if n.startswith("S.")))
PY
done
