#!/bin/bash
# A/B of env variants on the C2 bench (and optionally other configs): VARIANTS="A B ..." (commas = spaces)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for v in $VARIANTS; do
  env ${v//,/ } timeout -k 10 200 python bench.py $BENCH_ARGS --no-traffic --no-cpu-baseline --steps 20 > gpurun_out/b.json 2> gpurun_out/b.err || { echo "bench failed $v"; tail -5 gpurun_out/b.err; exit 2; }
  python3 -c "import json;b=json.load(open('gpurun_out/b.json'));k=b['kernels_ms'];print('$v', round(b['ms_per_step'],4), b['correct'], {a:round(v,3) for a,v in k.items() if not a.startswith('R.')})"
done
echo ok
