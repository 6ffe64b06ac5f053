#!/bin/bash
# A/B the C2 bench (CFG=c4|c5: that config) over tuning environments: scripts/ab.sh "ENV=.. ENV=.." "ENV=.." ...
# One line per variant: ms/step, correctness and the S-side kernel times.
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 120 python bench.py --config ${CFG:-c2} --no-cpu-baseline --no-traffic --verbose > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { echo "variant '$v' failed rc=$?"; exit 9; }
  python - "$v" gpurun_out/ab_$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
k = d["kernels_ms"]
print(f"{sys.argv[1] or 'default':40s} {d['ms_per_step']:.3f} ms {d['correct']} " +
      " ".join(f"{n}={k[n]:.3f}" for n in k if (n.startswith("S.") or n.startswith("np.")) and not n.endswith("scan")) +
      f" build={k.get('build', 0):.3f} probe={k.get('probe', 0):.3f}")
PY
done
