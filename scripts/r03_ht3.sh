#!/bin/bash
# Probe loop restructure (k_probe_ht2, PHJ_HT_VAR 10-13) vs k_probe_ht; build kernels at W=8 under rocprof.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 10 11 12 13; do
  PHJ_HT_VAR=$v timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-traffic > gpurun_out/ht3_c2_v$v.json 2> gpurun_out/ht3_c2_v$v.err || { echo "bench v$v failed"; tail -5 gpurun_out/ht3_c2_v$v.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/ht3_c2_v$v.json')); print('v$v', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'])"
done
PHJ_HT_VAR=10 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-traffic > gpurun_out/ht3_c5_v10.json 2> gpurun_out/ht3_c5.err || { echo "bench c5 failed"; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/ht3_c5_v10.json')); print('c5 v10', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ht3_w8 -o run -- python3 $GRAFT_REPO_ROOT/scripts/rehearse_world.py --worlds 8 --steps 10 > $GRAFT_REPO_ROOT/gpurun_out/ht3_w8.log 2>&1) || { echo "rocprof w8 failed"; tail -5 gpurun_out/ht3_w8.log; exit 4; }
f=$(ls gpurun_out/ht3_w8/*kernel_stats.csv gpurun_out/ht3_w8/*/*kernel_stats.csv 2>/dev/null | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:8.2f}')
PY
echo ok
