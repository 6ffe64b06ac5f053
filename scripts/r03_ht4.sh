#!/bin/bash
# Local R pass 2 + staged fill; probe variants 10/14/15/16; W=8 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py > gpurun_out/ht4_pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/ht4_pytest.log; exit 1; }
tail -2 gpurun_out/ht4_pytest.log
for v in 14 17; do
  PHJ_HT_VAR=$v timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-traffic > gpurun_out/ht4_c2_v$v.json 2> gpurun_out/ht4_c2_v$v.err || { echo "bench v$v failed"; tail -5 gpurun_out/ht4_c2_v$v.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/ht4_c2_v$v.json')); print('v$v', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'])"
done
PHJ_HT_VAR=14 timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/ht4_rehearse.jsonl 2> gpurun_out/ht4_rehearse.err || { echo "rehearse failed"; tail -5 gpurun_out/ht4_rehearse.err; exit 6; }
cut -c1-420 gpurun_out/ht4_rehearse.jsonl
(cd /tmp && PHJ_HT_VAR=14 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ht4_w8 -o run -- python3 $GRAFT_REPO_ROOT/scripts/rehearse_world.py --worlds 8 --steps 10 > $GRAFT_REPO_ROOT/gpurun_out/ht4_w8.log 2>&1) || { echo "rocprof w8 failed"; tail -5 gpurun_out/ht4_w8.log; exit 4; }
python - gpurun_out/ht4_w8/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:8.2f}')
PY
echo ok
