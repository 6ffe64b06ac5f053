#!/bin/bash
# fill with flattened LDS inserts; R chain first (PHJ_R_FIRST) with S.p1 on every slot (PHJ_P1_WPC2=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py > gpurun_out/ht5_pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/ht5_pytest.log; exit 1; }
tail -2 gpurun_out/ht5_pytest.log
for env in "PHJ_HT_VAR=17" "PHJ_HT_VAR=17 PHJ_P1_WPC2=2" "PHJ_HT_VAR=17 PHJ_P1_WPC2=2 PHJ_R_FIRST=1"; do
  tag=$(echo $env | tr ' =' '_-')
  env $env timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-traffic > gpurun_out/ht5_$tag.json 2> gpurun_out/ht5_$tag.err || { echo "bench $env failed"; tail -5 gpurun_out/ht5_$tag.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/ht5_$tag.json')); print('$env', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'])"
done
PHJ_HT_VAR=17 timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/ht5_rehearse.jsonl 2> gpurun_out/ht5_rehearse.err || { echo "rehearse failed"; tail -5 gpurun_out/ht5_rehearse.err; exit 6; }
cut -c1-420 gpurun_out/ht5_rehearse.jsonl
(cd /tmp && PHJ_HT_VAR=17 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ht5_w8 -o run -- python3 $GRAFT_REPO_ROOT/scripts/rehearse_world.py --worlds 8 --steps 10 > $GRAFT_REPO_ROOT/gpurun_out/ht5_w8.log 2>&1) || { echo "rocprof w8 failed"; tail -5 gpurun_out/ht5_w8.log; exit 4; }
python - gpurun_out/ht5_w8/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:8.2f} min_us {float(r["MinNs"])/1e3:8.2f}')
PY
echo ok
PHJ_HT_VAR=17 timeout -k 10 600 python scripts/pmc_kernel.py --config c2 --kernel "k_probe_ht2|k_scatter_chunked|k_ht_fill" \
  --group SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVE_CYCLES \
  --group SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INST_CYCLES_VMEM \
  --group TCC_ATOMIC_sum,TCC_EA0_ATOMIC_sum,TCC_HIT_sum,TCC_MISS_sum \
  --group TA_TA_BUSY_sum,TA_ADDR_STALLED_BY_TC_CYCLES_sum,TD_TD_BUSY_sum,TD_TC_STALL_sum \
  > gpurun_out/ht5_pmc.jsonl 2> gpurun_out/ht5_pmc.err || { echo "pmc failed"; tail -20 gpurun_out/ht5_pmc.err; exit 1; }
cut -c1-3000 gpurun_out/ht5_pmc.jsonl
