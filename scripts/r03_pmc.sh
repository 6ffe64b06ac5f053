#!/bin/bash
# Counter calibration on known byte counts (scripts/pmc_calib.hip) and the
# on-chip probe's and NoPartitioning probe's L2 / memory-side counters at s=1.05 (C2, C4) and s=1.25 (C5).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/calib
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters_list.txt 2>&1) || echo "list failed"
grep -o "TCC_EA0_RD[A-Z0-9_]*\|TCC_[A-Z]*HIT[A-Z_]*\|TCC_REQ\|TCP_TCC_[A-Z_]*REQ[A-Z_]*" gpurun_out/counters_list.txt | sort -u | tr '\n' ' '; echo
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "TCC_EA0_RDREQ_32B_sum TCC_REQ_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/calib/p$i -o run -- $GRAFT_REPO_ROOT/build/pmc_calib > $GRAFT_REPO_ROOT/gpurun_out/calib/p$i.log 2>&1) || { echo "calib pass $i ($grp) failed"; tail -3 gpurun_out/calib/p$i.log; }
done
python - <<'PY'
import csv, glob, json
out = {}
for f in sorted(glob.glob("gpurun_out/calib/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = f"{int(r['Dispatch_Id']):02d} {r['Kernel_Name'][:22]}"
        out.setdefault(k, {})
        out[k][r["Counter_Name"]] = out[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(out): print(k, json.dumps(out[k]))
json.dump(out, open("gpurun_out/calib.json", "w"), indent=1)
PY
for cfg in c2 c5 c4; do
timeout -k 10 400 python scripts/pmc_kernel.py --config $cfg --kernel "k_probe_ht|k_scatter_chunked|k_np_probe_ct" \
  --group FETCH_SIZE --group WRITE_SIZE \
  --group TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum \
  --group TCC_EA0_RDREQ_32B_sum,TCC_REQ_sum \
  --group TCP_TCC_READ_REQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum \
  > gpurun_out/probe_pmc_$cfg.jsonl 2> gpurun_out/probe_pmc_$cfg.err || { echo "pmc $cfg failed"; tail -20 gpurun_out/probe_pmc_$cfg.err; exit 1; }
cut -c1-1500 gpurun_out/probe_pmc_$cfg.jsonl
done
echo ok
