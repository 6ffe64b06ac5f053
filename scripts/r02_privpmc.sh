#!/bin/bash
# Private vs shared chains in pass 1: A/B and the write traffic of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
bash scripts/ab.sh "PHJ_P1_PRIV=0" "" "PHJ_P1_PRIV=0" "" || exit 1
timeout -k 10 600 python scripts/pmc_kernel.py --config c2 --kernel "k_scatter_(priv|chunked)" \
  --group FETCH_SIZE --group WRITE_SIZE --group TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum \
  --variant PHJ_P1_PRIV=0 --variant PHJ_P1_PRIV=1 \
  > gpurun_out/priv_pmc.jsonl 2> gpurun_out/priv_pmc.err || { echo failed; tail -20 gpurun_out/priv_pmc.err; exit 1; }
cat gpurun_out/priv_pmc.jsonl | cut -c1-1500
