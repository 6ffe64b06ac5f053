#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
KREGEX=${KREGEX:-k_probe_p1} timeout -k 10 600 python scripts/pmc_kernel.py --config c2 --kernel "$KREGEX" \
  --group TCP_TOTAL_CACHE_ACCESSES_sum,TCP_TCC_READ_REQ_sum,TCP_PENDING_STALL_CYCLES_sum,TCP_TCR_TCP_STALL_CYCLES_sum \
  --group TA_TA_BUSY_sum,TA_ADDR_STALLED_BY_TC_CYCLES_sum,TD_TD_BUSY_sum,TD_TC_STALL_sum,GRBM_GUI_ACTIVE \
  --group TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum \
  --group SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_INSTS_VMEM_RD,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS \
  --group SQ_INSTS_SALU,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INST_CYCLES_VMEM,SQ_LDS_IDX_ACTIVE,SQ_WAVE_CYCLES \
  --variant PHJ_P2PROBE=1 \
  > gpurun_out/p1_pmc.jsonl 2> gpurun_out/p1_pmc.err || { echo failed; tail -20 gpurun_out/p1_pmc.err; exit 1; }
cat gpurun_out/p1_pmc.jsonl | cut -c1-2500
