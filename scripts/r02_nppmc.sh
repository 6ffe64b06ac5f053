#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 900 python scripts/pmc_kernel.py --config c4 --kernel "np_probe" \
  --group TCP_TOTAL_CACHE_ACCESSES_sum,TCP_TCC_READ_REQ_sum,TCP_UTCL1_TRANSLATION_MISS_sum,TCP_PENDING_STALL_CYCLES_sum \
  --group TA_TA_BUSY_sum,TA_ADDR_STALLED_BY_TC_CYCLES_sum,TD_TD_BUSY_sum,TD_TC_STALL_sum,GRBM_GUI_ACTIVE \
  --group TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum,TCC_TAG_STALL_sum \
  --group SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_INSTS_VMEM_RD,SQ_INST_LEVEL_VMEM,SQ_ACCUM_PREV_HIRES,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT \
  --variant PHJ_NP_HOT=0,PHJ_NP_COOP=0 --variant PHJ_NP_HOT=0,PHJ_NP_COOP=1 --variant PHJ_NP_HOT=0,PHJ_NP_DIAG=2 --variant PHJ_NP_HOT=0,PHJ_NP_DIAG=1 --variant PHJ_NP_HOT=1 \
  > gpurun_out/np_pmc.jsonl 2> gpurun_out/np_pmc.err || { echo failed; tail -20 gpurun_out/np_pmc.err; exit 1; }
cat gpurun_out/np_pmc.jsonl | cut -c1-1500
