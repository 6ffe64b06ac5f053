#!/bin/bash
# Where k_ht_fill's time goes (C4: 32768 region tables over 10M codes; C2: 65536 tables beside S's pass 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in c4 c2; do
timeout -k 10 400 python scripts/pmc_kernel.py --config $cfg --kernel "k_ht_fill|k_ht_p2" \
  --group SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_BUSY_CYCLES,SQ_WAVES \
  --group SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_SALU,SQ_ACTIVE_INST_VALU \
  --group TCC_EA0_RDREQ_128B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_32B_sum --group WRITE_SIZE \
  --group TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum \
  > gpurun_out/fill_pmc_$cfg.jsonl 2> gpurun_out/fill_pmc_$cfg.err || { echo "pmc $cfg failed"; tail -20 gpurun_out/fill_pmc_$cfg.err; exit 1; }
cat gpurun_out/fill_pmc_$cfg.jsonl
done
echo ok
