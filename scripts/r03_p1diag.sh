#!/bin/bash
# S pass 1 (k_scatter_chunked VAR 13) with and without the chain claims (PHJ_P1_NOCLAIM: timing only),
# at 1 and 2 half-workgroups per CU, plus its PMC stall counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
for env in "PHJ_P1_WPC2=2" "PHJ_P1_WPC2=2 PHJ_P1_PLAINRANK=1" "PHJ_P1_WPC2=2 PHJ_P1_NOCLAIM=1" "PHJ_P1_WPC2=3" "PHJ_P1_WPC2=3 PHJ_P1_PLAINRANK=1" "PHJ_P1_WPC2=0" "PHJ_P1_WPC2=0 PHJ_P1_NOCLAIM=1"; do
  tag=$(echo $env | tr ' =' '_-')
  env $env timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-traffic --steps 10 > gpurun_out/p1d_$tag.json 2> gpurun_out/p1d_$tag.err || { echo "bench $env failed"; tail -5 gpurun_out/p1d_$tag.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/p1d_$tag.json')); print('$env', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'])"
done
timeout -k 10 600 python scripts/pmc_kernel.py --config c2 --kernel "k_scatter_chunked" \
  --group SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVE_CYCLES \
  --group SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INST_CYCLES_VMEM \
  --group TCC_ATOMIC_sum,TCC_EA0_ATOMIC_sum,TCC_HIT_sum,TCC_MISS_sum \
  --group TCC_EA0_RDREQ_128B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_32B_sum --group WRITE_SIZE \
  > gpurun_out/p1d_pmc.jsonl 2> gpurun_out/p1d_pmc.err || { echo "pmc failed"; tail -20 gpurun_out/p1d_pmc.err; exit 1; }
cut -c1-3000 gpurun_out/p1d_pmc.jsonl
echo ok
