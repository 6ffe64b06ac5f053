#!/bin/bash
# Bucketized code tables: parity subset, C2 probe variants (PHJ_HT_VAR), C5,
# W=1..8 rehearsal, probe/build PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py > gpurun_out/ht2_pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/ht2_pytest.log; exit 1; }
tail -2 gpurun_out/ht2_pytest.log
for v in 0 2 4 6 7 8 9; do
  PHJ_HT_VAR=$v timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-traffic > gpurun_out/ht2_c2_v$v.json 2> gpurun_out/ht2_c2_v$v.err || { echo "bench v$v failed"; tail -5 gpurun_out/ht2_c2_v$v.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/ht2_c2_v$v.json')); print('v$v', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'])"
done
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-traffic > gpurun_out/ht2_c5.json 2> gpurun_out/ht2_c5.err || { echo "bench c5 failed"; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/ht2_c5.json')); print('c5', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'])"
timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/ht2_rehearse.jsonl 2> gpurun_out/ht2_rehearse.err || { echo "rehearse failed"; tail -5 gpurun_out/ht2_rehearse.err; exit 6; }
cut -c1-400 gpurun_out/ht2_rehearse.jsonl
export TMPDIR=/tmp
timeout -k 10 500 python scripts/pmc_kernel.py --config c2 --kernel "k_probe_ht|k_build_ht|k_scatter_chunked" \
  --group TCC_EA0_RDREQ_128B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_32B_sum --group WRITE_SIZE \
  --group TCC_HIT_sum,TCC_MISS_sum,TCC_REQ_sum \
  --group TCP_TCC_READ_REQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum,TCP_TCC_ATOMIC_WITH_RET_REQ_sum \
  --group SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVE_CYCLES \
  > gpurun_out/ht2_pmc.jsonl 2> gpurun_out/ht2_pmc.err || { echo "pmc failed"; tail -20 gpurun_out/ht2_pmc.err; exit 1; }
cut -c1-3000 gpurun_out/ht2_pmc.jsonl
echo ok
