#!/bin/bash
# Packed 6-B build segments (PHJ_CODE_PACK): GPU suite, C2/C5 and rehearsal A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pack_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pack_pytest.log; exit 1; }
tail -2 gpurun_out/pack_pytest.log
for cfg in c2 c5; do
for env in "PHJ_CODE_PACK=0" "PHJ_CODE_PACK=1" "PHJ_CODE_PACK=0" "PHJ_CODE_PACK=1"; do
  tag=${cfg}_$(echo $env | tr ' =' '_-')
  env $env timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-traffic --steps 10 > gpurun_out/pk_$tag.json 2> gpurun_out/pk_$tag.err || { echo "bench $env failed"; tail -5 gpurun_out/pk_$tag.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/pk_$tag.json')); print('$cfg $env', round(d['ms_per_step'],3), d['correct'], {k: round(v,3) for k,v in d['kernels_ms'].items()})"
done
done
for env in "PHJ_CODE_PACK=0" "PHJ_CODE_PACK=1" "PHJ_CODE_PACK=0" "PHJ_CODE_PACK=1"; do
  env $env timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/pk_rehearse_$env.jsonl 2> gpurun_out/pk_rehearse.err || { echo "rehearse failed"; tail -5 gpurun_out/pk_rehearse.err; exit 5; }
  echo $env; cut -c1-60 gpurun_out/pk_rehearse_$env.jsonl
done
echo ok
