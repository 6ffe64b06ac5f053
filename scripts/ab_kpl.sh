set -o pipefail
for v in "PHJ_FUSED_KPL=4" "PHJ_FUSED_KPL=2"; do
  env $v timeout -k 10 200 python scripts/rehearse_world.py --worlds 1 8 > gpurun_out/kpl.jsonl 2> gpurun_out/kpl.err || { echo "$v failed"; tail -5 gpurun_out/kpl.err; exit 3; }
  python -c "
import json
for l in open('gpurun_out/kpl.jsonl'):
    d=json.loads(l); k=d['kernels_ms']; print('$v', d['world'], d['ms_per_step'], k['build'], k['probe'])"
done
