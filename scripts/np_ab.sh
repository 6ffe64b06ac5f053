set -o pipefail
mkdir -p gpurun_out
for v in "PHJ_NP_REGION=0" "PHJ_NP_REGION=1"; do
  env $v timeout -k 10 120 python bench.py --config c4 --no-cpu-baseline --no-traffic > gpurun_out/np_ab.json 2> gpurun_out/np_ab.err || { echo "$v failed"; tail -5 gpurun_out/np_ab.err; exit 3; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/np_ab.json')); print('$v', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'])"
done
