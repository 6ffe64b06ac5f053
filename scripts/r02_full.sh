#!/bin/bash
# Full GPU suite, the three bench configs, rocprof stats of C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for c in c2 c5 c4; do
  timeout -k 10 300 python bench.py --config $c --no-traffic --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/bench_$c.err; exit 2; }
  python3 -c "import json;b=json.load(open('gpurun_out/bench_$c.json'));k=b['kernels_ms'];print('$c', round(b['ms_per_step'],4), b['correct'], round(b['roofline']['frac'],3), b['roofline']['kernel'], {a:round(v,3) for a,v in k.items()})"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c2" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > "$GRAFT_REPO_ROOT/gpurun_out/prof_c2.log" 2>&1) || { echo "rocprof failed"; exit 3; }
echo ok
