#!/bin/bash
# Round 4 checkpoint (usage: r04_full.sh TAG): whole GPU suite, then the C2 bench line (traffic + CPU baseline), C4/C5,
# rocprof kernel stats of C2, and the W=1..8 rehearsal.
set -o pipefail
TAG=${1:-r04}
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 500 python bench.py --verbose > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench_c2.err; exit 2; }
cut -c1-1500 gpurun_out/${TAG}_bench_c2.json
for c in c4 c5; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/${TAG}_bench_$c.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_$c.json')); print('$c', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'], d['roofline'])"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_c2.log 2>&1) || { echo "rocprof failed"; exit 4; }
timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/${TAG}_rehearse.jsonl 2> gpurun_out/${TAG}_rehearse.err || { echo "rehearse failed"; tail -5 gpurun_out/${TAG}_rehearse.err; exit 5; }
cut -c1-120 gpurun_out/${TAG}_rehearse.jsonl
echo ok
