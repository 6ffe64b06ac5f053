#!/bin/bash
# GPU suite, then the C2 bench line (no PMC passes, no CPU legs) and the
# rocprof kernel stats of C2. Usage: r04_check.sh TAG [pytest-args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
TAG=${1:-chk}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread "$@" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-traffic > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench_c2.err; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_c2.json')); print('c2', round(d['ms_per_step'],4), d['correct'], d['kernels_ms'], d.get('probe_phase'))"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_c2.log 2>&1) || { echo "rocprof failed"; exit 4; }
echo ok
