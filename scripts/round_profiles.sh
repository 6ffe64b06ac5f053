#!/bin/bash
# Round-end evidence on one MI355X: bench lines (C2 with PMC traffic and CPU
# baseline; C4, C5; the N>1 exchange step on a world of one), rocprofv3
# kernel-trace stats for C2 and C4, and the per-rank W rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --verbose > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "c2 failed"; tail -5 gpurun_out/bench_c2.err; exit 1; }
for c in c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "$c failed"; tail -5 gpurun_out/bench_$c.err; exit 2; }
done
timeout -k 10 200 python bench.py --exchange --no-cpu-baseline --no-traffic > gpurun_out/bench_exchange.json 2> gpurun_out/bench_exchange.err || { echo "exchange failed"; exit 3; }
for c in c2 c4; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$c" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > "$GRAFT_REPO_ROOT/gpurun_out/prof_$c.log" 2>&1) || { echo "rocprof $c failed"; exit 4; }
done
timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/rehearse.jsonl 2> gpurun_out/rehearse.err || { echo "rehearse failed"; exit 5; }
for f in gpurun_out/bench_*.json; do echo "$f $(cut -c1-200 $f)"; done
echo ok
