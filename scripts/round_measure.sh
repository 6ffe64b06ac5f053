set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --verbose > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "bench failed"; tail -5 gpurun_out/bench_full.err; exit 2; }
cut -c1-400 gpurun_out/bench_full.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > $GRAFT_REPO_ROOT/gpurun_out/prof_stats.log 2>&1) || { echo "rocprof failed"; exit 3; }
tail -c 300 gpurun_out/prof_stats.log
timeout -k 10 200 python scripts/pcie_rate.py > gpurun_out/pcie.json 2> gpurun_out/pcie.err || { echo "pcie failed"; tail -3 gpurun_out/pcie.err; exit 4; }
cat gpurun_out/pcie.json
timeout -k 10 300 python scripts/rehearse_world.py > gpurun_out/rehearse.jsonl 2> gpurun_out/rehearse.err || exit 5
cut -c1-70 gpurun_out/rehearse.jsonl
