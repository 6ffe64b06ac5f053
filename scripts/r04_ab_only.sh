#!/bin/bash
# Round 4: C2 A/B only (two interleaved passes) of the environments given. Usage: r04_ab_only.sh "ENV=.." ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 100 --timeout-method thread -k "semijoin or random or preimage or zipf" > gpurun_out/abo_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/abo_pytest.log; exit 1; }
tail -1 gpurun_out/abo_pytest.log
PHJ_HT_WIDE=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 100 --timeout-method thread -k "semijoin or random or preimage or zipf or equal or extreme" > gpurun_out/abo_pytest_w.log 2>&1 || { echo "wide pytest failed"; tail -30 gpurun_out/abo_pytest_w.log; exit 1; }
tail -1 gpurun_out/abo_pytest_w.log
for r in 1 2; do
  timeout -k 10 900 bash scripts/ab.sh "$@" || exit 2
done
echo ok
