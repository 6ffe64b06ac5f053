set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PHJ_P1_PIPE=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -k "cluster_tables or adversarial or random_relations" -x -q --timeout 60 --timeout-method thread > gpurun_out/r05d_sanity.log 2>&1 || { echo "sanity failed"; tail -30 gpurun_out/r05d_sanity.log; exit 1; }
tail -1 gpurun_out/r05d_sanity.log
PHJ_P1_PIPE=1 bash scripts/round_measure.sh r05d tests=tests/test_gpu_chunk_guard.py,tests/test_gpu_parity.py,tests/test_gpu_schedules.py,tests/test_gpu_multirank.py,tests/test_gpu_fullsize.py || exit 2
bash scripts/ab.sh "" "PHJ_P1_PIPE=1" "PHJ_CL_PF=1" "PHJ_CL_PF=3" "PHJ_P1_WPC2=3" "PHJ_P1_WPC2=4" "PHJ_CL_BITS=11 PHJ_CL_CAP=8192" "PHJ_CL_BITS=11" "PHJ_CLUSTER=0" "PHJ_P1_PIPE=1" ""
