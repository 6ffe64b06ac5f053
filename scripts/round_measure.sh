#!/bin/bash
# Round measurement on one MI355X (gpurun): the steps given, in order, stopping
# at the first failure. Outputs under gpurun_out/TAG_*; copy what is judged into profiles/.
#   bash scripts/round_measure.sh TAG STEP [STEP ...]
# STEP:
#   suite            whole GPU suite (pytest -m gpu)
#   tests=FILES      the GPU tests in FILES (comma-separated)
#   bench            C2 bench line with PMC traffic and the CPU baseline
#   quick            C2 bench line without traffic / CPU baseline
#   c4c5             C4 and C5 bench lines (traffic, no CPU baseline)
#   exchange         the N>1 member step on a world of one (RCCL)
#   stats            rocprofv3 --kernel-trace --stats of the C2 bench (and C4)
#   rehearse         per-rank W = 1, 2, 4, 8 rehearsal on one GPU (scripts/rehearse_world.py)
#   pmc              counter calibration + probe / pass-1 PMC passes at C2, C5, C4
#   traces           kernel timelines of a C2 step and a rehearsed W=8 member step
#   counters         rocprofv3 -L on the box (which memory-side counters exist)
#   sweep            the reference's partition-count sweep through the CLI + the rehearsed GPU-count axis (scripts/sweep.py)
set -o pipefail
TAG=${1:?usage: round_measure.sh TAG STEP...}
shift
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${TAG}
prof() {   # prof NAME ARGS...: rocprofv3 kernel-trace stats of one bench.py run
  local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/${O}_$name" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" "$@" > "$GRAFT_REPO_ROOT/${O}_$name.log" 2>&1) || { echo "rocprof $name failed"; tail -5 ${O}_$name.log; return 1; }
  find ${O}_$name -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -d, -f1-8 {} | head -12
}
for step in "$@"; do
  case $step in
    suite)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > ${O}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 ${O}_pytest.log; exit 1; }
      tail -1 ${O}_pytest.log ;;
    tests=*)
      timeout -k 10 900 python -u -m pytest $(echo ${step#tests=} | tr ',' ' ') -m gpu -x -q --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 ${O}_pytest.log; exit 1; }
      tail -1 ${O}_pytest.log ;;
    bench)
      timeout -k 10 500 python bench.py --verbose > ${O}_bench_c2.json 2> ${O}_bench_c2.err || { echo "bench failed"; tail -5 ${O}_bench_c2.err; exit 2; }
      cut -c1-1500 ${O}_bench_c2.json ;;
    quick)
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --verbose > ${O}_quick.json 2> ${O}_quick.err || { echo "bench failed"; tail -5 ${O}_quick.err; exit 2; }
      cut -c1-1200 ${O}_quick.json ;;
    c4c5)
      for c in c4 c5; do
        timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > ${O}_bench_$c.json 2> ${O}_bench_$c.err || { echo "bench $c failed"; tail -5 ${O}_bench_$c.err; exit 3; }
        python -c "import json; d=json.load(open('${O}_bench_$c.json')); print('$c', round(d['ms_per_step'],3), d['correct'], d['kernels_ms'], d['roofline'])"
      done ;;
    exchange)
      timeout -k 10 200 python bench.py --exchange --no-cpu-baseline --no-traffic > ${O}_bench_exchange.json 2> ${O}_bench_exchange.err || { echo "exchange failed"; tail -5 ${O}_bench_exchange.err; exit 4; }
      cut -c1-600 ${O}_bench_exchange.json ;;
    stats)
      prof stats_c2 --steps 20 --warmup 3 --no-cpu-baseline --no-traffic || exit 5
      prof stats_c4 --config c4 --steps 20 --warmup 3 --no-cpu-baseline --no-traffic || exit 5 ;;
    rehearse)
      timeout -k 10 300 python scripts/rehearse_world.py > ${O}_rehearse.jsonl 2> ${O}_rehearse.err || { echo "rehearse failed"; tail -5 ${O}_rehearse.err; exit 6; }
      cut -c1-160 ${O}_rehearse.jsonl ;;
    pmc)
      # per kernel (pmc_kernel.py keeps the last matching dispatch): S's pass 1, the probe
      # (S's pass 1 is the KPF=2 form; R's the KPF=1 form of the same kernel; the LDS join's
      # main kernel, not its big-cluster companion)
      for kr in "c2:k_chunk_codes_pipe<.*, 2>\(" "c2:k_cluster_probe<" "c5:k_cluster_probe<" "c4:k_np_probe_ct"; do
        cfg=${kr%%:*}; k=${kr#*:}; kf=$(echo "$k" | tr -c 'a-z0-9_' '_')
        timeout -k 10 400 python scripts/pmc_kernel.py --config $cfg --kernel "$k" \
          --group FETCH_SIZE --group WRITE_SIZE \
          --group TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum \
          --group TCC_EA0_RDREQ_32B_sum,TCC_REQ_sum \
          --group TCC_EA0_RDREQ_DRAM_sum,TCC_EA0_RDREQ_sum \
          --group SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_BUSY_CYCLES,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_WAIT_INST_ANY,SQ_INSTS_SALU \
          --group SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_LDS_BANK_CONFLICT,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_ANY \
          > ${O}_pmc_${cfg}_$kf.jsonl 2> ${O}_pmc_${cfg}_$kf.err || { echo "pmc $cfg $k failed"; tail -20 ${O}_pmc_${cfg}_$kf.err; exit 7; }
        cut -c1-1500 ${O}_pmc_${cfg}_$kf.jsonl
      done ;;
    traces)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/${O}_w8trace" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/rehearse_world.py" --worlds 8 --steps 5 > "$GRAFT_REPO_ROOT/${O}_w8trace.log" 2>&1) || { echo "rocprof w8 failed"; tail -5 ${O}_w8trace.log; exit 8; }
      python3 scripts/trace_summary.py ${O}_w8trace --step-kernel "k_cluster_probe<" > ${O}_w8trace.txt 2>&1
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/${O}_c2trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > "$GRAFT_REPO_ROOT/${O}_c2trace.log" 2>&1) || { echo "rocprof c2 failed"; tail -5 ${O}_c2trace.log; exit 8; }
      python3 scripts/trace_summary.py ${O}_c2trace --step-kernel "k_cluster_probe<" > ${O}_c2trace.txt 2>&1
      tail -30 ${O}_c2trace.txt ;;
    counters)
      # the counters this box's rocprofv3 offers (a MALL / data-fabric split for C4?)
      timeout -k 10 120 rocprofv3 -L > ${O}_counters.txt 2>&1 || { echo "rocprofv3 -L failed"; tail -5 ${O}_counters.txt; exit 11; }
      grep -i -E "mall|dram|_df|gmi|ea0_rd" ${O}_counters.txt | head -30 ;;
    sweep)
      timeout -k 10 900 python scripts/sweep.py --skew 1.05 1.25 --rehearse-worlds 1 2 4 8 --out ${O}_sweep_cli > ${O}_sweep.log 2>&1 || { echo "sweep failed"; tail -5 ${O}_sweep.log; exit 9; }
      tail -24 ${O}_sweep.log ;;
    *) echo "unknown step $step"; exit 10 ;;
  esac
done
echo ok
