#!/bin/bash
# A/B the C2 bench over library builds on one box: scripts/ab_lib.sh LIB1 LIB2 ...
# (each LIB a libphj_hip.so built beforehand in-tree, e.g. from another commit or with
#  measurement-only compile flags: `make prof-lib` -> build/libphj_prof.so, the phase-clock
#  forms of S's pass 1 and of the LDS join (-DPHJ_P1_PROF=1 -DPHJ_CL_PROF=1, stderr per join);
#  `make build/libphj_res1.so HIPDEFS=-DPHJ_PIPE_RES=1`-style variants the same way; PHJ_LIB selects it)
set -o pipefail
mkdir -p gpurun_out
i=0
for lib in "$@"; do
  i=$((i+1))
  PHJ_LIB=$lib timeout -k 10 150 python bench.py --no-cpu-baseline --no-traffic --verbose > gpurun_out/abl_$i.json 2> gpurun_out/abl_$i.err || { echo "$lib failed"; tail -5 gpurun_out/abl_$i.err; exit 9; }
  python -c "import json,sys; d=json.load(open('gpurun_out/abl_$i.json')); k=d['kernels_ms']; print('$lib', round(d['ms_per_step'],3), d['correct'], {n: round(v,3) for n,v in k.items()})"
done
