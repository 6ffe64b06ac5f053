#!/bin/bash
# GPU suite + C2/C4/C5 benches + rocprof stats + W rehearsal (r03_full.sh), then
# the PMC calibration and probe counters (r03_pmc.sh) and the W=8 / C2 timelines.
bash scripts/r03_full.sh && bash scripts/r03_pmc.sh && bash scripts/r03_w8trace.sh
