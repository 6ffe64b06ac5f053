#!/bin/bash
# r03_pipe.sh, then the W=8 / C2 kernel timelines (r03_w8trace.sh).
bash scripts/r03_pipe.sh && bash scripts/r03_w8trace.sh
