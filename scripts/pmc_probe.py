#!/usr/bin/env python3
"""Workload for PMC passes: one calibration launch of known bytes
(k_count_range reads the 200M-tuple relation: 3.2 GB, 16 B per lane) and
`--steps` radix joins on the C2 workload."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--config", default="c2", choices=["c2", "c4", "c5"])
ap.add_argument("--primary", type=int, default=10_000_000)
ap.add_argument("--secondary", type=int, default=200_000_000)
args = ap.parse_args()
import partitionedhashjoin_amd as phj

alpha = 1.25 if args.config == "c5" else 1.05
params = phj.nopart_params() if args.config == "c4" else phj.radix_params((8, 8))
c = phj.Context(0)
# PMC_BUILD_START: R = [start, start + |R|) (4: the bench's shifted-R check, the
# three hottest Zipf keys absent from R)
c.generate_sequential(0, args.primary, int(os.environ.get("PMC_BUILD_START", "1")))
c.generate_zipf(1, args.secondary, alpha, 1, args.primary, 20240601)
c.count_in_range(1, 1, args.primary)
for _ in range(args.steps):
    r = c.join(params)
print("matches", r.matches)
print("TIMERS " + json.dumps([t[0] for t in r.timers()]))
