#!/usr/bin/env python3
"""Materialised join (phj_join_materialize) on the C2 / C4 workloads: device
time per join and per kernel, and a check of a slice of the rows
(Sequential R: payloadA = id - 1; Zipf S: payloadB = the probe row, unique).
One JSON line per algorithm."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import partitionedhashjoin_amd as phj

nR, nS, steps = 10_000_000, 200_000_000, 5
c = phj.Context(0)
c.generate_sequential(0, nR, 1)
c.generate_zipf(1, nS, 1.05, 1, nR, 20240601)
for name, p in (("radix-8+8-murmur3", phj.radix_params((8, 8), hash=phj.HASH_MURMUR3)),
                ("nopartitioning-xxh3", phj.nopart_params())):
    count = c.join(p).matches
    c.join_materialize(p)   # warm-up (allocations)
    t0 = time.perf_counter()
    acc = {}
    for _ in range(steps):
        r = c.join_materialize(p)
        for k, ms, nb in r.timers():
            acc[k] = acc.get(k, 0.0) + ms
    wall = (time.perf_counter() - t0) / steps * 1e3
    rows = c.joined(1_000_000)
    ok = (r.matches == count and np.array_equal(rows[:, 1], rows[:, 0] - 1)
          and len(np.unique(rows[:, 2])) == len(rows))
    print(json.dumps({"join": name, "rows": int(r.matches), "count_join": int(count), "rows_ok": bool(ok),
                      "ms_per_join": round(wall, 3), "total_ms": round(r.total_ms, 3),
                      "row_bytes": int(r.matches) * 24,
                      "kernels_ms": {k: round(v / steps, 4) for k, v in sorted(acc.items())}}), flush=True)
