#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel average duration and,
for the last bench step, the device timeline (start offsets and gaps).

  python scripts/trace_summary.py <dir with *_kernel_trace.csv> [--step-kernel NAME]
(the step ends at the last launch whose name contains NAME, default k_probe,
and the launches right behind it; "k_cluster_probe<" is the LDS join's probe)
  --steps: also every step between consecutive matches, one line each: the
  launches as name:gap-before+duration (us), and the span from one step's
  last launch to the next step's (the timed loop's steps, host gaps included)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    stats = defaultdict(list)
    for s, e, n in rows:
        stats[n.split("(")[0][:90]].append((e - s) / 1e3)
    print(f"{'kernel':92s} {'calls':>6s} {'avg_us':>9s} {'total_us':>10s}")
    for n, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n:92s} {len(v):6d} {sum(v) / len(v):9.1f} {sum(v):10.1f}")
    # timeline of the last step: from the last k_hist launch preceding the last k_probe
    key = sys.argv[sys.argv.index("--step-kernel") + 1] if "--step-kernel" in sys.argv else "k_probe"
    probes = [i for i, r in enumerate(rows) if key in r[2]]
    if probes:
        last = probes[-1]
        first = last
        while first > 0 and rows[first - 1][0] > rows[last][0] - 20_000_000 and key not in rows[first - 1][2]:
            first -= 1
        t0 = rows[first][0]
        print("\nlast step timeline (us): start  dur  gap-before  kernel")
        prev_end = None
        # (kernels after the last match in the same step, e.g. k_cluster_probe_big, belong to it)
        while last + 1 < len(rows) and rows[last + 1][0] < rows[last][1] + 200_000 and key not in rows[last + 1][2]:
            last += 1
        for s, e, n in rows[first:last + 1]:
            gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap:8.1f}  {n.split('(')[0][:70]}")
            prev_end = e if prev_end is None else max(prev_end, e)
        print(f"step span: {(rows[last][1] - t0) / 1e3:.1f} us")
    if "--steps" in sys.argv and probes:
        ends = []   # each step's last launch: the match and the launches right behind it
        for i in probes:
            j = i
            while j + 1 < len(rows) and rows[j + 1][0] < rows[j][1] + 200_000 and key not in rows[j + 1][2] \
                    and rows[j + 1][0] - rows[j][1] < 2_000:
                j += 1
            ends.append(j)
        print("\nsteps (us): span from the previous step's last launch; name:gap+duration")
        for a, b in zip(ends[:-1], ends[1:]):
            seq, prev = [], rows[a][1]
            for s_, e_, n in rows[a + 1:b + 1]:
                short = n.split("(")[0].replace("void ", "").replace("phj::", "").replace("__amd_rocclr_", "")[:28]
                seq.append(f"{short}:{(s_ - prev) / 1e3:.1f}+{(e_ - s_) / 1e3:.1f}")
                prev = e_
            print(f"{(rows[b][1] - rows[a][1]) / 1e3:9.1f}  " + " | ".join(seq))


if __name__ == "__main__":
    main()
