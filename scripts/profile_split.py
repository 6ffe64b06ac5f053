"""Split a rocprofv3 kernel trace into per-relation kernel averages.

The radix join launches the same kernel instantiations for R (10M) and S
(200M); rocprofv3's --stats averages them together. For kernels launched
an even number of times per step, the larger half of the durations is S.
Usage: python scripts/profile_split.py <run_kernel_trace.csv> [steps]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    d = collections.defaultdict(list)
    for r in rows:
        d[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    calls = collections.Counter(len(v) for v in d.values())
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else calls.most_common(1)[0][0]
    print(f"# {path}: {len(rows)} dispatches, {steps} launches per kernel per relation")
    print(f"{'kernel':70s} {'calls':>6s} {'avg_ms':>9s} {'S_avg_ms':>9s} {'R_avg_ms':>9s}")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        avg = sum(v) / len(v) / 1e6
        if len(v) == 2 * steps:
            s = sorted(v)
            print(f"{k[:70]:70s} {len(v):6d} {avg:9.4f} {sum(s[steps:]) / steps / 1e6:9.4f} "
                  f"{sum(s[:steps]) / steps / 1e6:9.4f}")
        else:
            print(f"{k[:70]:70s} {len(v):6d} {avg:9.4f}")


if __name__ == "__main__":
    main()
