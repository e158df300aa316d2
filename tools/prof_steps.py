#!/usr/bin/env python3
"""Per-step kernel table from a rocprofv3 kernel_trace.csv: only dispatches from the first step on (the first
`gather_kernel` -- the embedding gather that opens every training step -- marks it), so init-time work (orthogonal
QR, warm-up autotuning) is excluded; times are divided by the number of steps seen.
Usage: prof_steps.py <kernel_trace.csv> [marker_kernel]"""
import collections
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import family  # noqa: E402


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "gather_kernel"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [s for s, _, n in rows if marker in n]
    if not starts:
        print("marker not found")
        return
    t0, steps = starts[0], len(starts)
    agg = collections.defaultdict(lambda: [0, 0.0])
    for s, e, n in rows:
        if s < t0:
            continue
        name = n if n.startswith("Cijk_") or n.startswith("Custom_Cijk") else family(n)
        if name.startswith("Cijk_") or name.startswith("Custom_Cijk"):
            name = "hipBLASLt " + name.split("_MT")[1][:40] if "_MT" in name else name[:60]
        a = agg[name]
        a[0] += 1
        a[1] += (e - s) / 1e6
    wall = (rows[-1][1] - t0) / 1e6
    total = sum(v[1] for v in agg.values())
    print(f"steps {steps}; kernel time {total / steps:.2f} ms/step; wall from first step {wall / steps:.2f} ms/step")
    print("| kernel | calls/step | ms/step | avg us | share |")
    print("|---|---|---|---|---|")
    for k, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{k}` | {c / steps:g} | {ms / steps:.2f} | {1000 * ms / c:.1f} | {100 * ms / total:.1f}% |")


if __name__ == "__main__":
    main()
