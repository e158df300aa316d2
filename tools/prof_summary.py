#!/usr/bin/env python3
"""Condense a rocprofv3 kernel_stats.csv into a short table (per-call and total ms, share), grouped by kernel
family. Usage: prof_summary.py <kernel_stats.csv> [steps]"""
import csv
import re
import sys


def family(name: str) -> str:
    if name.startswith("Cijk_"):
        return "hipBLASLt/rocBLAS GEMM (torch, init-time QR)"
    if "rocsolver" in name or "rocblas" in name:
        return "rocSOLVER/rocBLAS (init-time QR)"
    m = re.search(r"(\w+_kernel)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:80]


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    rows = list(csv.DictReader(open(path)))
    agg = {}
    for r in rows:
        f = family(r["Name"])
        a = agg.setdefault(f, [0, 0.0])
        a[0] += int(r["Calls"])
        a[1] += float(r["TotalDurationNs"]) / 1e6
    total = sum(v[1] for v in agg.values())
    print(f"| kernel | calls | total ms | ms/step (/{steps:g}) | avg us | share |")
    print("|---|---|---|---|---|---|")
    for f, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{f}` | {c} | {ms:.1f} | {ms / steps:.2f} | {1000 * ms / max(c, 1):.1f} | {100 * ms / total:.1f}% |")


if __name__ == "__main__":
    main()
