#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel over all dispatches found under a directory tree.
Usage: pmc_summary.py <dir>"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    root = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = re.sub(r"\(.*", "", row["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")[-60:]
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, ctr in sorted(acc.items()):
        print(name)
        for c, v in sorted(ctr.items()):
            print(f"  {c:28s} {sum(v) / len(v):16.0f}   (n={len(v)})")
        c = {k: sum(v) / len(v) for k, v in ctr.items()}
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            w = c["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU"):
                if k in c:
                    print(f"  {k + ' / WAVE_CYCLES':40s} {c[k] / w:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "SQ_BUSY_CYCLES" in c and c["SQ_BUSY_CYCLES"]:
            print(f"  {'MFMA busy / (SQ busy * 4 SIMD)':40s} {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * c['SQ_BUSY_CYCLES']):.3f}")


if __name__ == "__main__":
    main()
