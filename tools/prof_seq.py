#!/usr/bin/env python3
"""GEMM dispatch sequence of ONE training step from a rocprofv3 kernel_trace.csv (the step between the last two
`gather_kernel` markers): index, kernel, grid, duration -- two runs of the same step (e.g. OBST_GEMM_LT=0 / 1) align
call by call. Usage: prof_seq.py <kernel_trace.csv> [substring filter, default gemm]"""
import csv
import sys


def main():
    path = sys.argv[1]
    keys = (sys.argv[2] if len(sys.argv) > 2 else "gemm,Cijk").split(",")
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("LDS_Block_Size", "")))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "gather_kernel" in r[2]]
    if len(marks) < 2:
        print("need two step markers")
        return
    i0, i1 = marks[-2], marks[-1]
    k = 0
    for s, e, n, g, lds in rows[i0:i1]:
        if any(x in n for x in keys):
            short = n.split("(")[0][:48]
            print(f"{k:4d} {short:48s} grid {g:>9s} lds {lds:>6s} {(e - s) / 1e3:9.1f} us")
            k += 1


if __name__ == "__main__":
    main()
