"""List the kernels of the last evaluation in a rocprofv3 trace that start inside a time
window (us from the evaluation's first Gram launch).
usage: python tools/window.py TRACE_DIR T0_US T1_US"""
import csv
import sys

tr = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
grams = [i for i, r in enumerate(tr) if "gram_kernel" in r["Kernel_Name"]]
ev = tr[grams[-1] - 1:]
t0 = int(ev[0]["Start_Timestamp"])
lo, hi = float(sys.argv[2]), float(sys.argv[3])


def nm(n):
    for k, s in (("tile_syrk", "SYRK"), ("trsm", "trsm"), ("potrf", "diag"), ("gram", "gram"), ("col_update", "colu"),
                 ("quad_bulk", "quad"), ("reduce", "red")):
        if k in n:
            return s
    return n[:8]


for r in ev:
    a = (int(r["Start_Timestamp"]) - t0) / 1e3
    b = (int(r["End_Timestamp"]) - t0) / 1e3
    if lo <= a <= hi:
        g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        print(f"{a:9.1f} {b:9.1f} {b - a:7.1f} {nm(r['Kernel_Name'])} grid {g}")
