"""Per-step view of the panel chain beside the bulk updates, from a rocprofv3 kernel trace.
usage: python tools/steps.py TRACE_DIR [step ...]"""
import csv
import sys

tr = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
grams = [i for i, r in enumerate(tr) if "gram_kernel" in r["Kernel_Name"]]
ev = tr[grams[-1] - 1:]
t0 = int(ev[0]["Start_Timestamp"])


def nm(r):
    n = r["Kernel_Name"]
    for k, s in (("tile_syrk", "SYRK"), ("trsm", "trsm"), ("potrf", "diag"), ("gram", "gram"), ("col_update", "colu"),
                 ("quad_bulk", "quad"), ("reduce", "red")):
        if k in n:
            return s
    return n[:8]


rows = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, nm(r),
         int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])) for r in ev]
syrks = [r for r in rows if r[2] == "SYRK"]
end = max(r[1] for r in rows)
print(f"eval {end / 1e3:.1f} us, bulk launches {len(syrks)}")
steps = [int(x) for x in sys.argv[2:]] or [0, 8, 14, 18]
for k in steps:
    if k >= len(syrks):
        continue
    a, b = syrks[k][0], syrks[k][1]
    print(f"--- SYRK {k}: {a / 1e3:.1f}-{b / 1e3:.1f} dur {(b - a) / 1e3:.1f} grid {syrks[k][3]}")
    for r in rows:
        if r[2] != "SYRK" and a - 5000 <= r[0] < b + 5000:
            print(f"   {r[0] / 1e3:9.1f} {r[1] / 1e3:9.1f} {(r[1] - r[0]) / 1e3:7.1f} {r[2]} grid {r[3]}")
