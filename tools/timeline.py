"""Timeline of the last evaluation in a rocprofv3 kernel trace: per-kernel start/end,
stream, grid; plus a summary of where the tail steps spend time.
usage: python tools/timeline.py TRACE_DIR [nhead] [ntail]"""
import csv
import sys

d = sys.argv[1]
nh = int(sys.argv[2]) if len(sys.argv) > 2 else 12
ntl = int(sys.argv[3]) if len(sys.argv) > 3 else 24
tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
grams = [i for i, r in enumerate(tr) if "gram_kernel" in r["Kernel_Name"]]
ev = tr[grams[-1]:]
t0 = int(ev[0]["Start_Timestamp"])


def nm(r):
    n = r["Kernel_Name"]
    for key, short in (("tile_gemm_kernel<0>", "syrk"), ("tile_gemm_kernel<1>", "trsm"), ("potrf", "diag"),
                       ("gram", "gram"), ("reduce", "reduce")):
        if key in n:
            return short
    return n[:10]


rows = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Stream_Id"], nm(r),
         int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))) for r in ev]
print(f"eval span {max(r[1] for r in rows) / 1e3:.1f} us, {len(rows)} kernels")
tot = {}
for r in rows:
    tot[r[3]] = tot.get(r[3], 0) + (r[1] - r[0])
print("kernel time per name (us):", {k: round(v / 1e3, 1) for k, v in tot.items()})
for r in rows[:nh] + [None] + rows[-ntl:]:
    if r is None:
        print("...")
        continue
    print(f"{r[0] / 1e3:9.1f} {r[1] / 1e3:9.1f} dur {(r[1] - r[0]) / 1e3:7.1f} s{r[2]} {r[3]:7s} grid {r[4]}")
