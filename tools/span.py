"""Where an evaluation's time goes, from a rocprofv3 kernel trace of repeated evaluations
(the last one is analysed): the bulk updates (tile_syrk / quad_bulk, stream s_main) against
the gaps between them, which are waits for the panel chain, plus the head (before the
first bulk update) and the tail (after the last).
usage: python tools/span.py TRACE_DIR"""
import csv
import sys

tr = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last evaluation with bulk updates: from its first Gram launch to its reduction
# (the bench's later extras, e.g. the N = 4096 line, run after it)
last_bulk = max(i for i, r in enumerate(tr) if "tile_syrk" in r["Kernel_Name"])
g0 = max(i for i in range(last_bulk) if "gram_kernel" in tr[i]["Kernel_Name"])
while g0 > 0 and "gram_kernel" in tr[g0 - 1]["Kernel_Name"]:
    g0 -= 1
g1 = min(i for i in range(last_bulk, len(tr)) if "reduce_final" in tr[i]["Kernel_Name"])
ev = tr[g0:g1 + 1]
t0 = int(ev[0]["Start_Timestamp"])
end = max(int(r["End_Timestamp"]) for r in ev) - t0
bulk = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, "quad" if "quad_bulk" in r["Kernel_Name"] else "syrk")
        for r in ev if "tile_syrk" in r["Kernel_Name"]]
head = bulk[0][0]
tail = end - bulk[-1][1]
busy = sum(b - a for a, b, _ in bulk)
gaps = [(i, bulk[i + 1][0] - bulk[i][1]) for i in range(len(bulk) - 1)]
print(f"eval {end / 1e3:.2f} ms: head {head / 1e3:.3f} ms, bulk busy {busy / 1e3:.2f} ms over {len(bulk)} launches, "
      f"gaps {sum(max(g, 0) for _, g in gaps) / 1e3:.3f} ms, tail {tail / 1e3:.3f} ms")
print("step  kind   bulk_ms   gap_before_next_us")
for i, (a, b, k) in enumerate(bulk):
    g = gaps[i][1] if i < len(gaps) else 0
    print(f"{i:4d}  {k}  {(b - a) / 1e3:8.3f}   {g / 1e3:8.1f}")
