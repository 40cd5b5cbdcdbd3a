"""Per-launch list of the last full evaluation in a rocprofv3 kernel trace (queue, grid,
start/end in us, duration, workgroups) and, per queue, the time its launches leave the GPU
between each other (dispatch gaps) -- how full the bulk stream keeps the chip.
usage: python tools/launch_list.py TRACE_DIR"""
import csv
import sys
from collections import defaultdict

tr = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
inits = [i for i, r in enumerate(tr) if "init_result_kernel" in r["Kernel_Name"]]
reds = [i for i, r in enumerate(tr) if "reduce_final" in r["Kernel_Name"]]
cand = [(a, b) for a in inits for b in reds if b > a and not any(a < x < b for x in inits)]
cand = [(a, b) for a, b in cand if any("tail_kernel" in tr[i]["Kernel_Name"] for i in range(a, b))]
a, b = cand[-1]
ev = tr[a:b + 1]
t0 = int(ev[0]["Start_Timestamp"])
print("keys:", [k for k in ev[0].keys()][:30])
byq = defaultdict(list)
for r in ev:
    n = r["Kernel_Name"].split("(")[0].replace("gaplac::", "")
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
    wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or "?"
    byq[r["Queue_Id"]].append((s, e, n, grid, wg))
    print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  q{r['Queue_Id']:>2s} grid {grid:>8s} wg {wg:>4s}  {n}")
for q, lst in byq.items():
    gaps = sum(max(0.0, lst[i + 1][0] - lst[i][1]) for i in range(len(lst) - 1))
    busy = sum(e - s for s, e, *_ in lst)
    print(f"queue {q}: {len(lst)} launches, busy {busy:.1f} us, gaps between launches {gaps:.1f} us")
