"""Per-stream busy fraction in 2 ms windows and the kernels after a given time, for the last
evaluation in a rocprofv3 kernel trace (gradient / posterior schedules: which stream ends last).
usage: python tools/grad_timeline.py TRACE_DIR [--after MS] [--queue Q]"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--after", type=float, default=1e9)
ap.add_argument("--queue", default=None)
a = ap.parse_args()
tr = list(csv.DictReader(open(f"{a.trace}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
inits = [i for i, r in enumerate(tr) if "init_result_kernel" in r["Kernel_Name"]]
ev = tr[inits[-1]:]
t0 = int(ev[0]["Start_Timestamp"])
rows = [((int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6, r["Queue_Id"],
         r["Kernel_Name"].split("(")[0].replace("gaplac::", ""), int(r["Grid_Size_X"]) // 256) for r in ev]
q = defaultdict(list)
for r in rows:
    q[r[2]].append(r)
end = max(r[1] for r in rows)
print(f"end {end:.3f} ms; per queue: " + ", ".join(f"q{k} last end {max(x[1] for x in v):.3f}" for k, v in q.items()))
for w0 in range(0, int(end) + 1, 2):
    print(w0, " ".join(f"q{k}:{sum(max(0, min(e, w0 + 2) - max(s, w0)) for s, e, *_ in v) / 2:.2f}"
                       for k, v in sorted(q.items())))
for r in rows:
    if r[0] > a.after and (a.queue is None or r[2] == a.queue):
        print(f"{r[0]:.3f} {r[1]:.3f} {(r[1] - r[0]) * 1e3:.0f}us q{r[2]} {r[3]} wg={r[4]}")
