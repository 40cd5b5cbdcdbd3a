"""Per-kernel summary of the LAST replayed evaluation in a rocprofv3 kernel trace of
tools/dist_replay.py (from its last gram_list_kernel launch to the end of the trace).
usage: python tools/replay_stats.py TRACE_DIR"""
import collections
import csv
import sys

tr = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
grams = [i for i, r in enumerate(tr) if "gram_list_kernel" in r["Kernel_Name"]]
ev = tr[grams[-1]:]
t0 = int(ev[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in ev)
agg = collections.defaultdict(lambda: [0, 0.0, 1e18, 0.0])
for r in ev:
    n = r["Kernel_Name"].split("(")[0][:48]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg[n]
    a[0] += 1
    a[1] += d
    a[2] = min(a[2], d)
    a[3] = max(a[3], d)
print(f"last evaluation: {(t1 - t0) / 1e6:.2f} ms, {len(ev)} kernels")
for n, (c, tot, lo, hi) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {n:48s} calls={c:6d} total={tot / 1e3:9.2f} ms avg={tot / c:8.1f} us min={lo:8.1f} max={hi:8.1f}")
