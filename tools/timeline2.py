"""Per-kernel timeline of the last full evaluation in a rocprofv3 kernel trace: every
dispatch (relative start / end in us, queue, short name), then per-name totals and the
time the bulk kernels (tile_syrk / tile_band / quad_bulk) leave the GPU without a bulk
workgroup (the chain-bound part of the evaluation).
usage: python tools/timeline2.py TRACE_DIR [--list]"""
import csv
import sys
from collections import defaultdict

tr = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
inits = [i for i, r in enumerate(tr) if "init_result_kernel" in r["Kernel_Name"]]
reds = [i for i, r in enumerate(tr) if "reduce_final" in r["Kernel_Name"]]
# the last evaluation that contains a tail kernel (the bench's headline mode)
cand = [(a, b) for a in inits for b in reds if b > a and not any(a < x < b for x in inits)]
cand = [(a, b) for a, b in cand if any("tail_kernel" in tr[i]["Kernel_Name"] or "tile_syrk" in tr[i]["Kernel_Name"]
                                       for i in range(a, b))]
a, b = cand[-1]
ev = tr[a:b + 1]
t0 = int(ev[0]["Start_Timestamp"])


def short(n):
    n = n.split("(")[0].replace("gaplac::", "")
    if n.startswith("void "):  # template kernels (tail_kernel<GRAM>) demangle with their return type
        n = n[5:]
    return n.split("<")[0]


rows = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Queue_Id"], short(r["Kernel_Name"]))
        for r in ev]
end = max(e for _, e, _, _ in rows)
print(f"evaluation {end / 1e6:.3f} ms, {len(rows)} dispatches")
tot = defaultdict(lambda: [0, 0.0])
for s, e, q, n in rows:
    tot[n][0] += 1
    tot[n][1] += (e - s) / 1e3
for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
    print(f"  {n:24s} {c:5d} calls {t:9.1f} us total")
bulkn = ("tile_syrk_kernel", "tile_band_kernel", "quad_bulk_kernel")
iv = sorted((s, e) for s, e, _, n in rows if n in bulkn)
cov, cur_s, cur_e = 0, None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            cov += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    cov += cur_e - cur_s
first_bulk = iv[0][0] if iv else 0
tail = [(s, e) for s, e, _, n in rows if n == "tail_kernel"]
print(f"bulk-type kernels cover {cov / 1e6:.3f} ms; first starts at {first_bulk / 1e6:.3f} ms")
if tail:
    print(f"tail_kernel {tail[0][0] / 1e6:.3f} .. {tail[0][1] / 1e6:.3f} ms ({(tail[0][1] - tail[0][0]) / 1e6:.3f} ms)")
if "--list" in sys.argv:
    for s, e, q, n in rows:
        print(f"{s / 1e3:9.3f} {e / 1e3:9.3f} {(e - s) / 1e3:8.3f}  q{q:>2s}  {n}")
