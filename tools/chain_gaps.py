"""How long the bulk-update kernels (tile_syrk_kernel) sit idle between launches
(waiting for the panel chain) in the last evaluation of a rocprofv3 trace."""
import csv
import sys

tr = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
grams = [i for i, r in enumerate(tr) if "gram_kernel" in r["Kernel_Name"]]
ev = tr[grams[-1]:]
t0 = int(ev[0]["Start_Timestamp"])
rest = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0) for r in ev if "tile_syrk_kernel" in r["Kernel_Name"]]
end = max(int(r["End_Timestamp"]) for r in ev) - t0
busy = sum(b - a for a, b in rest)
gaps = [(rest[i + 1][0] - rest[i][1]) for i in range(len(rest) - 1)]
print(f"eval {end/1e3:.1f} us; bulk kernels {len(rest)} busy {busy/1e3:.1f} us; idle between them {sum(gaps)/1e3:.1f} us; "
      f"after last bulk kernel {(end - rest[-1][1])/1e3:.1f} us; before first {rest[0][0]/1e3:.1f} us")
acc = 0
for i, g in enumerate(gaps):
    acc += g
    if i % 8 == 0 or i > len(gaps) - 4:
        print(f"  step {i:3d}: bulk dur {(rest[i][1]-rest[i][0])/1e3:8.1f} us, gap after {g/1e3:7.1f} us, cum idle {acc/1e3:8.1f}")
