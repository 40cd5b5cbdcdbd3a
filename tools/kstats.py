"""Print a rocprofv3 kernel_stats.csv summary: python tools/kstats.py DIR"""
import csv, sys
rows = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_stats.csv")))
for r in rows:
    print(f"  {r['Name'][:44]:44s} calls={r['Calls']:>6s} total={float(r['TotalDurationNs'])/1e6:9.2f} ms avg={float(r['AverageNs'])/1e3:9.1f} us {float(r['Percentage']):6.2f}%")
