"""Per-kernel FETCH_SIZE / WRITE_SIZE of tools/fetch_calib against the bytes it touches.
usage: python tools/pmc_calib.py FETCH_DIR WRITE_DIR"""
import csv
import glob
import sys

BYTES = 16384 * 16384 * 8


def per_kernel(d, counter):
    out = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                k = r["Kernel_Name"].split("(")[0]
                out.setdefault(k, []).append(float(r["Counter_Value"]) * 1024)
    return out


f = per_kernel(sys.argv[1], "FETCH_SIZE")
w = per_kernel(sys.argv[2], "WRITE_SIZE")
for k in sorted(set(f) | set(w)):
    fv = f.get(k, [0])
    wv = w.get(k, [0])
    print(f"{k:12s} FETCH_SIZE {sum(fv)/len(fv)/BYTES:6.3f} x bytes   WRITE_SIZE {sum(wv)/len(wv)/BYTES:6.3f} x bytes")
