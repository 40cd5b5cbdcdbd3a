"""Per-launch HBM traffic of the dominant kernel from rocprofv3 --pmc passes.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON [kernel-substring]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. gfx950 correction (MI355X_MICROARCH.md
§HBM, cdna_hip_programming.md §7): FETCH_SIZE reports 1/2 of the bytes of a wide
coalesced streaming read (16 B/lane), so fetch bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE
reads exactly for 16-B/lane streaming stores. The SYRK kernel's reads are 16 B/lane
(panel staging) plus 8 B/lane C-tile loads and its stores are 8 B/lane: the other widths
are uncalibrated, so the corrected number is an estimate.
"""
import csv
import glob
import json
import sys


def per_dispatch(d, counter, kern):
    vals = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and kern in r.get("Kernel_Name", ""):
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    fd, wd, out = sys.argv[1:4]
    kern = sys.argv[4] if len(sys.argv) > 4 else "tile_syrk_kernel"
    fetch = per_dispatch(fd, "FETCH_SIZE", kern)
    write = per_dispatch(wd, "WRITE_SIZE", kern)
    if not fetch or not write:
        print("no counter rows found", len(fetch), len(write))
        sys.exit(1)
    f_avg = sum(fetch) / len(fetch) * 1024
    w_avg = sum(write) / len(write) * 1024
    rec = {"kernel": kern, "dispatches": [len(fetch), len(write)],
           "fetch_size_bytes_raw_per_launch": f_avg, "write_size_bytes_per_launch": w_avg,
           "bytes_per_launch": 2 * f_avg + w_avg,
           "correction": "fetch x2 (gfx950 FETCH_SIZE half-count on 16B/lane streams); write as reported"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
