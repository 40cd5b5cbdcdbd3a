"""Summarise a GAPLAC_TAIL_TRACE file (tail_kernel per-task times, 100 MHz ticks):
per task type the mean execution time and wait, and per column k the critical chain
D(k) -> S(k+1,k) -> Q(k+1,k+1;k) -> D(k+1). Uses the LAST launch in the file."""
import sys
from collections import defaultdict

NAMES = {0: "D", 1: "S", 2: "U", 3: "Q"}


def main(path):
    blocks = []
    cur = None
    for line in open(path):
        if line.startswith("#"):
            cur = []
            blocks.append((line.strip(), cur))
            continue
        i, e, t0, t1, t2 = map(int, line.split())
        cur.append((e, t0, t1, t2))
    head, rows = blocks[-1]
    print(head)
    base = min(r[1] for r in rows)
    us = lambda t: (t - base) / 100.0  # noqa: E731
    dur = defaultdict(list)
    wait = defaultdict(list)
    by = {}
    for e, t0, t1, t2 in rows:
        ty, q, k, i, j = e & 3, (e >> 2) & 15, (e >> 6) & 127, (e >> 13) & 127, (e >> 20) & 127
        m = e >> 27  # model (batched launches)
        dur[ty].append((t2 - t1) / 100.0)
        wait[ty].append((t1 - t0) / 100.0)
        by[(ty, q, k, i, j) if m == 0 else (ty, q, k, i, j, m)] = (us(t0), us(t1), us(t2))
    for ty in sorted(dur):
        d, w = dur[ty], wait[ty]
        print(f"{NAMES[ty]}: n={len(d):5d} exec mean {sum(d) / len(d):7.2f} us max {max(d):7.2f}  "
              f"wait mean {sum(w) / len(w):7.2f} max {max(w):7.2f}")
    # U tasks by shape, with their MFMA rate per workgroup (fp64 peak per CU = 78.6/256 TF/s)
    ushape = defaultdict(list)
    for key, (t0, t1, t2) in by.items():
        ty, q = key[0], key[1]
        if ty == 2:
            ushape["K=1024 tile" if q == 6 else "K=512 tile" if q == 5 else "K=256 tile" if q == 7
                   else "K=128 tile" if q == 0 else "K=128 quadrant"].append(t2 - t1)
    flops = {"K=1024 tile": 2 * 128 * 128 * 1024, "K=512 tile": 2 * 128 * 128 * 512, "K=256 tile": 2 * 128 * 128 * 256,
             "K=128 tile": 2 * 128 * 128 * 128,
             "K=128 quadrant": 2 * 64 * 64 * 128}
    for name, d in sorted(ushape.items()):
        m = sum(d) / len(d)
        print(f"  U {name:15s} n={len(d):5d} exec mean {m:7.2f} us = {flops[name] / m / 1e6:.3f} TF/s per CU "
              f"({flops[name] / m / 1e6 / (78.6 / 256):.2f} of peak)")
    span = (max(r[3] for r in rows) - base) / 100.0
    ex = sum(sum(d) for d in dur.values())
    wt = sum(sum(w) for w in wait.values())
    grid = 256
    print(f"span {span:.1f} us; over {grid} workgroups: exec {ex / (grid * span):.3f}, wait {wt / (grid * span):.3f}, "
          f"rest (dequeue, idle) {1 - (ex + wt) / (grid * span):.3f}")
    T = max(key[2] for key in by) + 2
    print(f"{'k':>3} {'D start':>9} {'D end':>9} {'S start':>9} {'S end':>9} {'Q start':>9} {'Q end':>9} {'D+1 deq':>9}")
    for k in range(T - 1):
        d = by.get((0, 0, k, 0, 0))
        ss = [by.get((1, h, k, k + 1, 0)) for h in (0, 1)]
        qs = [by.get((3, q, k, k + 1, k + 1)) for q in (0, 2, 3)]
        dn = by.get((0, 0, k + 1, 0, 0))
        if not (d and all(ss) and all(qs) and dn):
            continue
        print(f"{k:3d} {d[1]:9.1f} {d[2]:9.1f} {min(x[1] for x in ss):9.1f} {max(x[2] for x in ss):9.1f} "
              f"{min(x[1] for x in qs):9.1f} {max(x[2] for x in qs):9.1f} {dn[0]:9.1f}")
    end = max(r[3] for r in rows)
    print(f"launch span {us(end):.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
