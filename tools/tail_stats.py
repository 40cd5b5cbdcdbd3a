"""Per-task-type statistics and the per-column critical path of the last persistent-tail
launch in a GAPLAC_TAIL_TRACE file (dequeue / start / end times per task, 100 MHz).
usage: python tools/tail_stats.py TRACE_FILE [ncu]"""
import collections
import sys

path = sys.argv[1]
ncu = int(sys.argv[2]) if len(sys.argv) > 2 else 256
blocks, cur = [], []
for line in open(path):
    if line.startswith("#"):
        if cur:
            blocks.append(cur)
        cur = []
    else:
        cur.append([int(x) for x in line.split()])
blocks.append(cur)
b = blocks[-1]
T0 = min(r[2] for r in b)
t1 = max(r[4] for r in b)
span = (t1 - T0) / 100.0
wait = sum(r[3] - r[2] for r in b) / 100.0
run = sum(r[4] - r[3] for r in b) / 100.0
print(f"tasks {len(b)}  span {span:.1f} us  workgroup-time {ncu * span:.0f} us: wait {wait:.0f} ({wait / ncu / span:.2f}), "
      f"run {run:.0f} ({run / ncu / span:.2f}), other {ncu * span - wait - run:.0f}")


def dec(e):
    return e & 3, (e >> 2) & 15, (e >> 6) & 127, (e >> 13) & 127, (e >> 20) & 127


names = {0: "D", 1: "S", 3: "Q"}
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for r in b:
    t, q, k, i, j = dec(r[1])
    key = names.get(t, "U") + (str(q) if t == 2 else ("w" if t == 1 and q == 2 else ""))
    agg[key][0] += 1
    agg[key][1] += (r[3] - r[2]) / 100
    agg[key][2] += (r[4] - r[3]) / 100
for k, v in sorted(agg.items()):
    print(f"  {k:4s} n={v[0]:6d} wait={v[1]:9.0f} us run={v[2]:9.0f} us  avg run {v[2] / v[0]:6.2f} us")
us = lambda t: (t - T0) / 100.0  # noqa: E731
D, S, Q = {}, {}, {}
for r in b:
    t, q, k, i, j = dec(r[1])
    if t == 0 and (r[1] >> 27) == 0:
        D[k] = r
    elif t == 1 and (r[1] >> 27) == 0:
        S.setdefault((i, k), []).append(r)
    elif t == 3 and (r[1] >> 27) == 0:
        Q.setdefault((i, k), []).append(r)
ks = sorted(D)
print("critical path per column (model 0): D run | D end -> S(k+1,k) end | -> Q(k+1) end | -> D(k+1) start")
tot = collections.Counter()
for k in ks[:-1]:
    d, dn = D[k], D.get(k + 1)
    s, qq = S.get((k + 1, k), []), Q.get((k + 1, k), [])
    if not s or not qq or not dn:
        continue
    se = max(x[4] for x in s)
    qe = max(x[4] for x in qq)
    parts = ((d[4] - d[3]) / 100, (se - d[4]) / 100, (qe - se) / 100, (dn[3] - qe) / 100)
    for n, p in zip(("D", "S", "Q", "hop"), parts):
        tot[n] += p
    if k % 8 == 0 or k == ks[-2]:
        print(f"  k={k:3d}: D {parts[0]:6.1f} | S {parts[1]:6.1f} | Q {parts[2]:6.1f} | hop {parts[3]:6.1f}")
print("  totals (us): " + "  ".join(f"{n} {v:.0f}" for n, v in tot.items()))
