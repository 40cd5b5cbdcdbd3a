"""Per-column hand-off detail of the last tail launch in a GAPLAC_TAIL_TRACE file: for each
tile column k, D(k)'s run, the start / end of S(k+1,k) and of the Q blocks of tile k+1,
the last update tasks on tile (k+1, k), and D(k+1)'s start, all relative to D(k)'s end (us).
usage: python tools/tail_crit.py TRACE_FILE"""
import sys


def load(path):
    blocks, cur = [], []
    for line in open(path):
        if line.startswith("#"):
            if cur:
                blocks.append(cur)
            cur = []
        elif line.strip():
            cur.append([int(x) for x in line.split()])
    blocks.append(cur)
    return blocks[-1]


def dec(e):
    return e & 3, (e >> 2) & 15, (e >> 6) & 127, (e >> 13) & 127, (e >> 20) & 127


def main():
    b = load(sys.argv[1])
    T0 = min(r[2] for r in b)
    us = lambda t: (t - T0) / 100.0  # noqa: E731
    D, S, Q, U = {}, {}, {}, {}
    for idx, r in enumerate(b):
        t, q, k, i, j = dec(r[1])
        if r[1] >> 27:
            continue  # model 0 only
        if t == 0:
            D[k] = r
        elif t == 1:
            S.setdefault((i, k), []).append(r)
        elif t == 3:
            Q.setdefault((i, k), []).append(r)
        else:
            U.setdefault((i, j), []).append((idx, q, k, r))
    tot_gap = 0.0
    for k in sorted(D):
        if k + 1 not in D or (k + 1, k) not in S:
            continue
        de = us(D[k][4])
        s = S[(k + 1, k)]
        qq = Q.get((k + 1, k), [])
        ss = min(us(r[3]) for r in s) - de
        se = max(us(r[4]) for r in s) - de
        qd = min(us(r[2]) for r in qq) - de if qq else float("nan")
        qs = min(us(r[3]) for r in qq) - de if qq else float("nan")
        qe = max(us(r[4]) for r in qq) - de if qq else float("nan")
        nxt = us(D[k + 1][3]) - de
        tot_gap += nxt
        last = sorted(U.get((k + 1, k), []), key=lambda x: x[3][4])[-1:]
        lu = " ".join(f"U#{ix} q{q} k{kk} deq {us(r[2]) - de:+.1f} start {us(r[3]) - de:+.1f} end {us(r[4]) - de:+.1f}"
                      for ix, q, kk, r in last)
        print(f"k={k:3d} D {us(D[k][4]) - us(D[k][3]):5.1f} | S start {ss:+6.1f} end {se:+6.1f} | "
              f"Q deq {qd:+6.1f} start {qs:+6.1f} end {qe:+6.1f} | D+1 {nxt:+6.1f} | last {lu}")
    print(f"sum of D(k) end -> D(k+1) start gaps: {tot_gap:.1f} us")


if __name__ == "__main__":
    main()
