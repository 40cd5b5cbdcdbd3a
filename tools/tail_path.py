"""Critical path of the last tail launch in a GAPLAC_TAIL_TRACE file (model 0 of a
single-evaluation list). Dependencies are tail_wait's rules (gaplac_kernels.hip):
  D(k)           every update of tile (k, k) with a column < k
  S(i,k)         every update of tile (i, k) with a column < k; D(k) (pipelined)
  U/Q (i,j) ; k  every update of tile (i, j) with a column < k; S(i,k+c), S(j,k+c) for the
                 task's panel columns (a Q block of tile k+1 follows S(k+1,k) pipelined)
From the last-ending task the walk steps to the dependency that ended last; each step
prints the task, its dequeue / start / end (us from the launch start) and the gap between
that dependency's end and the task's start (the hand-off plus any dequeue delay).
usage: python tools/tail_path.py TRACE_FILE [--summary]"""
import collections
import sys

TK_D, TK_S, TK_U, TK_Q = 0, 1, 2, 3
DEEP = {5: 4, 6: 8, 7: 2}


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


def name(t, q, k, i, j):
    if t == TK_D:
        return f"D({k})"
    if t == TK_S:
        return f"S({i},{k})h{q}"
    if t == TK_Q:
        return f"Q({i};{k})b{q}"
    return f"U({i},{j};{k})q{q}"


def main():
    b = load(sys.argv[1])
    T0 = min(r[2] for r in b)
    us = lambda t: (t - T0) / 100.0  # noqa: E731
    tasks = []
    upd = collections.defaultdict(list)  # tile -> update tasks
    S = collections.defaultdict(list)
    D = {}
    for r in b:
        if r[1] >> 27:
            continue
        t, q, k, i, j = dec(r[1])
        x = dict(t=t, q=q, k=k, i=i, j=j, deq=us(r[2]), st=us(r[3]), en=us(r[4]))
        tasks.append(x)
        if t == TK_D:
            D[k] = x
        elif t == TK_S:
            S[(i, k)].append(x)
        else:
            upd[(i, j)].append(x)

    def deps(x):
        t, k, i, j = x["t"], x["k"], x["i"], x["j"]
        out = []
        if t == TK_D:
            out += [y for y in upd[(k, k)] if y["k"] < k]
        elif t == TK_S:
            out += [y for y in upd[(i, k)] if y["k"] < k]
            if k in D:
                out.append(D[k])
        else:
            out += [y for y in upd[(i, j)] if y["k"] < k]
            nk = DEEP.get(x["q"], 1) if t == TK_U else 1
            for c in range(nk):
                out += S[(i, k + c)]
                if i != j:
                    out += S[(j, k + c)]
        return out

    x = max(tasks, key=lambda y: y["en"])
    path = []
    while x is not None:
        ds = deps(x)
        p = max(ds, key=lambda y: y["en"]) if ds else None
        path.append((x, p))
        x = p
    path.reverse()
    agg = collections.Counter()
    for x, p in path:
        run = x["en"] - x["st"]
        gap = x["st"] - p["en"] if p else x["st"]
        kind = "DSUQ"[x["t"]]
        agg[kind + " run"] += run
        agg[kind + " gap"] += gap
        if "--summary" not in sys.argv[2:]:
            print(f"{name(x['t'], x['q'], x['k'], x['i'], x['j']):18s} deq {x['deq']:8.1f} start {x['st']:8.1f} "
                  f"end {x['en']:8.1f} run {run:6.1f} gap {gap:+6.1f}" + ("  (dequeued after dep end)"
                                                                         if p and x["deq"] > p["en"] else ""))
    print(f"critical path {path[-1][0]['en']:.1f} us over {len(path)} tasks: " +
          ", ".join(f"{k} {v:.1f}" for k, v in sorted(agg.items())))


if __name__ == "__main__":
    main()
