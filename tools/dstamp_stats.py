"""Phase breakdown of the tail's diagonal-block (D) tasks from a tail trace's `.d` file.

The library writes `<trace>.d` next to the task timeline when GAPLAC_TAIL_TRACE is set on a
single evaluation: one "# N= T=" header per traced evaluation, then one line per tile column
k with 20 wall-clock stamps (100 MHz ticks) taken by thread 0 of the workgroup running D(k):
0 start, 1 after the block load, 2+2s phase-2 start of panel s, 3+2s after panel s's
phase-2 barrier, 19 end (see potrf_diag2_body's dstamp points).

usage: python tools/dstamp_stats.py <trace>.d [--all]
"""
import statistics as st
import sys

TICK_US = 0.01  # wall_clock64 runs at 100 MHz on gfx950


def blocks(path):
    out, cur, hdr = [], [], None
    for line in open(path):
        if line.startswith("#"):
            if hdr is not None:
                out.append((hdr, cur))
            hdr, cur = line[1:].strip(), []
        elif line.strip():
            cur.append([int(x) for x in line.split()])
    if hdr is not None:
        out.append((hdr, cur))
    return out


def summarize(rows):
    load, fin, tot = [], [], []
    p1 = [[] for _ in range(8)]
    p2 = [[] for _ in range(8)]
    for r in rows:
        s = r[1:]
        if len(s) < 20 or s[0] == 0 or s[19] == 0:
            continue
        load.append((s[1] - s[0]) * TICK_US)
        for q in range(8):
            prev = s[1] if q == 0 else s[3 + 2 * (q - 1)]
            p1[q].append((s[2 + 2 * q] - prev) * TICK_US)
            p2[q].append((s[3 + 2 * q] - s[2 + 2 * q]) * TICK_US)
        fin.append((s[19] - s[17]) * TICK_US)
        tot.append((s[19] - s[0]) * TICK_US)
    if not tot:
        return "no complete D stamps"
    lines = [f"D tasks {len(tot)}: total {st.mean(tot):.2f} us (median {st.median(tot):.2f}, "
             f"min {min(tot):.2f}, max {max(tot):.2f})",
             f"  load   {st.mean(load):.2f} us (min {min(load):.2f}, max {max(load):.2f})"]
    for q in range(8):
        lines.append(f"  panel {q}: phase 1 + barrier {st.mean(p1[q]):.2f} us, "
                     f"phase 2 {st.mean(p2[q]):.2f} us")
    lines.append(f"  after the last panel {st.mean(fin):.2f} us")
    return "\n".join(lines)


def main():
    path = sys.argv[1]
    bl = blocks(path)
    todo = bl if "--all" in sys.argv[2:] else bl[-1:]
    for hdr, rows in todo:
        print(f"# {hdr}")
        print(summarize(rows))


if __name__ == "__main__":
    main()
