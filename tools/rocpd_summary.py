"""Summarise a rocprofv3 rocpd sqlite database: per-kernel stats, or a timeline.

usage: python tools/rocpd_summary.py DB [--timeline N] [--match SUBSTR]
"""
import argparse
import collections
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    depth, out = 0, []
    for ch in name:  # drop template arguments and parameter lists
        if ch in "<(":
            depth += 1
        elif ch in ">)":
            depth -= 1
        elif depth == 0:
            out.append(ch)
    return "".join(out)[-90:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--timeline", type=int, default=0, help="print the last N dispatches in order")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start"))
    rows = [r for r in rows if a.match in r[0]]
    if a.timeline:
        sel = rows[-a.timeline:]
        prev = None
        for n, s, e, gx, wx in sel:
            gap = (s - prev) / 1e3 if prev else 0.0
            print(f"{(e - s) / 1e3:9.2f} us  gap {gap:7.2f}  grid {gx // max(wx, 1):7d}x{wx:<5d} {short(n)}")
            prev = e
        return
    agg = collections.defaultdict(list)
    for n, s, e, *_ in rows:
        agg[short(n)].append((e - s) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"{'calls':>6} {'avg_us':>9} {'total_us':>11} {'pct':>6}  name")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):6d} {sum(v) / len(v):9.2f} {sum(v):11.1f} {100 * sum(v) / tot:6.2f}  {k}")


if __name__ == "__main__":
    main()
