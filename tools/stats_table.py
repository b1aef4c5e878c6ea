"""Render a rocprofv3 --stats kernel_stats.csv as a fixed-width table (top N by total time).

usage: python tools/stats_table.py KERNEL_STATS_CSV [--top N] [--title TEXT]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--title", default="")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
if a.title:
    print("# " + a.title)
print(f"{'calls':>6} {'avg_us':>9} {'total_us':>10} {'pct':>6}  name")
for r in rows[: a.top]:
    print(f"{int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} {float(r['TotalDurationNs']) / 1e3:10.1f} "
          f"{float(r['Percentage']):6.2f}  {r['Name'][:160]}")
