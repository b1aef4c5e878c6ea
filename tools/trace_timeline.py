"""Timeline of the last N dispatches of a rocprofv3 --kernel-trace CSV
(duration, gap to the previous dispatch on any queue, queue, name).

usage: python tools/trace_timeline.py TRACE_CSV [--last N] [--match SUBSTR]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--last", type=int, default=120)
ap.add_argument("--match", default="")
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.csv)) if a.match in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = rows[-a.last:]
prev, busy = None, 0
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    busy += e - s
    print(f"{(e - s) / 1e3:8.2f} gap {gap:8.2f} q{r['Queue_Id']:>2} {r['Kernel_Name'][:90]}")
    prev = max(prev or 0, e)
span = int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])
print(f"busy {busy / 1e3:.1f} us over span {span / 1e3:.1f} us")
