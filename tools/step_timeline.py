"""One train step's kernels from a rocprofv3 kernel-trace CSV: start/end (us,
relative to the step's gather launch), duration, queue, short name.  The step
is the last pair of consecutive gather launches 0.3-1.5 ms apart.

usage: python tools/step_timeline.py TRACE_CSV [--gather SUBSTR]
"""
import argparse
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--gather", default="gather_grouped")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
g = [i for i, r in enumerate(rows) if a.gather in r["Kernel_Name"]]
best = None
for x, y in zip(g, g[1:]):
    d = int(rows[y]["Start_Timestamp"]) - int(rows[x]["Start_Timestamp"])
    if 300e3 < d < 1500e3:
        best = (x, y)
x, y = best
t0 = int(rows[x]["Start_Timestamp"])


def short(n):
    n = re.sub(r"^void ", "", n)
    n = n.replace("tt::(anonymous namespace)::", "")
    if n.startswith("Cijk"):
        return "hipBLASLt " + n[:40]
    m = re.search(r"detail::(\w+)", n) if "rocprim" in n else None
    if m:
        return "rocprim " + m.group(1)[:50]
    return n[:70]


for r in rows[x:y + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} q{r['Queue_Id']} {short(r['Kernel_Name'])}")
