"""Average SQ counters per kernel from rocprofv3 --pmc csv outputs.

usage: python tools/pmc_summary.py CSV [CSV ...] [--match SUBSTR]
"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv", nargs="+")
ap.add_argument("--match", default="pass_kernel")
a = ap.parse_args()
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in a.csv:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not any(m in k for m in a.match.split("\\|")):
            continue
        agg[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v) / len(v) / 1e6:10.2f} M")
