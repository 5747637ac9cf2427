#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv: name, calls, total ms, avg us."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print(path)
    rows = list(csv.DictReader(open(path)))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        name = re.sub(r"\(.*", "", r["Name"]).replace("void ", "")
        print(f"  {name[:60]:60s} {r['Calls']:>6} {float(r['TotalDurationNs'])/1e6:9.3f} ms {float(r['AverageNs'])/1e3:9.1f} us")
