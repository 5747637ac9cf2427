#!/usr/bin/env python3
"""Sum the host layer's TMV_HOST_TIMING phase lines of a log (stderr of a
run with TMV_HOST_TIMING=1): per (call tag, phase) the count, median and
total milliseconds.   python tools/phase_sum.py log [...]"""
import collections
import re
import sys

for path in sys.argv[1:]:
    m = collections.defaultdict(list)
    for line in open(path):
        r = re.match(r"\[(\S+)\]\s+(.+?)\s+([\d.]+) ms", line)
        if r:
            m[(r.group(1), r.group(2).strip())].append(float(r.group(3)))
    print(path)
    for k, v in sorted(m.items()):
        v2 = sorted(v)
        print("  %-24s %-26s n=%5d med %8.3f  total %9.2f ms" % (k[0], k[1], len(v), v2[len(v2) // 2], sum(v)))
