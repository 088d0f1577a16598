#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats CSV: total ms per step, calls per step, average us."""
import csv
import sys

path, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f'kernel total {tot / 1e6 / steps:.2f} ms per step')
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:7.3f} ms/step {int(r['Calls']) / steps:7.1f} calls "
          f"{float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:90]}")
