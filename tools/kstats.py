"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total/avg time, per-step share.

usage: python tools/kstats.py <run_kernel_stats.csv> [steps|auto] [top]
steps=auto (default): the number of adam_prep_kernel launches (one per train step, eager or replayed)."""
import csv
import sys

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
arg = sys.argv[2] if len(sys.argv) > 2 else "auto"
if arg == "auto":
    steps = float(sum(int(r["Calls"]) for r in rows if "adam_prep_kernel" in r["Name"]) or 1)
else:
    steps = float(arg)
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {float(r['Percentage']):6.2f}% "
          f"n={int(r['Calls']) / steps:6.1f}/step avg={float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:100]}")
print(f"total {tot / 1e6 / steps:.3f} ms/step over {steps:.0f} steps")
