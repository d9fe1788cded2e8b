"""Average PMC counters per kernel name over dispatches (rocprofv3 --pmc csv)."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
dur = {}
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"][:70]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for k in acc:
    print(k)
    for c in sorted(acc[k]):
        print(f"   {c:28s} {acc[k][c] / cnt[k][c]:16.1f}")
