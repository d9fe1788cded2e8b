"""Per-kernel register / scratch / occupancy from `hipcc -Rpass-analysis=kernel-resource-usage` output.
usage: python tools/kres.py <remarks.txt> [name-substring]"""
import re
import sys

cur, rows = None, []
for line in open(sys.argv[1], errors="replace"):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for r in rows:
    if sub in r["name"]:
        print(f"VGPR {r.get('VGPRs', '?'):>4} AGPR {r.get('AGPRs', '?'):>3} SGPR {r.get('TotalSGPRs', '?'):>4} "
              f"scratch {r.get('ScratchSize', '?'):>4} occ {r.get('Occupancy', '?')}  {r['name'][:110]}")
