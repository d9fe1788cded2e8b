"""Timeline of one replayed train step from a rocprofv3 kernel trace (run_kernel_trace.csv).

    python tools/timeline.py <run_kernel_trace.csv> [--top 30] [--step -1]

Steps are delimited by adam_prep_kernel launches (one per step); the replayed steps are the shortest ones.  For the
chosen step (default: the median replayed step) prints the wall time, the time with no kernel
running (gaps), the time with exactly one kernel running attributed to that kernel ("alone" = the
serial critical path the other stream did not cover), and the overlapped time.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("avt::", "")
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--step", type=int, default=None, help="index among the replayed steps")
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]))
    rows.sort()
    # one adam_prep_kernel per train step (Adam itself runs once per trunk region)
    mark = "adam_prep_kernel" if any("adam_prep_kernel" in r[2] for r in rows) else "adam_kernel"
    ends = [i for i, r in enumerate(rows) if mark in r[2]]
    steps = []
    for a, b in zip(ends, ends[1:]):
        seg = rows[a:b]
        t0 = rows[a][0]
        t1 = max(r[1] for r in seg)
        steps.append((t1 - t0, seg, t0))
    if not steps:
        raise SystemExit("no steps found")
    durs = sorted(s[0] for s in steps)
    print("step durations (us):", [round(s[0] / 1e3, 1) for s in steps])
    fast = [s for s in steps if s[0] <= durs[0] * 1.3]
    pick = fast[len(fast) // 2] if args.step is None else fast[args.step]
    wall, seg, t0 = pick
    ev = []
    for s, e, n, q in seg:
        ev.append((max(s, t0), 1, n))
        ev.append((e, -1, n))
    ev.sort(key=lambda x: (x[0], x[1]))
    active = defaultdict(int)
    nact = 0
    last = t0
    gap = 0
    alone = defaultdict(int)
    multi = 0
    for t, d, n in ev:
        dt = t - last
        if dt > 0:
            if nact == 0:
                gap += dt
            elif nact == 1:
                k = next(k for k, v in active.items() if v > 0)
                alone[k] += dt
            else:
                multi += dt
        last = t
        nact += d
        active[n] += d
    busy = defaultdict(int)
    cnt = defaultdict(int)
    for s, e, n, q in seg:
        busy[short(n)] += e - s
        cnt[short(n)] += 1
    al = defaultdict(int)
    for n, v in alone.items():
        al[short(n)] += v
    print(f"wall {wall / 1e3:.1f} us  kernels {len(seg)}  gaps {gap / 1e3:.1f} us  "
          f"alone {sum(alone.values()) / 1e3:.1f} us  overlapped {multi / 1e3:.1f} us")
    print(f"{'alone us':>9} {'busy us':>9} {'n':>4}  kernel")
    for n, v in sorted(al.items(), key=lambda x: -x[1])[:args.top]:
        print(f"{v / 1e3:9.1f} {busy[n] / 1e3:9.1f} {cnt[n]:4d}  {n}")


if __name__ == "__main__":
    main()
