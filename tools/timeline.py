"""GPU occupancy of a step from a rocprofv3 kernel trace (--kernel-trace --output-format csv): per step, the span from
the first kernel's start to the last one's end, the time with 0 / 1 / 2+ kernels in flight, and the largest idle gaps.
Steps are delimited by the Adam launches (--marker, the last kernel of a step's trunks; `--per-step` of them per step).
Usage: python tools/timeline.py <run_kernel_trace.csv> [--last 5] [--marker avt::adam_kernel] [--per-step 2]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=5)
    ap.add_argument("--marker", default="avt::adam_kernel")
    ap.add_argument("--per-step", type=int, default=2)
    a = ap.parse_args()
    ev = []
    for r in csv.DictReader(open(a.trace)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]))
    ev.sort()
    marks = [i for i, e in enumerate(ev) if e[2].startswith(a.marker)]
    ends = marks[a.per_step - 1::a.per_step]
    print(f"{len(ev)} kernels, {len(marks)} '{a.marker}' launches, queues {sorted({e[3] for e in ev})}")
    for k in range(max(0, len(ends) - a.last), len(ends)):
        if k == 0:
            continue
        seg = ev[ends[k - 1] + 1:ends[k] + 1]
        if not seg:
            continue
        t0, t1 = seg[0][0], max(e[1] for e in seg)
        pts = sorted([(s, 1) for s, _, _, _ in seg] + [(e, -1) for _, e, _, _ in seg])
        lvl, last, hist = 0, t0, {0: 0, 1: 0, 2: 0}
        gaps = []
        for t, d in pts:
            dt = t - last
            hist[min(lvl, 2)] += dt
            if lvl == 0 and dt > 0:
                gaps.append((dt, last - t0))
            lvl += d
            last = t
        span = (t1 - t0) / 1e3
        gaps.sort(reverse=True)
        print(f"step {k}: span {span:8.1f} us  kernels {len(seg):4d}  idle {hist[0] / 1e3:7.1f}  one {hist[1] / 1e3:7.1f}  "
              f"two+ {hist[2] / 1e3:7.1f} us  idle gaps > 5 us: {sum(1 for g, _ in gaps if g > 5000)}  largest "
              f"{[(round(g / 1e3, 1), round(at / 1e3)) for g, at in gaps[:5]]}")


if __name__ == "__main__":
    main()
