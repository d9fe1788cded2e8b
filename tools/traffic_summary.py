"""Per-kernel HBM bytes from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

FETCH_SIZE and WRITE_SIZE are reported in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE counts exactly half the bytes of wide (16 B/lane) streaming reads, so read bytes =
2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B stores and dword atomics.  The Adam kernel
(known bytes: 16 B/param read, 12 B/param written) is printed as the calibration check.

usage: python tools/traffic_summary.py <dir with FETCH_SIZE/ WRITE_SIZE/> <steps in the run> [--json out] [--batch B]
"""
import csv
import glob
import json
import sys
from collections import defaultdict

CONV = ("avt::conv_", "gemm_nt_kernel", "gemm_tn_kernel", "wgrad_slab_reduce_kernel")  # every conv kernel
BN = ("avt::bn_", "avt::stem_bn", "avt::stem_maxpool")


def load(d, ctr):
    tot, cnt = defaultdict(float), defaultdict(int)
    for path in glob.glob(f"{d}/{ctr}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != ctr:
                continue
            k = r["Kernel_Name"]
            tot[k] += float(r["Counter_Value"])
            cnt[k] += 1
    return tot, cnt


def kernel_rows(d):
    """[(kernel, dispatches, read bytes, write bytes)] over the whole run, largest first."""
    fetch, nf = load(d, "FETCH_SIZE")
    write, _ = load(d, "WRITE_SIZE")
    rows = []
    for k in set(fetch) | set(write):
        rd = 2.0 * fetch.get(k, 0.0) * 1024.0
        wr = write.get(k, 0.0) * 1024.0
        rows.append((k, nf.get(k, 0), rd, wr))
    rows.sort(key=lambda r: -(r[2] + r[3]))
    return rows


def summarize(d, steps, batch, source, lib_hash=None):
    """The per-step traffic record bench.py reads (conv family, BN family, whole step, per kernel)."""
    rows = kernel_rows(d)
    conv = [r for r in rows if any(c in r[0] for c in CONV)]
    conv_rd, conv_wr, conv_n = sum(r[2] for r in conv), sum(r[3] for r in conv), sum(r[1] for r in conv)
    bn_b = sum(rd + wr for k, n, rd, wr in rows if any(c in k for c in BN))
    tot_b = sum(rd + wr for k, n, rd, wr in rows)
    return {"per_gpu_batch": batch, "source": source, "lib_source_hash": lib_hash,
            "conv_dispatches_per_step": conv_n / steps, "conv_read_bytes_per_step": conv_rd / steps,
            "conv_write_bytes_per_step": conv_wr / steps,
            "conv_bytes_per_dispatch": (conv_rd + conv_wr) / max(conv_n, 1),
            "conv_kernels": sorted({r[0][:120] for r in conv}),
            "step_bytes": tot_b / steps, "bn_family_bytes_per_step": bn_b / steps,
            "per_kernel": {k[:120]: {"dispatches_per_step": n / steps, "read_bytes_per_step": rd / steps,
                                     "write_bytes_per_step": wr / steps} for k, n, rd, wr in rows}}


def main():
    d, steps = sys.argv[1], float(sys.argv[2])
    rows = kernel_rows(d)
    conv_rd = conv_wr = 0.0
    conv_n = 0
    for k, n, rd, wr in rows:
        if any(c in k for c in CONV):
            conv_rd += rd
            conv_wr += wr
            conv_n += n
    bn_b = sum(rd + wr for k, n, rd, wr in rows if any(c in k for c in BN))
    tot_b = sum(rd + wr for k, n, rd, wr in rows)
    print(f"step total: {tot_b / 1e9 / steps:.3f} GB/step; BN family {bn_b / 1e9 / steps:.3f} GB/step")
    for k, n, rd, wr in rows[:40]:
        print(f"{(rd + wr) / 1e9 / steps:8.3f} GB/step  read {rd / 1e9 / steps:7.3f}  write {wr / 1e9 / steps:7.3f}  "
              f"n={n / steps:6.1f}/step  {k[:90]}")
    print(f"conv family: {conv_n / steps:.0f} dispatches/step, read {conv_rd / 1e9 / steps:.3f} GB/step, "
          f"write {conv_wr / 1e9 / steps:.3f} GB/step, {(conv_rd + conv_wr) / max(conv_n, 1) / 1e6:.3f} MB/dispatch")
    for k, n, rd, wr in rows:
        if "adam_kernel" in k:
            print(f"calibration adam: read {rd / n / 1e6:.1f} MB/launch, write {wr / n / 1e6:.1f} MB/launch "
                  f"(algorithmic: 357.5 read / 268.2 write for 22,346,752 params)")
    if "--json" in sys.argv:
        out = sys.argv[sys.argv.index("--json") + 1]
        batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 128
        lib_hash = sys.argv[sys.argv.index("--lib-hash") + 1] if "--lib-hash" in sys.argv else None
        json.dump(summarize(d, steps, batch, "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --no-graph "
                            "(tools/pmc_traffic.sh); read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB", lib_hash),
                  open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
