"""Per-shape microbenchmark of avt_conv3d_fwd (the tube step's R3D-18 3x3x3 convs, b clips of t frames)
across the tap-gather NT kernel's tile configs (avt_set_nt64_config / avt_set_nt128_config).  Prints TFLOP/s.
usage: python tools/conv3d_bench.py [--clips 8] [--frames 16] [--nt64 1,0,2,...] [--nt128 -1,1,2,...]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import avtubes  # noqa: E402,F401
from avt_amd._lib import call  # noqa: E402
from conv_bench import P, S, timeit  # noqa: E402

# (name, H, W, C, K, stride): the R3D-18 trunk at 224x224 frames (no max-pool; tube.py)
SHAPES = [
    ("L1 3x3x3", 112, 112, 64, 64, 1),
    ("L2.0 s2", 112, 112, 64, 128, 2),
    ("L2 3x3x3", 56, 56, 128, 128, 1),
    ("L3.0 s2", 56, 56, 128, 256, 2),
    ("L3 3x3x3", 28, 28, 256, 256, 1),
    ("L4.0 s2", 28, 28, 256, 512, 2),
    ("L4 3x3x3", 14, 14, 512, 512, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=8)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--nt64", default="-1")
    ap.add_argument("--nt128", default="-1")
    ap.add_argument("--halo3d", default="1,0", help="avt_set_halo3d values to sweep (1: the halo Conv3d form where it "
                    "applies, 0: the tap-gather kernel)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    b, T = args.clips, args.frames
    total = {}
    warm = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    for _ in range(50):
        warm @ warm
    torch.cuda.synchronize()
    for name, H, W, C, K, st in SHAPES:
        Ho, Wo = (H + 2 - 3) // st + 1, (W + 2 - 3) // st + 1
        x = torch.randn(b, T, H, W, C, device=dev).relu().to(torch.bfloat16)
        w = torch.randn(K, C, 3, 3, 3, device=dev) * 0.05
        wf = torch.empty(K, 27 * C, device=dev, dtype=torch.bfloat16)
        call("avt_pack_conv3d_weight", P(w), P(wf), K, C, 3, 3, 3, 0, S())
        y = torch.empty(b * T, Ho, Wo, K, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * y.numel() * 27 * C
        line = f"{name:10s} M={b * T * Ho * Wo:8d} N={K:4d} K={27 * C:5d} |"
        cfgs = [("nt64", int(v)) for v in args.nt64.split(",")] if K == 64 else \
               [("nt128", int(v)) for v in args.nt128.split(",")]
        if st == 1 and (K % 128 == 0 or K == 64):  # (K = 64: the halo form only under avt_set_halo3d(2))
            cfgs = [("halo3d", int(v)) for v in args.halo3d.split(",")] + \
                   [c for c in cfgs if c not in (("nt128", -1), ("nt64", -1))]
        for knob, v in cfgs:
            call("avt_set_halo3d", v if knob == "halo3d" else 0)
            if knob != "halo3d":
                call("avt_set_nt64_config" if knob == "nt64" else "avt_set_nt128_config", v)
            ms = timeit(lambda: call("avt_conv3d_fwd", P(x), P(wf), P(y), None, b, T, H, W, C, K, 3, 3, 3, st, 1, 1,
                                     S()))
            line += f" {knob}[{v}] {flops / ms / 1e9:5.0f} ({ms * 1e3:6.1f} us)"
            total[(knob, v)] = total.get((knob, v), 0.0) + ms
        call("avt_set_nt64_config", -1)
        call("avt_set_nt128_config", -1)
        call("avt_set_halo3d", -1)
        print(line, flush=True)
    print({f"{k}[{v}]": round(ms, 3) for (k, v), ms in total.items()}, "ms total")


if __name__ == "__main__":
    main()
