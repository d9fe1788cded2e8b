"""Stem (7x7/s2, C = 4 vision / 1 audio, K = 64) wgrad at B = 128 under a sweep of the split policy
(avt_set_wgrad_policy target_blocks,min_kt).  Usage: python tools/stem_wgrad_bench.py "0,4;0,16;512,4"."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avtubes  # noqa: E402,F401
from avt_amd._lib import call, query  # noqa: E402
from avt_amd.trunk import P, stream_ptr  # noqa: E402

N = 128
pols = sys.argv[1] if len(sys.argv) > 1 else "0,4"
dev = torch.device("cuda")
for name, H, W, Cp, C in [("V.stem", 224, 224, 4, 3), ("A.stem", 257, 300, 1, 1)]:
    Pq, Qq = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    x = torch.randn(N, H, W, Cp, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, Pq, Qq, 64, device=dev).to(torch.bfloat16)
    dw = torch.zeros(64, 7, 7, C, device=dev)
    flops = 2.0 * N * Pq * Qq * 64 * 49 * C
    line = f"{name:8s} M={N * Pq * Qq:8d}"
    for pol in pols.split(";"):
        tb, mk = (int(s) for s in pol.split(","))
        call("avt_set_wgrad_policy", tb, mk)
        wsb = int(query("avt_conv2d_wgrad_workspace", N, H, W, Cp, C, 64, 7, 7, 2, 3))
        ws = torch.empty(max(1, wsb), device=dev, dtype=torch.uint8)
        fn = lambda: call("avt_conv2d_wgrad", P(x), P(dy), P(dw), N, H, W, Cp, C, 64, 7, 7, 2, 3, P(ws), wsb,
                          stream_ptr())
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        line += f" | [{pol}] {ms * 1e3:7.1f} us {flops / ms / 1e9:6.0f} TFLOP/s"
    call("avt_set_wgrad_policy", 0, 4)
    print(line, flush=True)
