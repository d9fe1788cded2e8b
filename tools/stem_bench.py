"""Microbenchmark of the 7x7/s2 stem forward kernels at the B=128 trunk shapes: the persistent
LDS-patch kernel (avt_set_stem_kernel(1)) vs the generic gather kernel (0).  Prints us per launch,
TFLOP/s of the real (unpadded) FLOPs and the output-store GB/s (the bound: 205 / 317 MB); then the
stem wgrads: the per-wave LDS-patch kernel (avt_set_stem_wgrad(1)) vs the generic one, with the
GB/s of the bytes they must read (input + dy)."""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avtubes  # noqa: E402,F401
from avt_amd._lib import call, query  # noqa: E402


def P(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def S():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    args = ap.parse_args()
    dev = torch.device("cuda")
    N = args.batch
    for name, cin, cp, H, W in (("vision", 3, 4, 224, 224), ("audio", 1, 1, 257, 300)):
        K, R = 64, 7
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        x = torch.randn(N, H, W, cp, device=dev).to(torch.bfloat16)
        if cp > cin:
            x[..., cin:] = 0
        kg = (R * R * cp + 31) // 32 * 32
        w = torch.randn(K, R, R, cin, device=dev) * 0.05
        wf = torch.empty(K, kg, device=dev, dtype=torch.bfloat16)
        call("avt_pack_conv_weight", P(w), K, R, R, cin, cp, kg, P(wf), None, S())
        y = torch.empty(N, OH, OW, K, device=dev, dtype=torch.bfloat16)
        acc = torch.empty(int(query("avt_bn_acc_doubles", N * OH * OW, K)), device=dev, dtype=torch.float64)
        flops = 2.0 * N * OH * OW * K * R * R * cin
        out_bytes = 2.0 * N * OH * OW * K
        line = f"{name:7s} N={N}"
        for kern in (1, 0):
            call("avt_set_stem_kernel", kern)
            ms = timeit(lambda: call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, cp, K, R, R, 2, 3, kg,
                                     S()))
            line += (f" | kernel {kern}: {ms * 1e3:7.1f} us {flops / ms / 1e9:6.0f} TFLOP/s "
                     f"store {out_bytes / ms / 1e6:6.0f} GB/s")
        call("avt_set_stem_kernel", 1)
        print(line, flush=True)
        # wgrad: the per-wave stem kernel (+ its slab reduce) vs the generic gather kernel
        dy = torch.randn(N, OH, OW, K, device=dev).to(torch.bfloat16)
        dw = torch.zeros(K, R, R, cin, device=dev)
        in_bytes = 2.0 * N * H * W * cp + 2.0 * N * OH * OW * K
        line = f"{name:7s} wgrad"
        for kern in (1, 0):
            call("avt_set_stem_wgrad", kern)
            wsb = int(query("avt_conv2d_wgrad_workspace", N, H, W, cp, cin, K, R, R, 2, 3))
            ws = torch.empty(max(wsb, 1), device=dev, dtype=torch.uint8)
            ms = timeit(lambda: call("avt_conv2d_wgrad", P(x), P(dy), P(dw), N, H, W, cp, cin, K, R, R, 2, 3, P(ws),
                                     wsb, S()))
            line += (f" | kernel {kern}: {ms * 1e3:7.1f} us {flops / ms / 1e9:6.0f} TFLOP/s "
                     f"read {in_bytes / ms / 1e6:6.0f} GB/s")
        call("avt_set_stem_wgrad", 1)
        print(line, flush=True)


if __name__ == "__main__":
    main()
