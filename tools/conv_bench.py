"""Per-shape microbenchmark of the libavt conv kernels (fwd / dgrad / wgrad) at the B=128 trunk
shapes.  Prints TFLOP/s per (shape, kind[, variant]).  Usage: python tools/conv_bench.py [--batch 128]"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avtubes  # noqa: E402,F401
from avt_amd._lib import call, query  # noqa: E402

# (name, H, W, C, K, R, stride, pad)
SHAPES = [
    ("V.l1 3x3", 56, 56, 64, 64, 3, 1, 1),
    ("V.l2 3x3", 28, 28, 128, 128, 3, 1, 1),
    ("V.l2.0 s2", 56, 56, 64, 128, 3, 2, 1),
    ("V.l3 3x3", 14, 14, 256, 256, 3, 1, 1),
    ("V.l4 3x3", 14, 14, 512, 512, 3, 1, 1),
    ("V.l4.0 256", 14, 14, 256, 512, 3, 1, 1),
    ("A.l1 3x3", 65, 75, 64, 64, 3, 1, 1),
    ("A.l2 3x3", 33, 38, 128, 128, 3, 1, 1),
    ("A.l3 3x3", 17, 19, 256, 256, 3, 1, 1),
    ("A.l4 3x3", 17, 19, 512, 512, 3, 1, 1),
    ("A.ds 1x1s2", 33, 38, 128, 256, 1, 2, 0),
    ("V.ds2 1x1s2", 56, 56, 64, 128, 1, 2, 0),
    ("V.ds3 1x1s2", 28, 28, 128, 256, 1, 2, 0),
    ("V.ds4 1x1", 14, 14, 256, 512, 1, 1, 0),
    ("A.ds2 1x1s2", 65, 75, 64, 128, 1, 2, 0),
    ("A.ds4 1x1", 17, 19, 256, 512, 1, 1, 0),
]


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
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--kinds", default="fwd,dgrad,wgrad")
    ap.add_argument("--only", default="")
    ap.add_argument("--wgrad-policy", default="0,4", help="';'-separated target_blocks,min_kt (0 = wave model)")
    ap.add_argument("--slab-max", default="1073741824,16", help="avt_set_wgrad_slab_max(max_splits, wave_cost)")
    ap.add_argument("--wgrad-tiles", default="1", help="comma list of avt_set_wgrad_tiles values to sweep")
    ap.add_argument("--nt64", default="", help="comma list of avt_set_nt64_config values to sweep")
    ap.add_argument("--nt128", default="", help="comma list of avt_set_nt128_config values to sweep")
    ap.add_argument("--slab", type=int, default=1, help="wgrad split-K through a slab (1) or atomics (0)")
    ap.add_argument("--wgrad-halo", default="3", help="comma list of avt_set_wgrad_halo values to sweep")
    ap.add_argument("--row3-kg", default="2", help="comma list of avt_set_wgrad_row3 k-group values to sweep")
    ap.add_argument("--halo", default="", help="comma list of avt_set_halo values to sweep (fwd/dgrad)")
    ap.add_argument("--small", default="", help="comma list of avt_set_small_tiles values to sweep (fwd/dgrad)")
    ap.add_argument("--stages", default="", help="';'-separated nst128,nst64 pairs of avt_set_halo_stages to sweep")
    ap.add_argument("--splitk", default="", help="comma list of avt_set_halo_splitk values (0 = plan) to sweep")
    ap.add_argument("--wgrad-nst", default="4,3", help="';'-separated nst,nst_big pairs of avt_set_wgrad_nst to sweep")
    args = ap.parse_args()
    dev = torch.device("cuda")
    N = args.batch
    call("avt_set_wgrad_slab_max", *(int(v) for v in args.slab_max.split(",")))
    kinds = args.kinds.split(",")
    tot = {}
    for name, H, W, C, K, R, st, pad in SHAPES:
        if args.only and not any(o in name for o in args.only.split(",")):
            continue
        Pq, Qq = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        x = torch.randn(N, H, W, C, device=dev).relu().to(torch.bfloat16)
        dy = torch.randn(N, Pq, Qq, K, device=dev).to(torch.bfloat16)
        w = torch.randn(K, R, R, C, device=dev) * 0.05
        kg = R * R * C
        wf = torch.empty(K, kg, device=dev, dtype=torch.bfloat16)
        wt = torch.empty(C, R * R * K, device=dev, dtype=torch.bfloat16)
        call("avt_pack_conv_weight", P(w), K, R, R, C, C, kg, P(wf), P(wt), S())
        y = torch.empty(N, Pq, Qq, K, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(N, H, W, C, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(K, R, R, C, device=dev)
        acc = torch.empty(int(query("avt_bn_acc_doubles", N * Pq * Qq, K)), device=dev, dtype=torch.float64)
        flops = 2.0 * N * Pq * Qq * K * C * R * R
        line = f"{name:12s} M={N * Pq * Qq:7d} N={K:4d} K={kg:5d}"
        if args.halo and R == 3 and st == 1:
            for hv in [int(s) for s in args.halo.split(",")]:
                call("avt_set_halo", hv)
                call("avt_set_conv_variant", 1)
                ms = timeit(lambda: call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st, pad,
                                         kg, S()))
                line += f" | halo[{hv}] fwd {flops / ms / 1e9:6.0f}"
                ms = timeit(lambda: call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, R, R, st,
                                         pad, S()))
                line += f" dgrad {flops / ms / 1e9:6.0f}"
            call("avt_set_halo", 1)
        if args.small:
            for sv in [int(v) for v in args.small.split(",")]:
                call("avt_set_small_tiles", sv)
                ms = timeit(lambda: call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st, pad,
                                         kg, S()))
                line += f" | small[{sv}] fwd {flops / ms / 1e9:6.0f}"
                tot[(f"fwd_small{sv}", 1)] = tot.get((f"fwd_small{sv}", 1), 0) + ms
                ms = timeit(lambda: call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, R, R, st,
                                         pad, S()))
                line += f" dgrad {flops / ms / 1e9:6.0f}"
                tot[(f"dgrad_small{sv}", 1)] = tot.get((f"dgrad_small{sv}", 1), 0) + ms
            call("avt_set_small_tiles", -2)
        if args.stages and R == 3 and st == 1:
            for pair in args.stages.split(";"):
                call("avt_set_halo_stages", *(int(v) for v in pair.split(",")))
                ms = timeit(lambda: call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st, pad,
                                         kg, S()))
                line += f" | nst[{pair}] fwd {flops / ms / 1e9:6.0f}"
                ms = timeit(lambda: call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, R, R, st,
                                         pad, S()))
                line += f" dgrad {flops / ms / 1e9:6.0f}"
            call("avt_set_halo_stages", 2, 3)
        if args.splitk and R == 3 and st == 1:
            for ks in [int(v) for v in args.splitk.split(",")]:
                call("avt_set_halo_splitk", ks, 0)
                for dg in (0, 1):
                    nf, nc = ctypes.c_longlong(0), ctypes.c_int(0)
                    call("avt_conv2d_splitk_plan", N, H, W, C, K, 3, 3, 1, 1, dg, ctypes.byref(nf), ctypes.byref(nc))
                    part = torch.empty(max(1, nf.value), device=dev)
                    cnt = torch.zeros(max(1, nc.value), device=dev, dtype=torch.int32)
                    pp, pc = (P(part), P(cnt)) if nc.value else (None, None)
                    if dg == 0:
                        ms = timeit(lambda: call("avt_conv2d_fwd_ws", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R,
                                                 st, pad, kg, pp, part.numel(), pc, cnt.numel(), S()))
                        line += f" | sk[{ks}:{nc.value and nf.value // (nc.value * 16384)}] fwd {flops / ms / 1e9:6.0f}"
                    else:
                        ms = timeit(lambda: call("avt_conv2d_dgrad_ws", P(dy), P(wt), P(dx), None, None, N, H, W, C,
                                                 K, R, R, st, pad, pp, part.numel(), pc, cnt.numel(), S()))
                        line += f" dgrad {flops / ms / 1e9:6.0f}"
                    tot[(f"{'dgrad' if dg else 'fwd'}_sk{ks}", 1)] = tot.get((f"{'dgrad' if dg else 'fwd'}_sk{ks}", 1), 0) + ms
            call("avt_set_halo_splitk", 0, 0)
        if (args.nt64 or args.nt128) and args.halo:
            call("avt_set_halo", 0)  # the tap-gather configs on every shape
        if args.nt64 and K == 64 or args.nt64 and C == 64:
            for cfg in [int(s) for s in args.nt64.split(",")]:
                call("avt_set_nt64_config", cfg)
                call("avt_set_conv_variant", 1)
                if K == 64:
                    ms = timeit(lambda: call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st,
                                             pad, kg, S()))
                    line += f" | nt64[{cfg}] fwd {flops / ms / 1e9:6.0f}"
                if C == 64:
                    ms = timeit(lambda: call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, R, R, st,
                                             pad, S()))
                    line += f" nt64[{cfg}] dgrad {flops / ms / 1e9:6.0f}"
            call("avt_set_nt64_config", -1)
        if args.nt128 and K % 128 == 0 or args.nt128 and C % 128 == 0:
            for cfg in [int(s) for s in args.nt128.split(",")]:
                call("avt_set_nt128_config", cfg)
                call("avt_set_conv_variant", 1)
                if K % 128 == 0:
                    ms = timeit(lambda: call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st,
                                             pad, kg, S()))
                    line += f" | nt128[{cfg}] fwd {flops / ms / 1e9:6.0f}"
                if C % 128 == 0:
                    ms = timeit(lambda: call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, R, R, st,
                                             pad, S()))
                    line += f" nt128[{cfg}] dgrad {flops / ms / 1e9:6.0f}"
            call("avt_set_nt128_config", -1)
        call("avt_set_halo", 1)
        for v in [int(s) for s in args.variants.split(",")]:
            call("avt_set_conv_variant", v)
            if "fwd" in kinds:
                ms = timeit(lambda: call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st, pad,
                                         kg, S()))
                line += f" | v{v} fwd {flops / ms / 1e9:6.0f}"
                tot[("fwd", v)] = tot.get(("fwd", v), 0) + ms
            if "dgrad" in kinds:
                ms = timeit(lambda: call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, R, R, st, pad,
                                         S()))
                line += f" dgrad {flops / ms / 1e9:6.0f}"
                tot[("dgrad", v)] = tot.get(("dgrad", v), 0) + ms
            if "wgrad" in kinds and v == 1:
                for hv, big, kgv in [(int(h), int(t), int(g)) for h in args.wgrad_halo.split(",")
                                     for t in args.wgrad_tiles.split(",") for g in args.row3_kg.split(",")]:
                    call("avt_set_wgrad_halo", hv)
                    if args.row3_kg != "2":
                        call("avt_set_wgrad_row3", kgv, -1, -1)
                    call("avt_set_wgrad_tiles", big)
                    for nstp in args.wgrad_nst.split(";"):
                      if nstp != "4,3":  # (the default: also runs on a library without the setter)
                          call("avt_set_wgrad_nst", *(int(v) for v in nstp.split(",")))
                      for pol in args.wgrad_policy.split(";"):
                          tb, mk = (int(s) for s in pol.split(","))
                          call("avt_set_wgrad_policy", tb, mk)
                          wsb = int(query("avt_conv2d_wgrad_workspace", N, H, W, C, C, K, R, R, st, pad))
                          ws = torch.empty(max(1, wsb), device=dev, dtype=torch.uint8)
                          ms = timeit(lambda: call("avt_conv2d_wgrad", P(x), P(dy), P(dw), N, H, W, C, C, K, R, R, st,
                                                   pad, P(ws), wsb if args.slab else 0, S()))
                          line += f" wgrad[h{hv},t{big},g{kgv},{tb},{mk},n{nstp}] {flops / ms / 1e9:6.0f}"
                          key = f"wgrad_h{hv}_t{big}_g{kgv}_{pol}_n{nstp}"
                          tot[(key, v)] = tot.get((key, v), 0) + ms
                if args.wgrad_nst != "4,3":
                    call("avt_set_wgrad_nst", 4, 3)
                call("avt_set_wgrad_policy", 0, 4)
                call("avt_set_wgrad_tiles", 1)
                call("avt_set_wgrad_halo", -1)
        print(line + "  TFLOP/s", flush=True)
    call("avt_set_conv_variant", 1)
    print({f"{k}_v{v}": round(ms, 3) for (k, v), ms in tot.items()}, "ms total")


if __name__ == "__main__":
    main()
