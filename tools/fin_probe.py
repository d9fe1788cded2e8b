"""Where does a BN finalize cost its time?  Chains conv(+stats) -> finalize -> apply of one trunk shape,
captured in a HIP graph (20 links), in four forms:
  A  conv with BN atomics -> finalize -> apply      (the step's forward)
  B  conv with BN atomics -> apply                  (finalize left out)
  C  conv without stats   -> finalize of a separate, already-filled accumulator -> apply
  D  conv without stats   -> apply
A-B: the finalize behind pending atomics; C-D: a finalize alone; B-D: the atomics themselves.
usage: python tools/fin_probe.py [--batch 128] [--shape l1|l3] [--streams 1|2]"""
import argparse
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--shape", default="l1")
    ap.add_argument("--links", type=int, default=20)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import avtubes  # noqa: F401
    from avt_amd._lib import call, query

    dev = torch.device("cuda", 0)
    N = args.batch
    H, W, C = {"l1": (56, 56, 64), "l2": (28, 28, 128), "l3": (14, 14, 256), "al1": (65, 75, 64)}[args.shape]
    K, R = C, 3
    P = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, H, W, C, generator=g).relu().to(torch.bfloat16).to(dev)
    w = (torch.randn(K, R, R, C, generator=g) * 0.05).float().to(dev)
    kg = R * R * C
    wf = torch.empty(K, kg, device=dev, dtype=torch.bfloat16)
    call("avt_pack_conv_weight", P(w), K, R, R, C, C, kg, P(wf), None, ctypes.c_void_p(0))
    y = torch.empty(N, H, W, K, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(y)
    acc = torch.zeros(int(query("avt_bn_acc_doubles", K)), device=dev, dtype=torch.float64)
    acc2 = torch.zeros_like(acc)
    gamma, beta = torch.ones(K, device=dev), torch.zeros(K, device=dev)
    rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
    stats = torch.empty(4, K, device=dev)
    rows = N * H * W
    torch.cuda.synchronize()

    def S():
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def conv(with_acc):
        call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc) if with_acc else None, N, H, W, C, K, R, R, 1, 1, kg, S())

    def fin(a):
        call("avt_bn_finalize", P(a), rows, K, P(gamma), P(beta), P(rm), P(rv), ctypes.c_float(0.1),
             ctypes.c_float(1e-5), P(stats[0]), P(stats[1]), P(stats[2]), P(stats[3]), S())

    def refill():  # valid statistics in acc2 for form C (its finalize re-zeroes it)
        conv(True)
        acc2.copy_(acc)
        acc.zero_()

    def apply():
        call("avt_bn_apply", P(y), P(stats[0]), P(stats[1]), None, None, None, P(out), rows, K, 1, S())

    # eager pass: valid stats for the forms without a finalize
    conv(True)
    fin(acc)
    apply()
    torch.cuda.synchronize()
    forms = {
        "A conv+atomics -> fin -> apply": lambda: (conv(True), fin(acc), apply()),
        "B conv+atomics -> apply": lambda: (conv(True), apply()),
        "C conv -> fin(other acc) -> apply": lambda: (conv(False), fin(acc2), apply()),
        "D conv -> apply": lambda: (conv(False), apply()),
    }
    res = {}
    for name, body in forms.items():
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            gr.capture_begin()
            for _ in range(args.links):
                body()
            gr.capture_end()
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            if name.startswith("C"):
                refill()
            acc.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gr.replay()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e6 / args.links)
        res[name] = sorted(ts)[len(ts) // 2]
    print(f"B={N} {args.shape} ({N}x{H}x{W}x{C}): us per link: " +
          "  ".join(f"{k}: {v:.1f}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
