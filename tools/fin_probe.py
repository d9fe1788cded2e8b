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
    ap.add_argument("--streams", type=int, default=1, help="2: a second chain (--shape2) concurrently on a "
                    "second stream, as the two trunks run")
    ap.add_argument("--shape2", default="al1")
    args = ap.parse_args()
    import avtubes  # noqa: F401
    from avt_amd._lib import call, query

    dev = torch.device("cuda", 0)
    N = args.batch
    P = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def S():
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def chain(shape, seed):
        H, W, C = {"l1": (56, 56, 64), "l2": (28, 28, 128), "l3": (14, 14, 256), "al1": (65, 75, 64),
                   "al3": (17, 19, 256)}[shape]
        K, R = C, 3
        g = torch.Generator().manual_seed(seed)
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
        keep = [x, w, wf, y, out, acc, acc2, gamma, beta, rm, rv, stats]

        def conv(with_acc):
            call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc) if with_acc else None, N, H, W, C, K, R, R, 1, 1, kg,
                 S())

        def fin(a):
            call("avt_bn_finalize", P(a), rows, K, P(gamma), P(beta), P(rm), P(rv), ctypes.c_float(0.1),
                 ctypes.c_float(1e-5), P(stats[0]), P(stats[1]), P(stats[2]), P(stats[3]), S())

        def apply():
            call("avt_bn_apply", P(y), P(stats[0]), P(stats[1]), None, None, None, P(out), rows, K, 1, S())

        def refill():
            conv(True)
            acc2.copy_(acc)
            acc.zero_()

        conv(True)
        fin(acc)
        apply()
        forms = {
            "A": lambda: (conv(True), fin(acc), apply()),
            "B": lambda: (conv(True), apply()),
            "C": lambda: (conv(False), fin(acc2), apply()),
            "D": lambda: (conv(False), apply()),
        }
        return forms, refill, acc, keep

    c1 = chain(args.shape, 0)
    c2 = chain(args.shape2, 1) if args.streams == 2 else None
    torch.cuda.synchronize()
    names = {"A": "A conv+atomics -> fin -> apply", "B": "B conv+atomics -> apply",
             "C": "C conv -> fin(other acc) -> apply", "D": "D conv -> apply"}
    res = {}
    for key, name in names.items():
        st = torch.cuda.Stream()
        st2 = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            gr.capture_begin()
            if c2 is not None:  # fork: the second chain on its own stream, joined at the end
                st2.wait_stream(st)
                with torch.cuda.stream(st2):
                    for _ in range(args.links):
                        c2[0][key]()
            for _ in range(args.links):
                c1[0][key]()
            if c2 is not None:
                st.wait_stream(st2)
            gr.capture_end()
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            for c in (c1, c2):
                if c is None:
                    continue
                if key == "C":
                    c[1]()
                c[2].zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gr.replay()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e6 / args.links)
        res[name] = sorted(ts)[len(ts) // 2]
    print(f"B={N} {args.shape}" + (f" || {args.shape2}" if c2 is not None else "") + ": us per link: " +
          "  ".join(f"{k}: {v:.1f}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
