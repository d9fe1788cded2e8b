"""Repeat one conv launch on the same inputs and count distinct outputs (a data race inside the kernel shows as
more than one).  usage: python tools/diag_rep.py [N H W C K] [launches]   (env knobs select the kernel)"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avtubes  # noqa: E402,F401
from avt_amd._lib import call  # noqa: E402

a = [int(v) for v in sys.argv[1:6]] if len(sys.argv) > 5 else [32, 14, 14, 512, 512]
n_launch = int(sys.argv[6]) if len(sys.argv) > 6 else 60
N, H, W, C, K = a
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(5)
dy = torch.randn(N, H, W, K, generator=g).to(torch.bfloat16).to(dev)
w = (torch.randn(K, 3, 3, C, generator=g) * 0.05).to(dev)
wf = torch.empty(K, 9 * C, device=dev, dtype=torch.bfloat16)
wt = torch.empty(C, 9 * K, device=dev, dtype=torch.bfloat16)
S = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
call("avt_pack_conv_weight", P(w), K, 3, 3, C, C, 9 * C, P(wf), P(wt), S())
seen = {}
fresh = os.environ.get("REP_FRESH", "")  # rewrite the operands right before each launch (on the same stream)
dy0 = dy.clone()
for i in range(n_launch):
    if "w" in fresh:
        call("avt_pack_conv_weight", P(w), K, 3, 3, C, C, 9 * C, P(wf), P(wt), S())
    if "x" in fresh:
        dy.copy_(dy0)
    dx = torch.empty(N, H, W, C, device=dev, dtype=torch.bfloat16)
    call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, 3, 3, 1, 1, S())
    torch.cuda.synchronize()
    key = hash(dx.view(torch.int16).cpu().numpy().tobytes())
    seen.setdefault(key, []).append(i)
print(f"dgrad {a}: {len(seen)} distinct outputs over {n_launch} launches "
      f"({sorted(len(v) for v in seen.values())})", flush=True)
