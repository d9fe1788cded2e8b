"""Triangulate a Conv3d tap-gather mismatch: avt_conv3d_fwd (halo form off) vs fp64 torch over a grid of shapes and
tile configs.  Prints the relative error per case."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avtubes  # noqa: E402,F401
from avt_amd._lib import call, query  # noqa: E402
from avt_amd.trunk import P  # noqa: E402
import ctypes  # noqa: E402


def S():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run(N, T, H, W, C, K, cfg, halo3d=0, stats=False, fill=None):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, T, H, W, C, generator=g).relu().to(torch.bfloat16)
    w = (torch.randn(K, C, 3, 3, 3, generator=g) * (2.0 / (K * 27)) ** 0.5).float()
    wd = w.cuda()
    wp = torch.empty(K, 27 * C, device="cuda", dtype=torch.bfloat16)
    call("avt_pack_conv3d_weight", P(wd), P(wp), K, C, 3, 3, 3, 0, S())
    y = torch.empty(N, T, H, W, K, device="cuda", dtype=torch.bfloat16)
    if fill is not None:
        y.fill_(fill)
    acc = torch.full((int(query("avt_bn_acc_doubles", N * T * H * W, K)),), float("nan"), device="cuda",
                     dtype=torch.float64) if stats else None
    xd = x.cuda()
    call("avt_set_halo3d", halo3d)
    call("avt_set_nt128_config", cfg)
    call("avt_conv3d_fwd", P(xd), P(wp), P(y), P(acc) if stats else None, N, T, H, W, C, K, 3, 3, 3, 1, 1, 1, S())
    call("avt_set_halo3d", -1)
    call("avt_set_nt128_config", -1)
    ref = F.conv3d(x.double().permute(0, 4, 1, 2, 3), w.to(torch.bfloat16).double(), padding=1).permute(0, 2, 3, 4, 1)
    d = (y.cpu().double() - ref).abs()
    err = (d.max() / ref.abs().max()).item()
    bad = (d > 0.02 * ref.abs().max()).nonzero()
    where = ""
    if len(bad):
        b = bad[0].tolist()
        where = f" first bad (n,t,h,w,k)={b} of {len(bad)}; bad t values {sorted(set(bad[:, 1].tolist()))[:8]}" \
                f" k range {bad[:, 4].min().item()}-{bad[:, 4].max().item()}"
    if len(bad):
        rows = sorted(set((b[0] * T * H * W + b[1] * H * W + b[2] * W + b[3]) for b in bad[:, :4].tolist()))
        print(f"   bad output rows {rows[:6]} .. {rows[-6:]} ({len(rows)} rows), row tiles of 128: "
              f"{sorted(set(r // 128 for r in rows))}", flush=True)
    print(f"N{N} T{T} H{H} W{W} C{C} K{K} cfg{cfg} halo3d{halo3d} stats{int(stats)} fill{fill}: rel err {err:.3e}{where}",
          flush=True)


for st in (False, True):
    for fill in (None, 7.0):
        run(1, 7, 13, 17, 256, 128, -1, stats=st, fill=fill)
        run(1, 7, 13, 17, 256, 256, -1, stats=st, fill=fill)
        run(1, 7, 13, 17, 128, 128, -1, stats=st, fill=fill)
