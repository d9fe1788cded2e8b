"""Split-K form of the 3x3/s1 halo conv (short layer3/4 grids at a few clips per GPU): avt_conv2d_fwd_ws /
avt_conv2d_dgrad_ws against fp64 references of the same op (base_models.py:23-26 conv3x3, as
test_kernels_gpu.py), BN partial statistics included; repeated launches are bitwise identical (the
last-arriving block sums the partials in split order and leaves the tickets zero)."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from avt_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
_KEEP = []


@pytest.fixture(autouse=True)
def _release():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()
    call("avt_set_halo_splitk", 0, 0)


def P(t):
    if t is None:
        return None
    _KEEP.append(t)
    return ctypes.c_void_p(t.data_ptr())


def S():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _plan(N, H, W, C, K, dgrad):
    nf, nc = ctypes.c_longlong(0), ctypes.c_int(0)
    call("avt_conv2d_splitk_plan", N, H, W, C, K, 3, 3, 1, 1, int(dgrad), ctypes.byref(nf), ctypes.byref(nc))
    return nf.value, nc.value


CASES = [(3, 14, 14, 256, 256), (2, 17, 19, 512, 512), (32, 14, 14, 512, 512), (8, 14, 14, 256, 512),
         (5, 17, 19, 512, 256)]


@pytest.mark.parametrize("ks", [2, 4, 8])
@pytest.mark.parametrize("case", CASES)
def test_splitk_fwd(case, ks):
    N, H, W, C, K = case
    call("avt_set_halo_splitk", ks, 0)
    nf, nc = _plan(N, H, W, C, K, False)
    assert nc > 0 and nf % (nc * 128 * 128) == 0
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, H, W, C, generator=g).relu().to(torch.bfloat16)
    w = (torch.randn(K, 3, 3, C, generator=g) * (2.0 / (K * 9)) ** 0.5).float()
    kg = 9 * C
    wf = torch.empty(K, kg, device=DEV, dtype=torch.bfloat16)
    call("avt_pack_conv_weight", P(w.to(DEV)), K, 3, 3, C, C, kg, P(wf), None, S())
    xd = x.to(DEV)
    part = torch.empty(nf, device=DEV)
    cnt = torch.zeros(nc, device=DEV, dtype=torch.int32)
    outs = []
    for _ in range(2):
        y = torch.empty(N, H, W, K, device=DEV, dtype=torch.bfloat16)
        acc = torch.full((int(query("avt_bn_acc_doubles", N * H * W, K)),), float("nan"), device=DEV,
                         dtype=torch.float64)
        call("avt_conv2d_fwd_ws", P(xd), P(wf), P(y), P(acc), N, H, W, C, K, 3, 3, 1, 1, kg, P(part), part.numel(),
             P(cnt), cnt.numel(), S())
        torch.cuda.synchronize()
        outs.append((y, acc))
    assert cnt.abs().max().item() == 0  # tickets left zero for the next launch
    assert torch.equal(outs[0][0], outs[1][0])  # arrival order does not change the bits
    y, acc = outs[0]
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.to(torch.bfloat16).double().permute(0, 3, 1, 2),
                   padding=1).permute(0, 2, 3, 1)
    assert rel_err(y, ref) < 8e-3
    rows = ref.reshape(-1, K)
    n = rows.shape[0]
    ac = acc.cpu()
    ns = int(ac[0]) + int(ac[1])
    a = ac[8:8 + ns * K * 3].view(ns, K, 3).sum(0)  # the slots the header reports (include/avt.h)
    np.testing.assert_allclose(a[:, 0].numpy(), rows.sum(0).numpy(), rtol=1e-4,
                               atol=1e-4 * rows.abs().max().item() * n ** 0.5)
    m2 = a[:, 1] + a[:, 2] - a[:, 0] ** 2 / n
    np.testing.assert_allclose(m2.numpy(), ((rows - rows.mean(0)) ** 2).sum(0).numpy(), rtol=1e-4)


@pytest.mark.parametrize("mode", ["plain", "add", "mask"])
@pytest.mark.parametrize("ks", [2, 8])
@pytest.mark.parametrize("case", CASES)
def test_splitk_dgrad(case, ks, mode):
    N, H, W, C, K = case
    call("avt_set_halo_splitk", ks, 0)
    nf, nc = _plan(N, H, W, C, K, True)
    assert nc > 0
    g = torch.Generator().manual_seed(3)
    dy = torch.randn(N, H, W, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(K, 3, 3, C, generator=g) * (2.0 / (K * 9)) ** 0.5).float()
    add = torch.randn(N, H, W, C, generator=g).to(torch.bfloat16) if mode != "plain" else None
    bits = torch.randint(0, 256, (N * H * W * C // 8,), generator=g, dtype=torch.uint8) if mode == "mask" else None
    kg = 9 * C
    wf = torch.empty(K, kg, device=DEV, dtype=torch.bfloat16)
    wt = torch.empty(C, 9 * K, device=DEV, dtype=torch.bfloat16)
    call("avt_pack_conv_weight", P(w.to(DEV)), K, 3, 3, C, C, kg, P(wf), P(wt), S())
    dyd = dy.to(DEV)
    addd = add.to(DEV) if add is not None else None
    bitsd = bits.to(DEV) if bits is not None else None
    part = torch.empty(nf, device=DEV)
    cnt = torch.zeros(nc, device=DEV, dtype=torch.int32)
    outs = []
    for _ in range(2):
        dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
        call("avt_conv2d_dgrad_ws", P(dyd), P(wt), P(dx), P(addd), P(bitsd), N, H, W, C, K, 3, 3, 1, 1, P(part),
             part.numel(), P(cnt), cnt.numel(), S())
        torch.cuda.synchronize()
        outs.append(dx)
    assert cnt.abs().max().item() == 0
    assert torch.equal(outs[0], outs[1])
    ref = F.conv_transpose2d(dy.double().permute(0, 3, 1, 2), w.to(torch.bfloat16).double().permute(0, 3, 1, 2),
                             padding=1).permute(0, 2, 3, 1)
    ref = ref.to(torch.bfloat16).double()  # the kernel rounds the conv to bf16 before the add
    if add is not None:
        a = add.double()
        if bits is not None:
            m = ((bits.view(-1, 1).int() >> torch.arange(8).view(1, 8)) & 1).view(N, H, W, C).double()
            a = a * m
        ref = ref + a
    assert rel_err(outs[0], ref) < 8e-3


def test_splitk_workspace_too_small_runs_unsplit():
    """A workspace sized for one plan, called after the knobs changed to a larger one: the call
    re-plans, sees the plan does not fit and runs without split-K -- bitwise equal to avt_conv2d_fwd."""
    N, H, W, C, K = 2, 17, 19, 512, 512
    call("avt_set_halo_splitk", 2, 0)
    nf, nc = _plan(N, H, W, C, K, False)
    assert nc > 0
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, H, W, C, generator=g).relu().to(torch.bfloat16).to(DEV)
    w = (torch.randn(K, 3, 3, C, generator=g) * (2.0 / (K * 9)) ** 0.5).float()
    kg = 9 * C
    wf = torch.empty(K, kg, device=DEV, dtype=torch.bfloat16)
    call("avt_pack_conv_weight", P(w.to(DEV)), K, 3, 3, C, C, kg, P(wf), None, S())
    part = torch.empty(nf, device=DEV)
    cnt = torch.zeros(nc, device=DEV, dtype=torch.int32)
    call("avt_set_halo_splitk", 8, 0)  # needs 4x the partials the workspace holds
    y = torch.empty(N, H, W, K, device=DEV, dtype=torch.bfloat16)
    call("avt_conv2d_fwd_ws", P(x), P(wf), P(y), None, N, H, W, C, K, 3, 3, 1, 1, kg, P(part), part.numel(), P(cnt),
         cnt.numel(), S())
    call("avt_set_halo_splitk", 1, 0)
    y0 = torch.empty_like(y)
    call("avt_conv2d_fwd", P(x), P(wf), P(y0), None, N, H, W, C, K, 3, 3, 1, 1, kg, S())
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    assert cnt.abs().max().item() == 0
