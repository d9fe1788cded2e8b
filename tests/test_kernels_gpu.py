"""Per-op parity of the libavt HIP kernels (called through the C-ABI) against fp64 CPU
references of the same op on the same (bf16-rounded) inputs."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from avt_amd._lib import call, query  # noqa: E402


_KEEP = []  # device temporaries passed to the C-ABI stay alive until the test ends


@pytest.fixture(autouse=True)
def _keep_alive():
    yield
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    _KEEP.clear()


def P(t):
    if t is None:
        return None
    _KEEP.append(t)
    return ctypes.c_void_p(t.data_ptr())


def S():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


DEV = "cuda"


def D(t):
    """t on the GPU, kept alive: a temporary freed while its kernel is still queued (or whose block
    the caching allocator hands to the next argument) would alias another operand."""
    d = t.to(DEV)
    _KEEP.append(d)
    return d


def rel_err(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def conv_out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


def pack(w_ohwi, cp, kg, with_t=True):
    K, R, S_, C = w_ohwi.shape
    wf = torch.empty(K, kg, device=DEV, dtype=torch.bfloat16)
    wt = torch.empty(C, R * S_ * K, device=DEV, dtype=torch.bfloat16) if with_t else None
    call("avt_pack_conv_weight", P(w_ohwi), K, R, S_, C, cp, kg, P(wf), P(wt), S())
    return wf, wt


CONV_CASES = [
    # N, H, W, C, K, R, stride, pad
    (2, 9, 11, 64, 64, 3, 1, 1),
    (2, 9, 11, 64, 128, 3, 2, 1),
    (3, 7, 5, 128, 256, 1, 2, 0),
    (2, 5, 6, 256, 512, 3, 1, 1),
    (1, 17, 19, 512, 512, 3, 1, 1),
    (2, 15, 13, 64, 128, 1, 2, 0),
    # halo-reuse kernel shapes (3x3/s1, W up to 79): tiles spanning images, M tails
    (1, 56, 56, 64, 64, 3, 1, 1),
    (1, 65, 75, 64, 64, 3, 1, 1),
    (2, 33, 38, 128, 128, 3, 1, 1),
    (3, 14, 14, 256, 256, 3, 1, 1),
    (2, 17, 19, 512, 512, 3, 1, 1),
    (1, 7, 79, 64, 128, 3, 1, 1),
]


def _rand_act(N, H, W, C, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(N, H, W, C, generator=g).to(torch.bfloat16)


def fwd_acc(rows, K):
    """A conv's BN statistics accumulator (include/avt.h), NaN-filled: every slot the producer reports must
    be overwritten (a slot it left unwritten turns the sums into NaN)."""
    return torch.full((int(query("avt_bn_acc_doubles", rows, K)),), float("nan"), device=DEV, dtype=torch.float64)


def bwd_ws(rows, C):
    """A BN-backward workspace (avt_bn_bwd_workspace bytes), filled with 0xFF (NaN as doubles)."""
    return torch.full((int(query("avt_bn_bwd_workspace", rows, C)),), 255, device=DEV, dtype=torch.uint8)


def acc_sums(acc, C, W, bwd=False):
    """[C][W] sums over the slots the producer(s) recorded in the header (fwd W=3: sum, M2, sum^2/n; bwd W=2)."""
    a = acc.detach().cpu()
    a = a.view(torch.float64) if a.dtype == torch.uint8 else a
    n = int(a[0].item()) + int(a[1].item())
    base = 8 + (C if bwd else 0)
    return a[base:base + n * C * W].view(n, C, W).sum(0)


@pytest.fixture(params=[0, -1], ids=["tile128", "tile64"])
def tiles(request):
    """Run with the 128-row fwd/dgrad tiles, then with the 64-row small-batch tiles (avt_set_small_tiles)."""
    call("avt_set_small_tiles", request.param)
    yield request.param
    call("avt_set_small_tiles", -2)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_and_bn_partials(case, tiles):
    N, H, W, C, K, R, st, pad = case
    x = _rand_act(N, H, W, C, 1).relu()
    g = torch.Generator().manual_seed(2)
    w = (torch.randn(K, R, R, C, generator=g) * (2.0 / (K * R * R)) ** 0.5).float()
    Pq, Qq = conv_out(H, R, st, pad), conv_out(W, R, st, pad)
    kg = R * R * C
    wf, _ = pack(w.to(DEV), C, kg, with_t=False)
    xd = x.to(DEV)
    y = torch.empty(N, Pq, Qq, K, device=DEV, dtype=torch.bfloat16)
    acc = fwd_acc(N * Pq * Qq, K)
    call("avt_conv2d_fwd", P(xd), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st, pad, kg, S())
    torch.cuda.synchronize()
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.to(torch.bfloat16).double().permute(0, 3, 1, 2), stride=st,
                   padding=pad).permute(0, 2, 3, 1)
    assert rel_err(y, ref) < 8e-3
    rows = ref.reshape(-1, K)
    a = acc_sums(acc, K, 3)
    n = rows.shape[0]
    s_ref = rows.sum(0)
    m2_ref = ((rows - rows.mean(0)) ** 2).sum(0)
    np.testing.assert_allclose(a[:, 0].numpy(), s_ref.numpy(), rtol=1e-4, atol=1e-4 * rows.abs().max().item() * n ** 0.5)
    m2 = a[:, 1] + a[:, 2] - a[:, 0] ** 2 / n
    np.testing.assert_allclose(m2.numpy(), m2_ref.numpy(), rtol=1e-4)
    # finalize only reads the slots (the next producer launch overwrites them): a second finalize of the same
    # accumulator gives the same bits
    gamma = torch.ones(K, device=DEV)
    beta = torch.zeros(K, device=DEV)
    stats = torch.empty(4, K, device=DEV)
    before = acc.clone()
    for _ in range(2):
        prev = stats.clone()
        call("avt_bn_finalize", P(acc), n, K, P(gamma), P(beta), None, None, ctypes.c_float(0.1),
             ctypes.c_float(1e-5), P(stats[0]), P(stats[1]), P(stats[2]), P(stats[3]), S())
    torch.cuda.synchronize()
    assert torch.equal(acc.view(torch.int64), before.view(torch.int64))
    assert torch.equal(stats, prev)
    np.testing.assert_allclose(stats[2].cpu().double().numpy(), rows.mean(0).numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(stats[3].cpu().double().numpy(), (m2_ref / n + 1e-5).rsqrt().numpy(), rtol=1e-4)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_variants_bitwise_equal(case):
    """The LDS-DMA pipelined kernel and the register-staged one sum in the same order."""
    N, H, W, C, K, R, st, pad = case
    x = _rand_act(N, H, W, C, 31).relu().to(DEV)
    g = torch.Generator().manual_seed(32)
    w = (torch.randn(K, R, R, C, generator=g) * 0.05).float().to(DEV)
    wf, wt = pack(w, C, R * R * C)
    Pq, Qq = conv_out(H, R, st, pad), conv_out(W, R, st, pad)
    dy = _rand_act(N, Pq, Qq, K, 33).to(DEV)
    outs = []
    call("avt_set_halo", 0)  # the halo kernel sums (chunk, tap) in another order: test_halo_matches_gather
    try:
        for variant in (0, 1):
            call("avt_set_conv_variant", variant)
            y = torch.empty(N, Pq, Qq, K, device=DEV, dtype=torch.bfloat16)
            call("avt_conv2d_fwd", P(x), P(wf), P(y), None, N, H, W, C, K, R, R, st, pad, R * R * C, S())
            dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
            call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), P(x), N, H, W, C, K, R, R, st, pad, S())
            outs.append((y, dx))
    finally:
        call("avt_set_conv_variant", 1)
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    # every tile / k-depth / stage config of the pipelined kernel accumulates in the same k order
    try:
        for knob, cfgs in (("avt_set_nt128_config", range(7)), ("avt_set_nt64_config", range(9))):
            for cfg in cfgs:
                call(knob, cfg)
                y = torch.empty(N, Pq, Qq, K, device=DEV, dtype=torch.bfloat16)
                call("avt_conv2d_fwd", P(x), P(wf), P(y), None, N, H, W, C, K, R, R, st, pad, R * R * C, S())
                dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
                call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), P(x), N, H, W, C, K, R, R, st, pad, S())
                torch.cuda.synchronize()
                assert torch.equal(y, outs[0][0]), (knob, cfg)
                assert torch.equal(dx, outs[0][1]), (knob, cfg)
    finally:
        call("avt_set_nt128_config", -1)
        call("avt_set_nt64_config", -1)
        call("avt_set_halo", 1)


@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[5] == 3 and c[6] == 1])
def test_halo_matches_gather(case):
    """Halo-reuse and tap-gather kernels agree to fp32-summation-order noise (bf16 outputs)."""
    N, H, W, C, K, R, st, pad = case
    x = _rand_act(N, H, W, C, 41).relu().to(DEV)
    g = torch.Generator().manual_seed(42)
    w = (torch.randn(K, R, R, C, generator=g) * 0.05).float().to(DEV)
    wf, wt = pack(w, C, R * R * C)
    dy = _rand_act(N, H, W, K, 43).to(DEV)
    outs = []
    try:
        for halo, halo8 in ((0, 1), (1, 0), (1, 1), (2, 1)):
            call("avt_set_halo", halo)
            call("avt_set_halo8", halo8)
            y = torch.empty(N, H, W, K, device=DEV, dtype=torch.bfloat16)
            acc = fwd_acc(N * H * W, K)
            call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st, pad, R * R * C, S())
            dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
            call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), P(x), N, H, W, C, K, R, R, st, pad, S())
            torch.cuda.synchronize()
            outs.append((y.float(), dx.float(), acc_sums(acc, K, 3)))
    finally:
        call("avt_set_halo", 1)
        call("avt_set_halo8", -1)
    (y0, dx0, a0) = outs[0]
    # 4-wave 128x128 and 8-wave 256x128 halo forms for W <= 19 (avt_set_halo8), the 8-wave forms for W <= 79
    for y1, dx1, a1 in outs[1:]:
        assert rel_err(y1, y0) < 1e-2 and rel_err(dx1, dx0) < 1e-2
        assert (y1 - y0).abs().gt(0).float().mean().item() < 0.1  # mostly bit-equal after bf16 rounding
        torch.testing.assert_close(a1[:, 0], a0[:, 0], rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("case", [(3, 14, 14, 256, 256, 3, 1, 1), (2, 17, 19, 512, 512, 3, 1, 1),
                                  (2, 5, 6, 256, 512, 3, 1, 1), (5, 14, 14, 512, 512, 3, 1, 1)])
def test_halo_stages_bitwise_equal(case):
    """The halo kernels' weight-ring depth (avt_set_halo_stages) changes only the load pipeline: every
    setting of both tiles (128-row, and 64-row via avt_set_small_tiles(-1)) gives bitwise-equal outputs
    and BN partial sums."""
    N, H, W, C, K, R, st, pad = case
    x = _rand_act(N, H, W, C, 51).relu().to(DEV)
    g = torch.Generator().manual_seed(52)
    w = (torch.randn(K, R, R, C, generator=g) * 0.05).float().to(DEV)
    wf, wt = pack(w, C, R * R * C)
    dy = _rand_act(N, H, W, K, 53).to(DEV)
    call("avt_set_halo8", 0)  # the ring-depth knob applies to the 4-wave 128 x 128 tile
    try:
        for small in (0, -1):
            call("avt_set_small_tiles", small)
            outs = []
            for nst in ((2, 2), (3, 3), (2, 4), (2, 5)):
                call("avt_set_halo_stages", *nst)
                y = torch.empty(N, H, W, K, device=DEV, dtype=torch.bfloat16)
                acc = fwd_acc(N * H * W, K)
                call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st, pad, R * R * C, S())
                dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
                call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, R, R, st, pad, S())
                torch.cuda.synchronize()
                outs.append((y.view(torch.int16).clone(), dx.view(torch.int16).clone(), acc_sums(acc, K, 3)[:, 0]))
            for o in outs[1:]:
                assert torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1])
                torch.testing.assert_close(o[2], outs[0][2], rtol=1e-9, atol=1e-6)
    finally:
        call("avt_set_halo_stages", 2, 3)
        call("avt_set_small_tiles", -2)
        call("avt_set_halo8", -1)


@pytest.mark.parametrize("N,H,W", [(3, 56, 56), (2, 65, 75), (21, 56, 56), (1, 7, 95)])
def test_c64_matches_gather(N, H, W):
    """Layer-1 persistent resident-weight kernel (avt_set_c64) vs the tap-gather kernel: fwd + BN partials,
    dgrad, dgrad + add, dgrad + masked add; partial last tiles and more tiles than CUs (N=21 at 56^2)."""
    C = K = 64
    x = _rand_act(N, H, W, C, 51).relu().to(DEV)
    g = torch.Generator().manual_seed(52)
    w = (torch.randn(K, 3, 3, C, generator=g) * 0.05).float().to(DEV)
    wf, wt = pack(w, C, 9 * C)
    dy = _rand_act(N, H, W, K, 53).to(DEV)
    add = _rand_act(N, H, W, C, 54).to(DEV)
    bits = torch.randint(0, 256, (N * H * W * C // 8,), generator=torch.Generator().manual_seed(55),
                         dtype=torch.uint8).to(DEV)
    outs = []
    try:
        for on in (0, 1):
            call("avt_set_c64", on)
            y = torch.empty(N, H, W, K, device=DEV, dtype=torch.bfloat16)
            acc = fwd_acc(N * H * W, K)
            call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, 3, 3, 1, 1, 9 * C, S())
            dx, dxa, dxm = (torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16) for _ in range(3))
            call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, 3, 3, 1, 1, S())
            call("avt_conv2d_dgrad", P(dy), P(wt), P(dxa), P(add), N, H, W, C, K, 3, 3, 1, 1, S())
            call("avt_conv2d_dgrad_mask", P(dy), P(wt), P(dxm), P(add), P(bits), N, H, W, C, K, 3, 3, 1, 1, S())
            torch.cuda.synchronize()
            a = acc_sums(acc, K, 3)
            n = N * H * W
            outs.append((y.float(), dx.float(), dxa.float(), dxm.float(), a[:, 0], a[:, 1] + a[:, 2] - a[:, 0] ** 2 / n))
    finally:
        call("avt_set_c64", 1)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2).cpu(), w.to(torch.bfloat16).double().permute(0, 3, 1, 2).cpu(),
                   padding=1).permute(0, 2, 3, 1)
    assert rel_err(outs[1][0], ref) < 8e-3
    refd = torch.nn.grad.conv2d_input((N, C, H, W), w.to(torch.bfloat16).double().permute(0, 3, 1, 2).cpu(),
                                      dy.double().permute(0, 3, 1, 2).cpu(), padding=1).permute(0, 2, 3, 1)
    assert rel_err(outs[1][1], refd) < 8e-3
    keep = ((bits.cpu().long().unsqueeze(1) >> torch.arange(8)) & 1).bool().reshape(N, H, W, C)
    assert rel_err(outs[1][2], refd + add.double().cpu()) < 8e-3
    assert rel_err(outs[1][3], refd + torch.where(keep, add.cpu(), torch.zeros_like(add.cpu())).double()) < 8e-3
    for k in range(4):  # same products, another fp32 summation order: bf16 outputs mostly bit-equal
        assert rel_err(outs[1][k], outs[0][k]) < 1e-2
        assert (outs[1][k] - outs[0][k]).abs().gt(0).float().mean().item() < 0.1
    rows = ref.reshape(-1, K)
    torch.testing.assert_close(outs[1][4].cpu(), rows.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(outs[1][5].cpu(), ((rows - rows.mean(0)) ** 2).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("cin,cp,H,W,N", [(3, 4, 20, 22, 2), (1, 1, 21, 17, 2), (3, 4, 224, 224, 2),
                                           (1, 1, 257, 300, 2), (3, 4, 224, 224, 7), (1, 1, 257, 300, 16)])
def test_stem_fwd_wgrad(cin, cp, H, W, N):
    """Both stem forward kernels (the persistent LDS-patch one -- several chunks per block at the larger
    N -- and the generic gather kernel) vs fp64, with their BN partial statistics; then the wgrad."""
    K, R, st, pad = 64, 7, 2, 3
    g = torch.Generator().manual_seed(3)
    x = torch.randn(N, cin, H, W, generator=g)
    xd = x.to(DEV)
    xn = torch.empty(N, H, W, cp, device=DEV, dtype=torch.bfloat16)
    call("avt_nchw_to_nhwc_bf16", P(xd), P(xn), N, cin, H, W, cp, S())
    w = (torch.randn(K, R, R, cin, generator=g) * 0.05).float()
    kg = (R * R * cp + 31) // 32 * 32
    wf, _ = pack(w.to(DEV), cp, kg, with_t=False)
    Pq, Qq = conv_out(H, R, st, pad), conv_out(W, R, st, pad)
    y = torch.empty(N, Pq, Qq, K, device=DEV, dtype=torch.bfloat16)
    xb = x.to(torch.bfloat16).double()
    wb = w.to(torch.bfloat16).double().permute(0, 3, 1, 2)
    ref = F.conv2d(xb, wb, stride=st, padding=pad).permute(0, 2, 3, 1)
    rows = ref.reshape(-1, K)
    n = rows.shape[0]
    outs = []
    try:
        for stem_kernel in (1, 0):  # the persistent LDS-patch stem kernel and the generic gather kernel
            call("avt_set_stem_kernel", stem_kernel)
            acc = fwd_acc(N * Pq * Qq, K)
            call("avt_conv2d_fwd", P(xn), P(wf), P(y), P(acc), N, H, W, cp, K, R, R, st, pad, kg, S())
            torch.cuda.synchronize()
            assert rel_err(y, ref) < 8e-3, stem_kernel
            a = acc_sums(acc, K, 3)
            # the stem kernel takes the statistics of the bf16 tensor it stores (on the MFMA pipe,
            # conv_stem.h), the generic kernel those of the fp32 values before rounding
            srows = y.reshape(-1, K).double().cpu() if stem_kernel else rows
            np.testing.assert_allclose(a[:, 0].numpy(), srows.sum(0).numpy(), rtol=1e-4,
                                       atol=1e-4 * srows.abs().max().item() * n ** 0.5)
            m2 = a[:, 1] + a[:, 2] - a[:, 0] ** 2 / n
            np.testing.assert_allclose(m2.numpy(), ((srows - srows.mean(0)) ** 2).sum(0).numpy(), rtol=1e-4)
            outs.append(y.clone())
    finally:
        call("avt_set_stem_kernel", 1)
    assert (outs[0].float() - outs[1].float()).abs().gt(0).float().mean().item() < 0.05
    assert torch.equal(xn[..., :cin].float().cpu(), x.to(torch.bfloat16).permute(0, 2, 3, 1).float())
    dy = _rand_act(N, Pq, Qq, K, 4)
    ref_dw = torch.nn.grad.conv2d_weight(xb, (K, cin, R, R), dy.double().permute(0, 3, 1, 2), stride=st, padding=pad)
    init = torch.randn(K, R, R, cin, generator=g).to(DEV)  # wgrad accumulates into dw
    dws = []
    try:
        # the per-wave stem wgrad kernel (twice: deterministic), the generic kernel, and the generic
        # kernel's atomics path (no workspace)
        for stem_wgrad, slab in ((1, True), (1, True), (0, True), (1, False)):
            call("avt_set_stem_wgrad", stem_wgrad)
            dw = init.clone()
            wgrad(xn, dy.to(DEV), dw, N, H, W, cp, cin, K, R, st, pad, slab=slab)
            torch.cuda.synchronize()
            assert rel_err((dw - init).permute(0, 3, 1, 2), ref_dw) < 2e-4, (stem_wgrad, slab)
            dws.append(dw)
    finally:
        call("avt_set_stem_wgrad", 1)
    assert torch.equal(dws[0], dws[1])


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad(case, tiles):
    N, H, W, C, K, R, st, pad = case
    Pq, Qq = conv_out(H, R, st, pad), conv_out(W, R, st, pad)
    dy = _rand_act(N, Pq, Qq, K, 5)
    g = torch.Generator().manual_seed(6)
    w = (torch.randn(K, R, R, C, generator=g) * 0.05).float()
    _, wt = pack(w.to(DEV), C, R * R * C)
    dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    call("avt_conv2d_dgrad", P(D(dy)), P(wt), P(dx), None, N, H, W, C, K, R, R, st, pad, S())
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.to(torch.bfloat16).double().permute(0, 3, 1, 2),
                                     dy.double().permute(0, 3, 1, 2), stride=st, padding=pad).permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    assert rel_err(dx, ref) < 8e-3
    # accumulate path: dx2 = dgrad + add
    add = _rand_act(N, H, W, C, 7)
    dx2 = torch.empty_like(dx)
    call("avt_conv2d_dgrad", P(D(dy)), P(wt), P(dx2), P(D(add)), N, H, W, C, K, R, R, st, pad, S())
    torch.cuda.synchronize()
    assert rel_err(dx2, ref + add.double()) < 8e-3
    # masked accumulate (identity block: dx = dgrad + g * [out > 0] from avt_bn_apply_mask's bits): bitwise
    # equal to the plain accumulate of the pre-masked add
    bits = torch.randint(0, 256, (N * H * W * C // 8,), generator=torch.Generator().manual_seed(8), dtype=torch.uint8)
    keep = ((bits.long().unsqueeze(1) >> torch.arange(8)) & 1).bool().reshape(N, H, W, C)
    addm = torch.where(keep, add, torch.zeros_like(add))
    dx3, dx4 = torch.empty_like(dx), torch.empty_like(dx)
    call("avt_conv2d_dgrad", P(D(dy)), P(wt), P(dx3), P(D(addm)), N, H, W, C, K, R, R, st, pad, S())
    call("avt_conv2d_dgrad_mask", P(D(dy)), P(wt), P(dx4), P(D(add)), P(D(bits)), N, H, W, C, K, R, R, st, pad, S())
    torch.cuda.synchronize()
    assert torch.equal(dx3, dx4)


@pytest.mark.parametrize("case", [(2, 9, 11, 64, 128, 3, 2, 1), (3, 7, 5, 128, 256, 1, 2, 0),
                                  (32, 56, 56, 64, 128, 3, 2, 1), (32, 33, 38, 128, 256, 3, 2, 1),
                                  (5, 65, 75, 64, 128, 1, 2, 0), (1, 2, 3, 64, 64, 3, 2, 1)])
def test_strided_dgrad_one_launch(case, tiles):
    """The stride-2 dgrad's parity classes in one launch (avt_set_s2_dgrad_one(1), the default) against one
    launch per class: bitwise equal, with and without an accumulated add, and accumulating in place."""
    N, H, W, C, K, R, st, pad = case
    Pq, Qq = conv_out(H, R, st, pad), conv_out(W, R, st, pad)
    dy = D(_rand_act(N, Pq, Qq, K, 15))
    w = (torch.randn(K, R, R, C, generator=torch.Generator().manual_seed(16)) * 0.05).float()
    _, wt = pack(w.to(DEV), C, R * R * C)
    add = D(_rand_act(N, H, W, C, 17))
    outs = []
    try:
        for one in (1, 0):
            call("avt_set_s2_dgrad_one", one)
            dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
            dxa = torch.empty_like(dx)
            dxi = add.clone()
            call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, R, R, st, pad, S())
            call("avt_conv2d_dgrad", P(dy), P(wt), P(dxa), P(add), N, H, W, C, K, R, R, st, pad, S())
            call("avt_conv2d_dgrad", P(dy), P(wt), P(dxi), P(dxi), N, H, W, C, K, R, R, st, pad, S())
            torch.cuda.synchronize()
            outs.append((dx, dxa, dxi))
    finally:
        call("avt_set_s2_dgrad_one", 1)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.to(DEV).to(torch.bfloat16).double().permute(0, 3, 1, 2),
                                     dy.double().permute(0, 3, 1, 2), stride=st, padding=pad).permute(0, 2, 3, 1)
    assert rel_err(outs[0][0], ref) < 8e-3
    assert rel_err(outs[0][1], ref + add.double()) < 8e-3


def wgrad(x, dy, dw, N, H, W, cp, creal, K, R, st, pad, slab=True):
    wsb = int(query("avt_conv2d_wgrad_workspace", N, H, W, cp, creal, K, R, R, st, pad)) if slab else 0
    ws = torch.empty(max(wsb, 1), device=DEV, dtype=torch.uint8)
    call("avt_conv2d_wgrad", P(x), P(dy), P(dw), N, H, W, cp, creal, K, R, R, st, pad, P(ws) if slab else None, wsb,
         S())


@pytest.mark.parametrize("nst", [(4, 3), (8, 5), (6, 4)], ids=["ring4", "ring8", "ring6"])
@pytest.mark.parametrize("big", [1, 0, "halo", "halo3", "halo3k2", "halo3k2np", "halo3k4"])
@pytest.mark.parametrize("slab", [True, False])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_wgrad(case, slab, big, nst):
    """big: the 256-wide tap-gather tiles (1), 128-wide only (0), or the halo-reuse kernel for the
    3x3/s1 cases, nine taps ("halo") or one filter row ("halo3") per block (off by default;
    conv_wgrad_halo.h).  nst: ring depth of the 4-wave / 8-wave tap-gather tiles (avt_set_wgrad_nst;
    the deep rings change the split plan too).  With the slab every form is run twice: bitwise equal."""
    if str(big).startswith("halo") and nst != (4, 3):
        pytest.skip("ring depth does not apply to the halo wgrad")
    hv = {"halo": 1, "halo3": 2, "halo3k2": 2, "halo3k2np": 2, "halo3k4": 2}.get(big, 0)
    N, H, W, C, K, R, st, pad = case
    Pq, Qq = conv_out(H, R, st, pad), conv_out(W, R, st, pad)
    x = _rand_act(N, H, W, C, 8).relu()
    dy = _rand_act(N, Pq, Qq, K, 9)
    dw = torch.full((K, R, R, C), 0.25, device=DEV)  # accumulates into an existing gradient
    dw2 = dw.clone()
    try:
        call("avt_set_wgrad_tiles", 1 if hv else big)
        call("avt_set_wgrad_halo", hv)
        call("avt_set_wgrad_row3", {"halo3k2": 2, "halo3k2np": 2, "halo3k4": 4}.get(big, 1), -1,
             0 if big == "halo3k2np" else 1)
        call("avt_set_wgrad_nst", *nst)
        xd, dyd = x.to(DEV), dy.to(DEV)
        wgrad(xd, dyd, dw, N, H, W, C, C, K, R, st, pad, slab)
        if slab:
            wgrad(xd, dyd, dw2, N, H, W, C, C, K, R, st, pad, slab)
    finally:
        call("avt_set_wgrad_tiles", 1)
        call("avt_set_wgrad_halo", -1)  # back to the environment defaults (AVT_WGRAD_HALO, AVT_ROW3_*)
        call("avt_set_wgrad_row3", -1, -1, -1)
        call("avt_set_wgrad_nst", 4, 3)
    ref = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (K, C, R, R), dy.double().permute(0, 3, 1, 2),
                                      stride=st, padding=pad)
    torch.cuda.synchronize()
    assert rel_err(dw.permute(0, 3, 1, 2) - 0.25, ref) < 2e-4
    if slab:
        assert torch.equal(dw, dw2)


FUSED_WGRAD_CASES = CONV_CASES + [
    # the 32-clip shard's layer2-4 and shortcut wgrads (the slab's split counts the fused reduce targets)
    (32, 14, 14, 256, 256, 3, 1, 1), (32, 17, 19, 256, 256, 3, 1, 1), (8, 14, 14, 512, 512, 3, 1, 1),
    (32, 28, 28, 128, 128, 3, 1, 1), (32, 28, 28, 128, 256, 1, 2, 0), (16, 14, 14, 256, 512, 3, 1, 1),
]
# shapes whose plan takes the fused reduce (moderate split counts; a 256 x 256 tile split 14 ways reads 3.4 MB of
# partials in its last block, past the 2 MB default bound, and keeps the separate reduce)
FUSED_EXPECTED = {(32, 14, 14, 256, 256, 3, 1, 1), (32, 17, 19, 256, 256, 3, 1, 1), (8, 14, 14, 512, 512, 3, 1, 1)}


@pytest.mark.parametrize("tiles", [1, 0])
@pytest.mark.parametrize("case", FUSED_WGRAD_CASES)
def test_conv_wgrad_fused_reduce(case, tiles):
    """avt_conv2d_wgrad_tk (an A/B knob, avt_set_wgrad_fused(1); off by default: measured slower): the last block of
    each output tile sums the split partials into dw (write-through
    partials, agent-scope tickets).  Against fp64, run twice (bitwise: the tickets are left zero and the summation order
    is fixed), and against the separate reduce launch (avt_conv2d_wgrad): the same split order, so equal up to the
    reduce's wave grouping of a few-tile slab (G > 1)."""
    N, H, W, C, K, R, st, pad = case
    Pq, Qq = conv_out(H, R, st, pad), conv_out(W, R, st, pad)
    xd, dyd = _rand_act(N, H, W, C, 12).relu().to(DEV), _rand_act(N, Pq, Qq, K, 13).to(DEV)
    try:
        call("avt_set_wgrad_tiles", tiles)
        call("avt_set_wgrad_fused", 1, -1)
        call("avt_set_wgrad_slots_pct", 100)  # FUSED_EXPECTED: the split counts of the whole-chip plan
        nt = int(query("avt_conv2d_wgrad_tickets", N, H, W, C, C, K, R, R, st, pad))
        wsb = int(query("avt_conv2d_wgrad_workspace", N, H, W, C, C, K, R, R, st, pad))
        ws = torch.empty(max(wsb, 1), device=DEV, dtype=torch.uint8)
        tk = torch.zeros(max(nt, 1), device=DEV, dtype=torch.int32)
        outs = []
        for fused in (True, True, False):
            dw = torch.full((K, R, R, C), 0.25, device=DEV)
            call("avt_conv2d_wgrad_tk", P(xd), P(dyd), P(dw), N, H, W, C, C, K, R, R, st, pad, P(ws), wsb,
                 P(tk) if fused else None, nt if fused else 0, S())
            outs.append(dw)
        torch.cuda.synchronize()
    finally:
        call("avt_set_wgrad_tiles", 1)
        call("avt_set_wgrad_fused", -1, -1)
        call("avt_set_wgrad_slots_pct", -1)
    if case in FUSED_EXPECTED:
        assert nt > 0, "the fused reduce should apply to this shape"
    assert int(tk.abs().sum()) == 0, "tickets not left zero"
    ref = torch.nn.grad.conv2d_weight(xd.cpu().double().permute(0, 3, 1, 2), (K, C, R, R),
                                      dyd.cpu().double().permute(0, 3, 1, 2), stride=st, padding=pad)
    assert rel_err(outs[0].permute(0, 3, 1, 2) - 0.25, ref) < 2e-4
    assert torch.equal(outs[0], outs[1])
    d = (outs[0] - outs[2]).abs().max().item()
    print(f"{case} tiles={tiles} tickets={nt}: |fused - separate| = {d:.3e}")
    assert d <= 1e-6 * outs[2].abs().max().item()


def test_wgrad_slot_share_auto():
    """The split planner's slot share (avt_set_wgrad_slots_pct): auto is 65 % of the chip's block slots at a batch of
    <= 32, 75 % at <= 64 and 100 % above (the other trunk's kernels run beside a wgrad): the workspace (the plan's slab) of auto is the
    fixed share's at each batch size; out-of-range shares are refused."""
    shapes = [(14, 14, 512, 512, 3, 1, 1), (17, 19, 256, 256, 3, 1, 1), (28, 28, 128, 128, 3, 1, 1)]
    try:
        for H, W, C, K, R, st, pad in shapes:
            ws = {}
            for N in (32, 64, 128):
                for pct in (0, 65, 75, 100):
                    call("avt_set_wgrad_slots_pct", pct)
                    ws[N, pct] = int(query("avt_conv2d_wgrad_workspace", N, H, W, C, C, K, R, R, st, pad))
            assert ws[32, 0] == ws[32, 65] and ws[64, 0] == ws[64, 75] and ws[128, 0] == ws[128, 100], ws
        with pytest.raises(RuntimeError):
            call("avt_set_wgrad_slots_pct", 101)
    finally:
        call("avt_set_wgrad_slots_pct", -1)


def test_wgrad_deferred_batched_reduce():
    """avt_conv2d_wgrad_defer leaves each wgrad's slab (where its reduce would run one wave per position) and one
    avt_wgrad_reduce_batch sums them all: bitwise equal to the per-wgrad reduce launches (the same split order), dw
    untouched by the reduce until the batch runs, and more slabs than one launch takes (24) split over launches."""
    from avt_amd._lib import SlabReduceDesc

    shapes = [(32, 14, 14, 256, 256, 3, 1, 1), (8, 14, 14, 512, 512, 3, 1, 1), (32, 28, 28, 128, 128, 3, 1, 1),
              (32, 28, 28, 128, 256, 1, 2, 0), (3, 14, 14, 256, 256, 3, 1, 1), (2, 17, 19, 512, 512, 3, 1, 1)] * 8  # 4 of the 6 shapes split K
    keep, descs, refs, outs = [], [], [], []
    call("avt_set_wgrad_slots_pct", 100)  # the whole-chip plan's split counts (4 of the 6 shapes split)
    for n, (N, H, W, C, K, R, st, pad) in enumerate(shapes):
        Pq, Qq = conv_out(H, R, st, pad), conv_out(W, R, st, pad)
        xd, dyd = _rand_act(N, H, W, C, 40 + n).relu().to(DEV), _rand_act(N, Pq, Qq, K, 80 + n).to(DEV)
        wsb = int(query("avt_conv2d_wgrad_workspace", N, H, W, C, C, K, R, R, st, pad))
        ws = torch.empty(max(wsb, 1), device=DEV, dtype=torch.uint8)
        ref = torch.full((K, R, R, C), 0.25, device=DEV)
        call("avt_conv2d_wgrad", P(xd), P(dyd), P(ref), N, H, W, C, C, K, R, R, st, pad, P(ws), wsb, S())
        torch.cuda.synchronize()
        dw = torch.full((K, R, R, C), 0.25, device=DEV)
        ws2 = torch.empty(max(wsb, 1), device=DEV, dtype=torch.uint8)
        d = SlabReduceDesc()
        call("avt_conv2d_wgrad_defer", P(xd), P(dyd), P(dw), N, H, W, C, C, K, R, R, st, pad, P(ws2), wsb,
             ctypes.byref(d), S())
        keep += [xd, dyd, ws, ws2]
        refs.append(ref)
        outs.append(dw)
        if d.splits > 0:
            descs.append(d)
    call("avt_set_wgrad_slots_pct", -1)
    assert len(descs) > 24, len(descs)
    torch.cuda.synchronize()
    # before the batch: a deferred dw holds only the initial value
    untouched = [o for o in outs if torch.all(o == 0.25)]
    assert len(untouched) == len(descs)
    arr = (SlabReduceDesc * len(descs))(*descs)
    call("avt_wgrad_reduce_batch", arr, len(descs), S())
    torch.cuda.synchronize()
    for n, (o, r) in enumerate(zip(outs, refs)):
        assert torch.equal(o, r), (n, shapes[n], (o - r).abs().max().item())


def test_wgrad_large_splitk():
    # many pixels -> split-K with fp32 atomics
    N, H, W, C, K, R, st, pad = 8, 56, 56, 64, 64, 3, 1, 1
    x = _rand_act(N, H, W, C, 10).relu()
    dy = _rand_act(N, H, W, K, 11)
    dw = torch.zeros(K, R, R, C, device=DEV)
    wgrad(x.to(DEV), dy.to(DEV), dw, N, H, W, C, C, K, R, st, pad)
    ref = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (K, C, R, R), dy.double().permute(0, 3, 1, 2),
                                      stride=st, padding=pad)
    torch.cuda.synchronize()
    assert rel_err(dw.permute(0, 3, 1, 2), ref) < 2e-4


# ------------------------------------------------------------------------------------------ BN
def _tile_acc(c):
    """The accumulator a conv epilogue would leave (include/avt.h): header (slot count) + per 128-row tile t
    its own slot (sum_t, M2_t, sum_t^2/n_t) (fp64)."""
    rows = c.double().reshape(-1, c.shape[-1])
    C = rows.shape[1]
    ts = list(range(0, rows.shape[0], 128))
    acc = torch.zeros(len(ts), C, 3, dtype=torch.float64)
    for i, t in enumerate(ts):
        blk = rows[t:t + 128]
        s = blk.sum(0)
        acc[i, :, 0] = s
        acc[i, :, 1] = ((blk - blk.mean(0)) ** 2).sum(0)
        acc[i, :, 2] = s * s / blk.shape[0]
    hdr = torch.zeros(8, dtype=torch.float64)
    hdr[0] = len(ts)
    return torch.cat([hdr, acc.reshape(-1)])


@pytest.mark.parametrize("shape", [(2, 9, 11, 64), (4, 5, 7, 512), (3, 33, 38, 128)])
def test_bn_forward_train(shape):
    N, H, W, C = shape
    c = (_rand_act(N, H, W, C, 12).float() * 1.7 + 0.3).to(torch.bfloat16)
    res = _rand_act(N, H, W, C, 13)
    g = torch.Generator().manual_seed(14)
    gamma = 1 + 0.02 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    rm, rv = torch.zeros(C), torch.ones(C)
    acc = _tile_acc(c).to(DEV)
    stats = torch.empty(4, C, device=DEV)
    rmd, rvd = rm.to(DEV), rv.to(DEV)
    rows = N * H * W
    call("avt_bn_finalize", P(acc), rows, C, P(D(gamma)), P(D(beta)), P(rmd), P(rvd),
         ctypes.c_float(0.1), ctypes.c_float(1e-5), P(stats[0]), P(stats[1]), P(stats[2]), P(stats[3]), S())
    out = torch.empty_like(c, device=DEV)
    call("avt_bn_apply", P(D(c)), P(stats[0]), P(stats[1]), P(D(res)), None, None, P(out), rows, C, 1, S())
    torch.cuda.synchronize()
    cn = c.double().permute(0, 3, 1, 2)
    rm64, rv64 = rm.double(), rv.double()
    ref = F.batch_norm(cn, rm64, rv64, gamma.double(), beta.double(), True, 0.1, 1e-5)
    ref = (ref + res.double().permute(0, 3, 1, 2)).relu().permute(0, 2, 3, 1)
    assert rel_err(out, ref) < 8e-3
    np.testing.assert_allclose(rmd.cpu().numpy(), rm64.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(rvd.cpu().numpy(), rv64.numpy(), rtol=1e-4, atol=1e-5)


def test_bn_finalize_tall():
    """The forward finalize over 8200 tile slots (a GEMM of 2^20 rows: the tube step's 16-frame stem and
    layer1 have ~12.5 k), against the fp64 statistics of the same rows."""
    T, C = 8200, 64
    g = torch.Generator().manual_seed(21)
    rows = (torch.randn(T * 128, C, generator=g) * 1.3 + 0.4).to(torch.bfloat16).double()
    blk = rows.view(T, 128, C)
    s = blk.sum(1)
    acc = torch.stack([s, ((blk - blk.mean(1, keepdim=True)) ** 2).sum(1), s * s / 128], dim=2)
    hdr = torch.zeros(8, dtype=torch.float64)
    hdr[0] = T
    accd = torch.cat([hdr, acc.reshape(-1)]).to(DEV)
    gamma = torch.ones(C, device=DEV)
    beta = torch.zeros(C, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    stats = torch.empty(4, C, device=DEV)
    call("avt_bn_finalize", P(accd), T * 128, C, P(gamma), P(beta), P(rm), P(rv), ctypes.c_float(0.1),
         ctypes.c_float(1e-5), P(stats[0]), P(stats[1]), P(stats[2]), P(stats[3]), S())
    torch.cuda.synchronize()
    mean, var = rows.mean(0), rows.var(0, unbiased=False)
    np.testing.assert_allclose(stats[2].cpu().double().numpy(), mean.numpy(), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(stats[3].cpu().double().numpy(), (1 / (var + 1e-5).sqrt()).numpy(), rtol=1e-6)
    np.testing.assert_allclose(rv.cpu().double().numpy(), (0.9 + 0.1 * rows.var(0, unbiased=True)).numpy(),
                               rtol=1e-6)


@pytest.mark.parametrize("shape", [(2, 9, 11, 64), (4, 5, 7, 512), (3, 33, 38, 128)])
@pytest.mark.parametrize("masked", [True, False])
def test_bn_backward(shape, masked):
    N, H, W, C = shape
    c = (_rand_act(N, H, W, C, 15).float() * 1.3 - 0.2).to(torch.bfloat16)
    gy = _rand_act(N, H, W, C, 16)
    g = torch.Generator().manual_seed(17)
    gamma = 1 + 0.02 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    cn = c.double().permute(0, 3, 1, 2).requires_grad_(True)
    gm = gamma.double().requires_grad_(True)
    bt = beta.double().requires_grad_(True)
    yb = F.batch_norm(cn, None, None, gm, bt, True, 0.1, 1e-5)
    y = yb.relu() if masked else yb
    y.backward(gy.double().permute(0, 3, 1, 2))
    mean = c.double().reshape(-1, C).mean(0)
    var = c.double().reshape(-1, C).var(0, unbiased=False)
    inv = (var + 1e-5).rsqrt()
    yd = y.detach().permute(0, 2, 3, 1).to(torch.bfloat16).to(DEV).contiguous()
    rows = N * H * W
    ws = bwd_ws(rows, C)
    dgamma = torch.zeros(C, device=DEV)
    dbeta = torch.zeros(C, device=DEV)
    gc = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    gmask = torch.empty_like(gc)
    call("avt_bn_bwd", P(D(gy)), P(yd if masked else None), P(D(c)), P(D(mean.float())),
         P(D(inv.float())), P(D(gamma)), P(dgamma), P(dbeta), P(gc), P(gmask), P(ws), rows, C, S())
    torch.cuda.synchronize()
    assert rel_err(gc, cn.grad.permute(0, 2, 3, 1)) < 2e-2
    assert rel_err(dgamma, gm.grad) < 1e-2
    assert rel_err(dbeta, bt.grad) < 1e-3


@pytest.mark.parametrize("shape", [(2, 9, 11, 64), (4, 5, 7, 512), (3, 33, 38, 128), (2, 17, 19, 256)])
@pytest.mark.parametrize("two", [False, True])
def test_bn_mask_bits_fwd_bwd(shape, two):
    """avt_bn_apply_mask = avt_bn_apply + the ReLU bits of out; avt_bn_bwd_mask (one BN, or bn2 +
    downsample.1 sharing g') = avt_bn_bwd fed y = out, per BN; and the fp64 autograd of the block's
    relu(bn2(c2) + bnd(cd))."""
    N, H, W, C = shape
    rows = N * H * W
    c = (_rand_act(N, H, W, C, 31).float() * 1.3 - 0.2).to(torch.bfloat16)
    cd = (_rand_act(N, H, W, C, 32).float() * 0.9 + 0.1).to(torch.bfloat16)
    gy = _rand_act(N, H, W, C, 33)
    g = torch.Generator().manual_seed(34)
    gam, bet = 1 + 0.02 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    gam2, bet2 = 1 + 0.02 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    st, st2 = _bn_batch_stats(c, gam, bet), _bn_batch_stats(cd, gam2, bet2)
    cdev, cddev, gydev = D(c), D(cd), D(gy)
    res = (P(cddev), P(st2[0]), P(st2[1])) if two else (P(cddev), None, None)
    y = torch.empty_like(cdev)
    y2 = torch.empty_like(cdev)
    bits = torch.empty(rows * C // 8, device=DEV, dtype=torch.uint8)
    call("avt_bn_apply", P(cdev), P(st[0]), P(st[1]), *res, P(y), rows, C, 1, S())
    call("avt_bn_apply_mask", P(cdev), P(st[0]), P(st[1]), *res, P(y2), P(bits), rows, C, S())
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    pos = (y.float() > 0).reshape(-1, 8).cpu().long()
    assert torch.equal(bits.cpu().long(), (pos << torch.arange(8)).sum(1))
    from avt_amd._lib import BnBwdTarget

    def target(xc, s, gamma):
        t = BnBwdTarget()
        t.keep = [torch.zeros(C, device=DEV), torch.zeros(C, device=DEV), torch.empty_like(xc),
                  bwd_ws(rows, C), D(gamma)]
        t.xc, t.mean, t.invstd, t.gamma = xc.data_ptr(), s[2].data_ptr(), s[3].data_ptr(), t.keep[4].data_ptr()
        t.dgamma, t.dbeta, t.gc, t.workspace = [k.data_ptr() for k in t.keep[:4]]
        return t

    t1 = target(cdev, st, gam)
    t2 = target(cddev, st2, gam2) if two else None
    call("avt_bn_bwd_mask", P(gydev), P(bits), ctypes.byref(t1), ctypes.byref(t2) if two else None, rows, C, S())
    torch.cuda.synchronize()
    for t, xc, s, gamma in ([(t1, cdev, st, gam)] + ([(t2, cddev, st2, gam2)] if two else [])):
        ws = bwd_ws(rows, C)
        dg, db, gc = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV), torch.empty_like(xc)
        call("avt_bn_bwd", P(gydev), P(y), P(xc), P(s[2]), P(s[3]), P(D(gamma)), P(dg), P(db), P(gc), None, P(ws),
             rows, C, S())
        torch.cuda.synchronize()
        # same mask and sums; the two reduce kernels sum in different orders (k1/k2 an ulp -> a bf16 ulp of gc)
        torch.testing.assert_close(t.keep[2].float(), gc.float(), rtol=8e-3, atol=1e-4)
        torch.testing.assert_close(t.keep[0], dg, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(t.keep[1], db, rtol=1e-5, atol=1e-6)
    # fp64 autograd of the block output relu(bn2(c) + [bnd(cd) | cd])
    cn = c.double().permute(0, 3, 1, 2).requires_grad_(True)
    cdn = cd.double().permute(0, 3, 1, 2).requires_grad_(True)
    gm, bt = gam.double().requires_grad_(True), bet.double().requires_grad_(True)
    gm2, bt2 = gam2.double().requires_grad_(True), bet2.double().requires_grad_(True)
    r = F.batch_norm(cdn, None, None, gm2, bt2, True, 0.1, 1e-5) if two else cdn
    (F.batch_norm(cn, None, None, gm, bt, True, 0.1, 1e-5) + r).relu().backward(gy.double().permute(0, 3, 1, 2))
    assert rel_err(t1.keep[2], cn.grad.permute(0, 2, 3, 1)) < 2e-2
    assert rel_err(t1.keep[0], gm.grad) < 1e-2
    assert rel_err(t1.keep[1], bt.grad) < 1e-3
    if two:
        assert rel_err(t2.keep[2], cdn.grad.permute(0, 2, 3, 1)) < 2e-2
        assert rel_err(t2.keep[0], gm2.grad) < 1e-2
        assert rel_err(t2.keep[1], bt2.grad) < 1e-3


def _bn_batch_stats(c, gamma, beta):
    """fp32 (scale, shift, mean, invstd) of train-mode BN over NHWC c, as avt_bn_finalize makes them."""
    C = c.shape[-1]
    mean = c.double().reshape(-1, C).mean(0)
    inv = (c.double().reshape(-1, C).var(0, unbiased=False) + 1e-5).rsqrt()
    scale = (gamma.double() * inv).float()
    shift = (beta.double() - mean * scale.double()).float()
    return torch.stack([scale, shift, mean.float(), inv.float()]).to(DEV)


@pytest.mark.parametrize("shape", [(2, 9, 11, 64), (4, 5, 7, 512), (3, 33, 38, 128)])
def test_bn_relu_bwd(shape):
    """BasicBlock.bn1 backward with the ReLU mask recomputed from (c, scale, shift): equals avt_bn_bwd
    fed the avt_bn_apply output as y, and the fp64 autograd of relu(batch_norm(c))."""
    N, H, W, C = shape
    c = (_rand_act(N, H, W, C, 21).float() * 1.3 - 0.2).to(torch.bfloat16)
    gy = _rand_act(N, H, W, C, 22)
    g = torch.Generator().manual_seed(23)
    gamma = 1 + 0.02 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    st = _bn_batch_stats(c, gamma, beta)
    rows = N * H * W
    cd, gyd, gmd = c.to(DEV), gy.to(DEV), gamma.to(DEV)
    y = torch.empty_like(cd)
    call("avt_bn_apply", P(cd), P(st[0]), P(st[1]), None, None, None, P(y), rows, C, 1, S())
    outs = []
    for fused in (True, False):
        ws = bwd_ws(rows, C)
        dgamma, dbeta = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        gc = torch.empty_like(cd)
        if fused:
            call("avt_bn_relu_bwd", P(gyd), P(cd), P(st[0]), P(st[1]), P(st[2]), P(st[3]), P(gmd), P(dgamma),
                 P(dbeta), P(gc), P(ws), rows, C, S())
        else:
            call("avt_bn_bwd", P(gyd), P(y), P(cd), P(st[2]), P(st[3]), P(gmd), P(dgamma), P(dbeta), P(gc), None,
                 P(ws), rows, C, S())
        torch.cuda.synchronize()
        outs.append((gc.float(), dgamma, dbeta))
    # same mask and sums, reduced in different orders (k1/k2 an ulp -> a bf16 ulp of gc)
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=8e-3, atol=1e-4)
    for a, b in zip(outs[0][1:], outs[1][1:]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    cn = c.double().permute(0, 3, 1, 2).requires_grad_(True)
    gm = gamma.double().requires_grad_(True)
    bt = beta.double().requires_grad_(True)
    F.batch_norm(cn, None, None, gm, bt, True, 0.1, 1e-5).relu().backward(gy.double().permute(0, 3, 1, 2))
    assert rel_err(outs[0][0], cn.grad.permute(0, 2, 3, 1)) < 2e-2
    assert rel_err(outs[0][1], gm.grad) < 1e-2
    assert rel_err(outs[0][2], bt.grad) < 1e-3


@pytest.mark.parametrize("shape", [(2, 12, 14, 64), (2, 129, 150, 64), (1, 7, 9, 64), (3, 112, 112, 64), (2, 9, 192, 64)])
def test_stem_fused(shape):
    """Stem bn1 -> relu -> maxpool fused both ways (base_models.py:200-203).  fwd: bitwise equal to
    avt_bn_apply + avt_maxpool3s2_fwd, carg = c at the argmax; bwd: fp64 autograd reference."""
    N, H, W, C = shape
    c = (_rand_act(N, H, W, C, 24).float() * 1.5 - 0.3).to(torch.bfloat16)
    g = torch.Generator().manual_seed(25)
    gamma = 1 + 0.02 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    st = _bn_batch_stats(c, gamma, beta)
    cd = c.to(DEV)
    P2, Q2 = conv_out(H, 3, 2, 1), conv_out(W, 3, 2, 1)
    y = torch.empty(N, P2, Q2, C, device=DEV, dtype=torch.bfloat16)
    idx = torch.empty(N, P2, Q2, C, device=DEV, dtype=torch.uint8)
    carg = torch.empty_like(y)
    call("avt_stem_bn_relu_maxpool_fwd", P(cd), P(st[0]), P(st[1]), P(y), P(idx), P(carg), N, H, W, C, S())
    h = torch.empty_like(cd)
    call("avt_bn_apply", P(cd), P(st[0]), P(st[1]), None, None, None, P(h), N * H * W, C, 1, S())
    y2, idx2 = torch.empty_like(y), torch.empty_like(idx)
    call("avt_maxpool3s2_fwd", P(h), P(y2), P(idx2), N, H, W, C, S())
    torch.cuda.synchronize()
    assert torch.equal(y, y2) and torch.equal(idx, idx2)
    # carg == c at (2p-1+idx//3, 2q-1+idx%3)
    ii = idx.long().cpu()
    hh = (2 * torch.arange(P2).view(1, P2, 1, 1) - 1 + ii // 3).clamp(0, H - 1)
    ww = (2 * torch.arange(Q2).view(1, 1, Q2, 1) - 1 + ii % 3).clamp(0, W - 1)
    nn_ = torch.arange(N).view(N, 1, 1, 1).expand_as(ii)
    cc = torch.arange(C).view(1, 1, 1, C).expand_as(ii)
    assert torch.equal(carg.cpu(), c[nn_, hh, ww, cc])

    gy = _rand_act(N, P2, Q2, C, 26)
    ws = bwd_ws(N * H * W, C)
    dgamma, dbeta = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    gc = torch.empty_like(cd)
    call("avt_stem_maxpool_bn_relu_bwd", P(D(gy)), P(idx), P(carg), P(cd), P(st[0]), P(st[1]), P(st[2]),
         P(st[3]), P(D(gamma)), P(dgamma), P(dbeta), P(gc), P(ws), N, H, W, C, S())
    torch.cuda.synchronize()
    cn = c.double().permute(0, 3, 1, 2).requires_grad_(True)
    gm = gamma.double().requires_grad_(True)
    bt = beta.double().requires_grad_(True)
    hr = F.batch_norm(cn, None, None, gm, bt, True, 0.1, 1e-5).relu()
    # route the pool through the kernel's bf16 activation values (straight-through), so bf16 ties
    # pick the same (first) window position; the gradient itself stays fp64
    hk = h.cpu().double().permute(0, 3, 1, 2)
    hr = hr + (hk - hr).detach()
    F.max_pool2d(hr, 3, 2, 1).backward(gy.double().permute(0, 3, 1, 2))
    assert rel_err(gc, cn.grad.permute(0, 2, 3, 1)) < 2e-2
    assert rel_err(dgamma, gm.grad) < 1e-2
    assert rel_err(dbeta, bt.grad) < 1e-3


# ------------------------------------------------------------------------------------------ pools
@pytest.mark.parametrize("shape", [(2, 12, 14, 64), (2, 129, 150, 64), (1, 7, 9, 64)])
def test_maxpool(shape):
    N, H, W, C = shape
    x = _rand_act(N, H, W, C, 18).relu()  # post-ReLU, many ties at 0 like the stem
    P2, Q2 = conv_out(H, 3, 2, 1), conv_out(W, 3, 2, 1)
    y = torch.empty(N, P2, Q2, C, device=DEV, dtype=torch.bfloat16)
    idx = torch.empty(N, P2, Q2, C, device=DEV, dtype=torch.uint8)
    xd = x.to(DEV)
    call("avt_maxpool3s2_fwd", P(xd), P(y), P(idx), N, H, W, C, S())
    gy = _rand_act(N, P2, Q2, C, 19)
    gx = torch.empty_like(xd)
    call("avt_maxpool3s2_bwd", P(D(gy)), P(idx), P(gx), N, H, W, C, S())
    xn = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xn, 3, 2, 1)
    yr.backward(gy.double().permute(0, 3, 1, 2))
    torch.cuda.synchronize()
    assert torch.equal(y.cpu().double(), yr.detach().permute(0, 2, 3, 1))
    # gradients: exact except where a window has tied maxima (routing may differ); ties only at 0
    # here and those positions are masked by the ReLU backward in the real network.
    ref = xn.grad.permute(0, 2, 3, 1)
    nz = x.double() > 0
    assert rel_err(gx.cpu().double() * nz, ref * nz) < 8e-3


@pytest.mark.parametrize("B,HW,C", [(3, 323, 512), (5, 25, 512), (2, 7, 64)])
def test_audio_pool_norm(B, HW, C):
    a = _rand_act(B, HW, 1, C, 20).reshape(B, HW, C)
    an = torch.empty(B, C, device=DEV)
    amax = torch.empty(B, C, device=DEV, dtype=torch.int32)
    anorm = torch.empty(B, device=DEV)
    ad = a.to(DEV)
    call("avt_audio_pool_norm_fwd", P(ad), P(an), P(amax), P(anorm), B, HW, C, S())
    g = torch.Generator().manual_seed(21)
    gan = torch.randn(B, C, generator=g)
    ga = torch.empty_like(ad)
    call("avt_audio_pool_norm_bwd", P(D(gan)), P(an), P(amax), P(anorm), P(ga), B, HW, C, S())
    at = a.double().permute(0, 2, 1).reshape(B, C, HW, 1).requires_grad_(True)
    r = F.normalize(F.adaptive_max_pool2d(at, 1).flatten(1), dim=1)
    r.backward(gan.double())
    torch.cuda.synchronize()
    assert rel_err(an, r.detach()) < 1e-6
    assert rel_err(ga, at.grad.reshape(B, C, HW).permute(0, 2, 1)) < 8e-3


# ------------------------------------------------------------------------------------------ head
def _head_inputs(B, h, w, C, seed):
    g = torch.Generator().manual_seed(seed)
    v = (torch.randn(B, h, w, C, generator=g).abs() + 0.3 * torch.rand(B, 1, 1, C, generator=g)).to(torch.bfloat16)
    an = F.normalize(torch.randn(B, C, generator=g).abs() + 0.5, dim=1)
    return v, an


@pytest.mark.parametrize("B,h,w,trimap,neg", [(2, 14, 14, True, True), (8, 14, 14, True, True), (5, 4, 4, False, True),
                                           (3, 7, 9, True, False), (40, 14, 14, True, True)])
def test_hardway_head(B, h, w, trimap, neg):
    import avenet_oracle as orc

    C = 512
    v, an = _head_inputs(B, h, w, C, 22)
    Pn = h * w
    dev = dict(device=DEV, dtype=torch.float32)
    L = B + (2 if neg else 1)
    inv, vsum = torch.empty(B, Pn, **dev), torch.empty(B, Pn, **dev)
    A0 = torch.empty(B, Pn, B, **dev)
    save = torch.empty(int(query("avt_hardway_save_floats", B)), **dev)
    logits, A, Pos, Neg, wA = (torch.empty(B, L, **dev), torch.empty(B, Pn, **dev), torch.empty(B, Pn, **dev),
                               torch.empty(B, Pn, **dev), torch.empty(B, Pn, **dev))
    vd, and_ = v.to(DEV), an.to(DEV)
    call("avt_hardway_fwd", P(vd), P(and_), B, Pn, C, 0.65, 0.4, 0.03, int(trimap), int(neg), P(inv), P(vsum), P(A0),
         P(save), P(logits), P(A), P(Pos), P(Neg), P(wA), S())
    loss = torch.empty((), **dev)
    dl = torch.empty(B, L, **dev)
    call("avt_hardway_ce", P(logits), B, L, 1.0, P(loss), P(dl), S())
    dA0 = torch.empty(B, Pn, B, **dev)
    dvh = torch.empty(B, Pn, C, **dev)
    gv = torch.empty_like(vd)
    gan = torch.empty(B, C, **dev)
    call("avt_hardway_bwd", P(vd), P(and_), P(inv), P(A0), P(save), P(dl), B, Pn, C, 0.65, 0.4, 0.03, int(trimap),
         int(neg), None, None, None, P(dA0), P(dvh), P(gv), P(gan), 0, S())
    torch.cuda.synchronize()
    # fp64 oracle on the same (bf16) features
    vt = v.double().permute(0, 3, 1, 2).requires_grad_(True)
    at = an.double().requires_grad_(True)
    img_n = F.normalize(vt, dim=1)
    rA, rlog, rwA, rPos, rNeg = orc.hardway_head(img_n, at, 0.65, 0.4, 0.03, trimap, neg)
    rloss = orc.hardway_ce(rlog)
    rloss.backward()
    assert (A.cpu().double() - rA.detach().reshape(B, Pn)).abs().max() < 1e-5
    assert (logits.cpu().double() - rlog.detach()).abs().max() < 2e-3
    assert abs(loss.item() - rloss.item()) < 1e-5 * max(1.0, abs(rloss.item()))
    assert (Pos.cpu().double() - rPos.detach().reshape(B, Pn)).abs().max() < 1e-3
    assert (Neg.cpu().double() - rNeg.detach().reshape(B, Pn)).abs().max() < 1e-3
    assert (wA.cpu().double() - rwA.detach().reshape(B, Pn)).abs().max() < 1e-5
    assert rel_err(gan, at.grad) < 2e-3
    assert rel_err(gv, vt.grad.permute(0, 2, 3, 1)) < 1e-2


def test_pack_batched_matches_single():
    """avt_pack_conv_weights_batched (vector fwd copy + LDS-tiled dgrad transpose) == the per-conv
    pack, bitwise, incl. the padded stem layout, a misaligned source and partial 64x64 tiles."""
    import struct
    # K, R, C, Cp, Kg, flat offset (floats)
    cases = [(64, 7, 3, 4, 224, 0), (64, 7, 1, 1, 64, 9408), (128, 3, 64, 64, 576, 12544),
             (96, 3, 40, 40, 360, 86272), (256, 1, 128, 128, 128, 120833), (512, 3, 512, 512, 4608, 153604)]
    total = max(o + K * R * R * C for K, R, C, _, _, o in cases)
    g = torch.Generator().manual_seed(40)
    flat = torch.randn(total, generator=g).to(DEV)
    descs, singles, outs, maxel = [], [], [], 0
    for K, R, C, Cp, Kg, o in cases:
        w = flat[o:o + K * R * R * C]
        wf = torch.empty(K, Kg, device=DEV, dtype=torch.bfloat16)
        wt = torch.empty(C, R * R * K, device=DEV, dtype=torch.bfloat16) if C == Cp else None
        descs.append(struct.pack("<QQQiiiiii", w.data_ptr(), wf.data_ptr(), 0 if wt is None else wt.data_ptr(),
                                 K, R * R, C, Cp, Kg, 0))
        maxel = max(maxel, K * Kg + (0 if wt is None else wt.numel()))
        outs.append((wf, wt))
        sf, st_ = torch.empty_like(wf), (torch.empty_like(wt) if wt is not None else None)
        call("avt_pack_conv_weight", P(w), K, R, R, C, Cp, Kg, P(sf), P(st_), S())
        singles.append((sf, st_))
    table = torch.frombuffer(bytearray(b"".join(descs)), dtype=torch.uint8).to(DEV)
    call("avt_pack_conv_weights_batched", P(table), len(descs), maxel, S())
    torch.cuda.synchronize()
    for (wf, wt), (sf, st_) in zip(outs, singles):
        assert torch.equal(wf, sf)
        if wt is not None:
            assert torch.equal(wt, st_)


def test_adam_matches_torch():
    import avenet_oracle as orc

    g = torch.Generator().manual_seed(23)
    n = 1001
    p0 = torch.randn(n, generator=g)
    opt = orc.AdamRef(lr=1e-3, weight_decay=1e-4)
    pr = {"p": p0.clone().double()}
    pd = p0.clone().to(DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    for t in range(1, 4):
        gr = torch.randn(n, generator=g)
        opt.step(pr, {"p": gr.double()})
        call("avt_adam_step", P(pd), P(D(gr)), P(m), P(v), n, 1.0, 1e-3, 0.9, 0.999, 1e-8, 1e-4, t, S())
    torch.cuda.synchronize()
    assert rel_err(pd - p0.to(DEV), pr["p"] - p0.double()) < 1e-4


def _dgrad_bn_ref(g, xc, stats, y=None):
    """Reference of the fused BN-backward epilogue from the plain dgrad result g (bf16): the mask, the
    masked gradient and the fp64 sums (sum g', sum g' * xhat) per channel."""
    g, xc = g.double().cpu(), xc.double().cpu()
    sc, sh, mean, inv = (stats[i].double().cpu() for i in range(4))
    mask = (y.double().cpu() > 0) if y is not None else (xc.float() * sc.float() + sh.float() > 0)
    gm = torch.where(mask, g, torch.zeros_like(g))
    xhat = (xc - mean) * inv
    C = g.shape[-1]
    return gm, gm.reshape(-1, C).sum(0), (gm * xhat).reshape(-1, C).sum(0)


def _bn_stats_rand(C, seed):
    g = torch.Generator().manual_seed(seed)
    sc = 1.0 + 0.2 * torch.randn(C, generator=g)
    sh = 0.3 * torch.randn(C, generator=g)
    mean = 0.1 * torch.randn(C, generator=g)
    inv = 1.0 + 0.5 * torch.rand(C, generator=g)
    return torch.stack([sc, sh, mean, inv]).float()


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("mode", ["relu_fma", "mask_y", "two_bn"])
def test_conv_dgrad_bn_epilogue(case, mode):
    """avt_conv2d_dgrad_bn: the store epilogue masks the dgrad result by the BN's ReLU (recomputed from
    (xc, scale, shift) or read from y) and accumulates that BN's backward reductions (and a second
    BN's) -- bitwise the masked plain-dgrad result, sums == fp64 sums of it; then
    avt_bn_bwd_premasked consumes the accumulator like avt_bn_bwd."""
    # the epilogue lives in the tap-gather / halo kernels, which the small-tile path never picks for it:
    # compare like with like
    call("avt_set_c64", 0)
    call("avt_set_small_tiles", 0)
    try:
        _dgrad_bn_epilogue(case, mode)
    finally:
        call("avt_set_c64", 1)
        call("avt_set_small_tiles", -2)


def _dgrad_bn_epilogue(case, mode):
    N, H, W, C, K, R, st, pad = case
    Pq, Qq = conv_out(H, R, st, pad), conv_out(W, R, st, pad)
    dy = _rand_act(N, Pq, Qq, K, 15)
    g = torch.Generator().manual_seed(16)
    w = (torch.randn(K, R, R, C, generator=g) * 0.05).float()
    _, wt = pack(w.to(DEV), C, R * R * C)
    add = _rand_act(N, H, W, C, 17) if mode != "two_bn" else None
    plain = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    call("avt_conv2d_dgrad", P(D(dy)), P(wt), P(plain), P(D(add) if add is not None else None), N, H, W, C, K, R, R,
         st, pad, S())
    xc = _rand_act(N, H, W, C, 18)
    stats = _bn_stats_rand(C, 19)
    y = _rand_act(N, H, W, C, 20) if mode == "mask_y" else None
    acc, acc2 = bwd_ws(N * H * W, C), bwd_ws(N * H * W, C)
    xc2, stats2 = _rand_act(N, H, W, C, 21), _bn_stats_rand(C, 22)
    from avt_amd._lib import DgradBnEpi

    e = DgradBnEpi()
    e.xc, e.stats, e.acc = P(D(xc)).value, P(D(stats)).value, acc.data_ptr()
    e.y = P(D(y)).value if y is not None else None
    if mode == "two_bn":
        e.xc2, e.stats2, e.acc2 = P(D(xc2)).value, P(D(stats2)).value, acc2.data_ptr()
    dx = torch.empty_like(plain)
    call("avt_conv2d_dgrad_bn", P(D(dy)), P(wt), P(dx), P(D(add) if add is not None else None), N, H, W, C, K, R, R,
         st, pad, ctypes.byref(e), S())
    torch.cuda.synchronize()
    gm, s1, s2 = _dgrad_bn_ref(plain, xc, stats, y)
    assert torch.equal(dx.cpu().double(), gm)
    a = acc_sums(acc, C, 2, bwd=True)
    tol = 1e-5 * gm.abs().sum(0 if gm.dim() == 1 else tuple(range(gm.dim() - 1))).max().item() + 1e-6
    np.testing.assert_allclose(a[:, 0].numpy(), s1.numpy(), atol=tol)
    np.testing.assert_allclose(a[:, 1].numpy(), s2.numpy(), atol=tol * 4)
    if mode == "two_bn":
        _, s1b, s3 = _dgrad_bn_ref(plain, xc2, stats2, None)
        b = acc_sums(acc2, C, 2, bwd=True)
        np.testing.assert_allclose(b[:, 0].numpy(), s1.numpy(), atol=tol)  # sum g' of the FIRST BN's mask
        xh2 = (xc2.double() - stats2[2].double()) * stats2[3].double()
        np.testing.assert_allclose(b[:, 1].numpy(), (gm * xh2).reshape(-1, C).sum(0).numpy(), atol=tol * 4)
    # premasked finalize + apply == the reference BN backward on g'
    gamma = (1.0 + 0.1 * torch.randn(C, generator=g)).float().to(DEV)
    dgamma, dbeta = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    gc = torch.empty_like(dx)
    rows = N * H * W
    call("avt_bn_bwd_premasked", P(dx), P(D(xc)), P(D(stats[2])), P(D(stats[3])), P(gamma), P(dgamma), P(dbeta), P(gc),
         P(acc), rows, C, S())
    torch.cuda.synchronize()
    xhat = (xc.double() - stats[2].double()) * stats[3].double()
    k1, k2 = s1 / rows, s2 / rows
    ref_gc = gamma.double().cpu() * stats[3].double() * (gm - k1 - xhat * k2)
    assert rel_err(gc, ref_gc) < 8e-3
    np.testing.assert_allclose(dbeta.cpu().double().numpy(), s1.numpy(), atol=tol)
    np.testing.assert_allclose(dgamma.cpu().double().numpy(), s2.numpy(), atol=tol * 4)


@pytest.mark.parametrize("case", [(2, 9, 11, 64, 128, 3, 2, 1), (2, 15, 13, 64, 128, 3, 2, 1)])
def test_strided_dgrad_skip00_then_downsample_epilogue(case):
    """A first block's input gradient: the 3x3/s2 conv1 dgrad stores its class-(0,0) pixels plain
    (skip_class00), the in-place 1x1/s2 downsample dgrad adds to them and applies the epilogue: the
    union equals the masked sum of both dgrads, the sums cover every pixel once."""
    N, H, W, C, K, R, st, pad = case
    Pq, Qq = conv_out(H, 3, 2, 1), conv_out(W, 3, 2, 1)
    dy1, dyd = _rand_act(N, Pq, Qq, K, 25), _rand_act(N, Pq, Qq, K, 26)
    g = torch.Generator().manual_seed(27)
    w1 = (torch.randn(K, 3, 3, C, generator=g) * 0.05).float()
    wd = (torch.randn(K, 1, 1, C, generator=g) * 0.05).float()
    _, wt1 = pack(w1.to(DEV), C, 9 * C)
    _, wtd = pack(wd.to(DEV), C, C)
    ref = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    call("avt_conv2d_dgrad", P(D(dy1)), P(wt1), P(ref), None, N, H, W, C, K, 3, 3, 2, 1, S())
    call("avt_conv2d_dgrad", P(D(dyd)), P(wtd), P(ref), P(ref), N, H, W, C, K, 1, 1, 2, 0, S())
    xc, y, stats = _rand_act(N, H, W, C, 28), _rand_act(N, H, W, C, 29), _bn_stats_rand(C, 30)
    acc = bwd_ws(N * H * W, C)
    from avt_amd._lib import DgradBnEpi

    e = DgradBnEpi()
    e.xc, e.y, e.stats, e.acc = P(D(xc)).value, P(D(y)).value, P(D(stats)).value, acc.data_ptr()
    e.skip_class00 = 1
    dx = torch.empty_like(ref)
    call("avt_conv2d_dgrad_bn", P(D(dy1)), P(wt1), P(dx), None, N, H, W, C, K, 3, 3, 2, 1, ctypes.byref(e), S())
    e.skip_class00 = 0
    e.append_slots = 1  # the downsample dgrad's sums go after the conv1 dgrad's (include/avt.h)
    call("avt_conv2d_dgrad_bn", P(D(dyd)), P(wtd), P(dx), P(dx), N, H, W, C, K, 1, 1, 2, 0, ctypes.byref(e), S())
    torch.cuda.synchronize()
    gm, s1, s2 = _dgrad_bn_ref(ref, xc, stats, y)
    assert torch.equal(dx.cpu().double(), gm)
    a = acc_sums(acc, C, 2, bwd=True)
    tol = 1e-5 * gm.abs().sum((0, 1, 2)).max().item() + 1e-6
    np.testing.assert_allclose(a[:, 0].numpy(), s1.numpy(), atol=tol)
    np.testing.assert_allclose(a[:, 1].numpy(), s2.numpy(), atol=tol * 4)


@pytest.mark.parametrize("case", [(32, 17, 19, 256, 256, 3, 1, 1), (32, 14, 14, 256, 256, 3, 1, 1),
                                  (32, 14, 14, 512, 512, 3, 1, 1), (6, 6, 6, 256, 256, 3, 1, 1)])
def test_small_grid_conv_repeatable(case):
    """Small-batch grids (configs[2]'s 32-clip shard: the 64-row tiles) give the same bits on every launch:
    forward, BN partial sums and dgrad over repeated launches on the same inputs (a data race inside a
    kernel shows up here as run-to-run differences far below the fp64-comparison tolerances)."""
    N, H, W, C, K, R, st, pad = case
    x = _rand_act(N, H, W, C, 81).relu().to(DEV)
    g = torch.Generator().manual_seed(82)
    w = (torch.randn(K, R, R, C, generator=g) * 0.05).float().to(DEV)
    wf, wt = pack(w, C, R * R * C)
    dy = _rand_act(N, H, W, K, 83).to(DEV)
    outs = []
    for _ in range(12):
        y = torch.empty(N, H, W, K, device=DEV, dtype=torch.bfloat16)
        acc = fwd_acc(N * H * W, K)
        call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st, pad, R * R * C, S())
        dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
        call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, R, R, st, pad, S())
        torch.cuda.synchronize()
        outs.append((y.view(torch.int16).clone(), dx.view(torch.int16).clone(), acc_sums(acc, K, 3)))
    for i, o in enumerate(outs[1:], 1):
        assert torch.equal(o[0], outs[0][0]), f"launch {i}: forward output differs"
        assert torch.equal(o[2], outs[0][2]), f"launch {i}: BN partial sums differ"
        assert torch.equal(o[1], outs[0][1]), f"launch {i}: dgrad differs"


@pytest.mark.parametrize("case", [(2, 17, 19, 512, 512, 3, 1, 1), (2, 33, 38, 128, 128, 3, 1, 1)])
def test_halo8_form_and_ring_bitwise_equal(case):
    """The 8-wave 256 x 128 halo tile's A/B knobs (avt_set_halo8_form: 4 waves of 128 x 64; avt_set_halo8_nst:
    a 4-stage weight ring; avt_set_halo_tps2: one wait + barrier per two taps for >= 8 chunks, an A/B knob) change
    the wave layout, the DMA depth and the synchronisation, not the k order of any output: conv
    outputs, plain dgrads and BN-epilogue dgrads are bitwise equal; the BN slot sums are bitwise equal under the
    4-stage ring and equal to rounding under the 4-wave form (its reduction partition differs)."""
    N, H, W, C, K, R, st, pad = case
    x = _rand_act(N, H, W, C, 71).relu().to(DEV)
    g = torch.Generator().manual_seed(72)
    w = (torch.randn(K, R, R, C, generator=g) * 0.05).float().to(DEV)
    wf, wt = pack(w, C, R * R * C)
    dy = _rand_act(N, H, W, K, 73).to(DEV)
    xc, stats = _rand_act(N, H, W, C, 74).to(DEV), _bn_stats_rand(C, 75).to(DEV)
    from avt_amd._lib import DgradBnEpi

    call("avt_set_halo8", 1)
    outs = []
    try:
        for form, nst, tps2 in ((0, 3, 0), (1, 3, 0), (0, 4, 0), (0, 3, 1)):
            call("avt_set_halo8_form", form)
            call("avt_set_halo8_nst", nst)
            call("avt_set_halo_tps2", tps2)
            y = torch.empty(N, H, W, K, device=DEV, dtype=torch.bfloat16)
            acc = fwd_acc(N * H * W, K)
            call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, C, K, R, R, st, pad, R * R * C, S())
            dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
            call("avt_conv2d_dgrad", P(dy), P(wt), P(dx), None, N, H, W, C, K, R, R, st, pad, S())
            ws = bwd_ws(N * H * W, C)
            e = DgradBnEpi()
            e.xc, e.stats, e.acc = P(xc).value, P(stats).value, ws.data_ptr()
            dxe = torch.empty_like(dx)
            call("avt_conv2d_dgrad_bn", P(dy), P(wt), P(dxe), None, N, H, W, C, K, R, R, st, pad, ctypes.byref(e), S())
            torch.cuda.synchronize()
            outs.append((y.view(torch.int16).clone(), dx.view(torch.int16).clone(), dxe.view(torch.int16).clone(),
                         acc_sums(acc, K, 3), acc_sums(ws, C, 2, bwd=True)))
    finally:
        call("avt_set_halo8_form", -1)
        call("avt_set_halo8_nst", -1)
        call("avt_set_halo_tps2", -1)
        call("avt_set_halo8", -1)
    # outputs and dgrads bitwise; the 4-wave form sums the statistics over its own wave/thread partition (another
    # fp32 order): its slots to rounding, the 4-stage ring's and the two-tap loop's bitwise
    for form, o in zip((1, 0, 0), outs[1:]):
        for a, b in zip(o[:3], outs[0][:3]):
            assert torch.equal(a, b)
        for a, b in zip(o[3:], outs[0][3:]):
            if form:
                np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-5, atol=1e-6 * b.abs().max().item())
            else:
                assert torch.equal(a, b)
    with pytest.raises(RuntimeError):
        call("avt_set_halo8_nst", 5)


def test_dgrad_bn_epilogue_needs_lds_dma_kernels():
    """The register-staged conv variant (avt_set_conv_variant(0)) has no BN-backward epilogue: a dgrad that asks
    for one is refused instead of leaving the accumulator's header and slots unwritten."""
    N, H, W, C, K = 2, 9, 11, 64, 64
    dy = _rand_act(N, H, W, K, 81).to(DEV)
    w = (torch.randn(K, 3, 3, C, generator=torch.Generator().manual_seed(82)) * 0.05).float().to(DEV)
    _, wt = pack(w, C, 9 * C)
    xc, stats = _rand_act(N, H, W, C, 83).to(DEV), _bn_stats_rand(C, 84).to(DEV)
    ws = bwd_ws(N * H * W, C)
    from avt_amd._lib import DgradBnEpi

    e = DgradBnEpi()
    e.xc, e.stats, e.acc = P(xc).value, P(stats).value, ws.data_ptr()
    dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    call("avt_set_conv_variant", 0)
    try:
        with pytest.raises(RuntimeError, match="epilogue"):
            call("avt_conv2d_dgrad_bn", P(dy), P(wt), P(dx), None, N, H, W, C, K, 3, 3, 1, 1, ctypes.byref(e), S())
    finally:
        call("avt_set_conv_variant", 1)


@pytest.mark.parametrize("header", [float("nan"), -1.0, 1e9])
def test_bn_finalize_rejects_bad_slot_header(header):
    """A statistics accumulator whose header was never written (garbage slot count) gives NaN statistics
    from avt_bn_finalize / avt_bn_bwd_premasked -- no reads beyond the workspace's slots."""
    rows, C = 300, 64
    acc = fwd_acc(rows, C)
    acc[0], acc[1] = header, 0.0
    gamma, beta = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    stats = torch.empty(4, C, device=DEV)
    call("avt_bn_finalize", P(acc), rows, C, P(gamma), P(beta), None, None, ctypes.c_float(0.1),
         ctypes.c_float(1e-5), P(stats[0]), P(stats[1]), P(stats[2]), P(stats[3]), S())
    ws = bwd_ws(rows, C)
    ws.view(torch.float64)[0], ws.view(torch.float64)[1] = header, 0.0
    g, xc = _rand_act(1, rows, 1, C, 85).to(DEV), _rand_act(1, rows, 1, C, 86).to(DEV)
    dgamma, dbeta = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    gc = torch.empty_like(g)
    call("avt_bn_bwd_premasked", P(g), P(xc), P(stats[2]), P(stats[3]), P(gamma), P(dgamma), P(dbeta), P(gc),
         P(ws), rows, C, S())
    torch.cuda.synchronize()
    assert torch.isnan(stats[2]).all() and torch.isnan(stats[3]).all()
    assert torch.isnan(dbeta).all() and torch.isnan(dgamma).all()


@pytest.mark.parametrize("N,H,W,Cin", [(2, 20, 22, 3), (2, 21, 17, 1), (1, 224, 224, 3), (2, 9, 8, 3)])
def test_stem_dgrad(N, H, W, Cin):
    """avt_conv_stem_dgrad: the 7x7 / s2 / p3 stem conv's input gradient (base_models.py:135-138 under autograd) vs
    torch's conv2d_input in fp64 on the same bf16 output gradient and fp32 weights."""
    P_, Q_ = conv_out(H, 7, 2, 3), conv_out(W, 7, 2, 3)
    gy = _rand_act(N, P_, Q_, 64, 91)
    w = torch.randn(64, 7, 7, Cin, generator=torch.Generator().manual_seed(92)) * 0.05  # OHWI
    gx = torch.empty(N, Cin, H, W, device=DEV)
    call("avt_conv_stem_dgrad", P(D(gy)), P(D(w.contiguous())), P(gx), N, H, W, Cin, S())
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_input((N, Cin, H, W), w.double().permute(0, 3, 1, 2), gy.double().permute(0, 3, 1, 2),
                                     stride=2, padding=3)
    assert rel_err(gx, ref) < 1e-5
