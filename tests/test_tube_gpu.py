"""3-D tube path on the GPU (FullModel = R3D-18 + audio ResNet-18 + HardWayAttention; BASELINE
config 4): Conv3d / video-stem kernels vs fp64 on identical bf16 inputs, the R3D-18 forward vs the
oracle, and the full train_3D.py step vs golden vectors produced by the reference FullModel
(oracle/gen_golden_tube.py), in both audio modes (folded repeated spectrogram / one per clip)."""
import ctypes
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import avenet_oracle as orc
import tube_oracle as tor
from avt_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
_KEEP = []


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


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _golden(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False))


CONV3D_CASES = [
    # N, T, H, W, C, K, stride
    (2, 4, 9, 11, 64, 64, 1),
    (2, 4, 9, 11, 64, 128, 2),
    (1, 5, 7, 6, 128, 256, 2),
    (2, 3, 5, 4, 256, 256, 1),
    (1, 16, 14, 14, 256, 512, 2),
    (1, 2, 3, 3, 512, 512, 1),
    # stride 1, N % 128 == 0 or N = 64: the halo kernel's three-patch Conv3d form -- clip ends inside a tile (several
    # clips, T = 1..16), image widths on every patch-size path (W <= 39: 336 rows; W = 56: 416; N = 64: 488), ragged M
    (2, 4, 9, 11, 128, 128, 1),
    (3, 1, 14, 14, 128, 256, 1),
    (3, 5, 28, 28, 128, 128, 1),
    (1, 3, 56, 56, 128, 128, 1),
    (2, 16, 14, 14, 512, 512, 1),
    (1, 7, 13, 17, 256, 128, 1),
    (2, 3, 112, 112, 64, 64, 1),
    (3, 2, 21, 30, 64, 64, 1),
    (1, 5, 56, 56, 128, 64, 1),
]


@pytest.mark.parametrize("halo3d", [2, 0])
@pytest.mark.parametrize("case", CONV3D_CASES)
def test_conv3d_fwd_and_bn_stats(case, halo3d):
    """Conv3d fwd + its BN statistics vs fp64 torch, on the halo kernel's Conv3d form where it applies (halo3d=2, the
    default: stride 1, N % 128 == 0 or N = 64) and on the tap-gather kernel (halo3d=0)."""
    N, T, H, W, C, K, st = case
    if halo3d == 0 and not (st == 1 and (K % 128 == 0 or K == 64)):
        pytest.skip("the halo form does not apply to this shape: halo3d=1 already runs the tap gather")
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, T, H, W, C, generator=g).relu().to(torch.bfloat16)
    w = (torch.randn(K, C, 3, 3, 3, generator=g) * (2.0 / (K * 27)) ** 0.5).float()
    wd = w.to(DEV)
    wp = torch.empty(K, 27 * C, device=DEV, dtype=torch.bfloat16)
    call("avt_pack_conv3d_weight", P(wd), P(wp), K, C, 3, 3, 3, 0, S())
    Ho, Wo = (H + 2 - 3) // st + 1, (W + 2 - 3) // st + 1
    y = torch.empty(N, T, Ho, Wo, K, device=DEV, dtype=torch.bfloat16)
    acc = torch.full((int(query("avt_bn_acc_doubles", N * T * Ho * Wo, K)),), float("nan"), device=DEV,
                     dtype=torch.float64)
    xd = x.to(DEV)
    try:
        call("avt_set_halo3d", halo3d)
        call("avt_conv3d_fwd", P(xd), P(wp), P(y), P(acc), N, T, H, W, C, K, 3, 3, 3, st, 1, 1, S())
    finally:
        call("avt_set_halo3d", -1)
    ref = F.conv3d(x.double().permute(0, 4, 1, 2, 3), w.to(torch.bfloat16).double(), stride=(1, st, st), padding=1)
    ref = ref.permute(0, 2, 3, 4, 1)
    err = rel_err(y, ref)
    assert err < 8e-3, err
    # BN statistics from the epilogue accumulators
    gamma = torch.ones(K, device=DEV)
    beta = torch.zeros(K, device=DEV)
    stats = torch.empty(4, K, device=DEV)
    rows = N * T * Ho * Wo
    call("avt_bn_finalize", P(acc), rows, K, P(gamma), P(beta), None, None, ctypes.c_float(0.1),
         ctypes.c_float(1e-5), P(stats[0]), P(stats[1]), P(stats[2]), P(stats[3]), S())
    r = ref.reshape(-1, K)
    mean = r.mean(0)
    np.testing.assert_allclose(stats[2].cpu().double().numpy(), mean.numpy(), atol=1e-3 * r.abs().max().item())
    var = r.var(0, unbiased=False)
    np.testing.assert_allclose((1 / stats[3].cpu().double() ** 2 - 1e-5).numpy(), var.numpy(), rtol=2e-2,
                               atol=1e-4 * var.max().item())


@pytest.mark.parametrize("case", [(2, 16, 14, 14, 512, 512), (3, 5, 9, 11, 256, 128), (1, 4, 28, 28, 256, 256)])
def test_conv3d_halo_two_tap_bitwise(case):
    """The Conv3d halo form with one wait + barrier per two taps (avt_set_halo_tps2(1), an A/B knob for >= 8 virtual
    chunks: the R3D-18 layer3/4) and per tap (0, the default): the same k order, bitwise-equal outputs and BN slots."""
    N, T, H, W, C, K = case
    g = torch.Generator().manual_seed(13)
    x = torch.randn(N, T, H, W, C, generator=g).relu().to(torch.bfloat16).to(DEV)
    w = (torch.randn(K, C, 3, 3, 3, generator=g) * (2.0 / (K * 27)) ** 0.5).float().to(DEV)
    wp = torch.empty(K, 27 * C, device=DEV, dtype=torch.bfloat16)
    call("avt_pack_conv3d_weight", P(w), P(wp), K, C, 3, 3, 3, 0, S())
    rows = N * T * H * W
    outs = []
    try:
        for tps2 in (0, 1):
            call("avt_set_halo_tps2", tps2)
            y = torch.empty(N, T, H, W, K, device=DEV, dtype=torch.bfloat16)
            acc = torch.full((int(query("avt_bn_acc_doubles", rows, K)),), float("nan"), device=DEV,
                             dtype=torch.float64)
            call("avt_conv3d_fwd", P(x), P(wp), P(y), P(acc), N, T, H, W, C, K, 3, 3, 3, 1, 1, 1, S())
            torch.cuda.synchronize()
            nslots = (rows + 255) // 256
            # header + the written slots, as bits (the header's unused words keep the NaN fill)
            outs.append((y.view(torch.int16).clone(), acc[:8 + nslots * K * 3].view(torch.int64).clone()))
    finally:
        call("avt_set_halo_tps2", -1)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("C,K", [(64, 64), (64, 128), (128, 128)])
def test_conv3d_tile_configs(C, K):
    """Conv3d at a GEMM M >= 65536 (where the tile choice depends on K) under every tile config the
    planner picks from (launch_nt): bitwise-equal outputs (the same k order per element), checked against
    torch on output frames 0-1."""
    N, T, H, W = 1, 8, 96, 96
    g = torch.Generator().manual_seed(12)
    x = torch.randn(N, T, H, W, C, generator=g).relu().to(torch.bfloat16)
    w = (torch.randn(K, C, 3, 3, 3, generator=g) * (2.0 / (K * 27)) ** 0.5).float()
    wp = torch.empty(K, 27 * C, device=DEV, dtype=torch.bfloat16)
    call("avt_pack_conv3d_weight", P(w.to(DEV)), P(wp), K, C, 3, 3, 3, 0, S())
    xd = x.to(DEV)
    knobs = [("avt_set_nt64_config", v) for v in (-1, 1, 0)] if K == 64 else \
            [("avt_set_nt128_config", v) for v in (-1, 1, 6)]
    outs = []
    try:
        call("avt_set_halo3d", 0)  # the tap-gather tiles (the halo form takes K % 128 == 0 by default)
        for fn, v in knobs:
            call(fn, v)
            y = torch.empty(N, T, H, W, K, device=DEV, dtype=torch.bfloat16)
            call("avt_conv3d_fwd", P(xd), P(wp), P(y), None, N, T, H, W, C, K, 3, 3, 3, 1, 1, 1, S())
            outs.append(y)
        torch.cuda.synchronize()
    finally:
        call("avt_set_nt64_config", -1)
        call("avt_set_nt128_config", -1)
        call("avt_set_halo3d", -1)
    for (fn, v), o in zip(knobs[1:], outs[1:]):
        assert torch.equal(o, outs[0]), (fn, v)
    # output frames 0 and 1 read input frames 0-2 only
    ref = F.conv3d(x[:, :3].float().permute(0, 4, 1, 2, 3), w.to(torch.bfloat16).float(), padding=1)[:, :, :2]
    err = rel_err(outs[0][:, :2], ref.permute(0, 2, 3, 4, 1))
    assert err < 8e-3, err


@pytest.mark.parametrize("shape", [(2, 4, 32, 32), (1, 16, 30, 22), (1, 3, 17, 9)])
def test_video_stem_fold(shape):
    """Stem Conv3d(3,64,(7,7,7),s(1,2,2),p3) = im2col (temporal taps -> channels) + 7x7/s2 conv."""
    b, T, H, W = shape
    g = torch.Generator().manual_seed(3)
    video = torch.randn(b, 3, T, H, W, generator=g)
    w = (torch.randn(64, 3, 7, 7, 7, generator=g) * (2.0 / (64 * 343)) ** 0.5).float()
    vd, wd = video.to(DEV), w.to(DEV)
    x = torch.empty(b, T, H, W, 32, device=DEV, dtype=torch.bfloat16)
    call("avt_video_stem_im2col", P(vd), P(x), b, 3, T, H, W, 7, 3, S())
    wp = torch.empty(64, 49 * 32, device=DEV, dtype=torch.bfloat16)
    call("avt_pack_conv3d_weight", P(wd), P(wp), 64, 3, 7, 7, 7, 1, S())
    Ho, Wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    y = torch.empty(b * T, Ho, Wo, 64, device=DEV, dtype=torch.bfloat16)
    call("avt_conv2d_fwd", P(x), P(wp), P(y), None, b * T, H, W, 32, 64, 7, 7, 2, 3, 49 * 32, S())
    ref = F.conv3d(video.to(torch.bfloat16).double(), w.to(torch.bfloat16).double(), stride=(1, 2, 2), padding=3)
    ref = ref.permute(0, 2, 3, 4, 1).reshape(b * T, Ho, Wo, 64)
    err = rel_err(y, ref)
    assert err < 8e-3, err
    # the folded layout itself: channel kt*4+c of frame t holds x[c][t+kt-3] (bf16), zero padded
    xc = x.cpu().float()
    vb = video.to(torch.bfloat16).float()
    for t in range(T):
        for kt in range(7):
            tt = t + kt - 3
            for c in range(4):
                got = xc[0, t, :, :, kt * 4 + c]
                exp = vb[0, c, tt] if (0 <= tt < T and c < 3) else torch.zeros(H, W)
                assert torch.equal(got, exp), (t, kt, c)
    assert torch.count_nonzero(xc[..., 28:]) == 0


def test_repeat_and_sum_rows():
    a = torch.randn(3, 512, device=DEV)
    r = torch.empty(12, 512, device=DEV)
    call("avt_repeat_rows_f32", P(a), P(r), 3, 4, 512, S())
    assert torch.equal(r, a.repeat_interleave(4, 0))
    s = torch.empty(3, 512, device=DEV)
    call("avt_sum_rep_rows_f32", P(r), P(s), 3, 4, 512, S())
    torch.testing.assert_close(s, 4 * a)


def _fullmodel(seed=0):
    from avt_amd.model import FullModel

    m = FullModel(orc.Args())
    m.load_state_dict(tor.make_tube_state(seed))
    return m.to(DEV).train()


def _tube_inputs(g):
    b, t, size, f, fr = g["shape"].tolist()
    return tor.make_video(b, t, size), orc.make_spectrogram(b, f, fr)


@pytest.mark.parametrize("name", ["fullmodel_tiny_b2t4", "fullmodel_mid_b2t4"])
def test_r3d_layer4_vs_reference(golden_dir, name):
    """The vidnet layer4 map (the reference forward hook's output) vs the fp64 reference."""
    g = _golden(golden_dir, name)
    video, _ = _tube_inputs(g)
    m = _fullmodel()
    eng = m.engine()
    eng.pack_weights()
    with torch.no_grad():
        v = eng.vid.forward(video.to(DEV), eng.store, True)  # [(b t), h, w, 512]
    torch.cuda.synchronize()
    b, t = video.shape[0], video.shape[2]
    got = v.float().cpu().view(b, t, v.shape[1], v.shape[2], 512).permute(0, 4, 1, 2, 3)
    ref = torch.from_numpy(g["layer4_f64_slice"])
    err = (got.double().flatten()[:256] - ref).abs().max().item() / ref.abs().max().item()
    print(f"{name}: layer4 rel err {err:.3e}")
    assert err < 5e-2, err
    cs = np.array([got.double().sum().item(), (got.double() ** 2).sum().item()])
    np.testing.assert_allclose(cs, g["layer4_f64_checksum"][:2], rtol=2e-2)


@pytest.mark.parametrize("name", ["fullmodel_tiny_b2t4", "fullmodel_mid_b2t4"])
@pytest.mark.parametrize("per_clip", [False, True])
def test_fullmodel_step_vs_reference(golden_dir, name, per_clip):
    g = _golden(golden_dir, name)
    video, spec = _tube_inputs(g)
    b, t = video.shape[0], video.shape[2]
    audio = spec if per_clip else tor.repeat_spectrogram(spec, t)
    m = _fullmodel()
    A, logits = m(audio.to(DEV), video.to(DEV))
    loss = torch.nn.CrossEntropyLoss()(logits, torch.zeros(b * t, dtype=torch.long, device=DEV))
    loss.backward()
    torch.cuda.synchronize()
    A, lg = A.detach().cpu().double().numpy(), logits.detach().cpu().double().numpy()
    off = ~np.eye(b * t, b * t + 2, k=1, dtype=bool)
    dev = {"A_abs": np.abs(A - g["A_f64"]).max(),
           "logits_off_abs": np.abs(lg[off] - g["logits_f64"][off]).max(),
           "loss_rel": abs(loss.item() - g["loss_f64"].item()) / abs(g["loss_f64"].item())}
    floors = {"A_abs": 1e-2, "logits_off_abs": 2e-2, "loss_rel": 1e-3}
    for k, v in dev.items():
        tol = max(floors[k], 3 * float(g["bf16ref_dev/" + k]))
        print(f"{name} per_clip={per_clip}: {k} = {v:.3e} (bf16 reference {float(g['bf16ref_dev/' + k]):.3e}, "
              f"tol {tol:.3e})")
        assert v <= tol, (k, v, tol)
    params = dict(m.named_parameters())
    names = [str(n) for n in g["param_names"]]
    gn = np.array([params[n].grad.norm().item() for n in names])
    rel = np.abs(gn - g["grad_norm_f64"]) / g["grad_norm_f64"]
    dref = g["bf16ref_dev/gradnorm_rel"]
    print(f"{name}: grad-norm rel err max {rel.max():.3e} median {np.median(rel):.3e} (bf16 reference max "
          f"{dref.max():.3e} median {np.median(dref):.3e})")
    assert np.median(rel) <= max(3 * np.median(dref), 5e-2)
    assert rel.max() <= max(1.5 * dref.max(), 0.1)
    for n in params:  # vidnet (detached), audnet.conv1/conv1_flow/fc: no gradient, as the reference
        if n not in names:
            assert params[n].grad is None, n


def test_per_clip_equals_folded_audio(golden_dir):
    """The de-duplicated audio trunk gives the folded batch's outputs and buffers, and gradients as
    close to the fp64 reference as the folded run's (bf16 trunks: the two round differently)."""
    g = _golden(golden_dir, "fullmodel_tiny_b2t4")
    video, spec = _tube_inputs(g)
    outs = []
    for per_clip in (False, True):
        m = _fullmodel()
        audio = spec if per_clip else tor.repeat_spectrogram(spec, 4)
        A, logits = m(audio.to(DEV), video.to(DEV))
        loss = torch.nn.CrossEntropyLoss()(logits, torch.zeros(8, dtype=torch.long, device=DEV))
        loss.backward()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
        outs.append((logits.detach(), grads, {k: v.clone() for k, v in m.state_dict().items()}))
    (l0, g0, s0), (l1, g1, s1) = outs
    torch.testing.assert_close(l1, l0, atol=2e-3, rtol=1e-3)
    assert g0.keys() == g1.keys()
    # both modes against the fp64 oracle's full gradients (CPU, same inputs/weights)
    sd64 = tor.make_tube_state(0, torch.float64)
    sd32 = tor.make_tube_state(0)
    for k in sd64:
        if sd64[k].is_floating_point():
            sd64[k] = sd32[k].double()
    _, _, _, gref = tor.tube_train_step(sd64, spec.double(), video.double(), None)

    def cos(a, b):
        return F.cosine_similarity(a.flatten().double().cpu(), b.flatten().double(), dim=0).item()

    c0 = {n: cos(g0[n], gref[n]) for n in gref}
    c1 = {n: cos(g1[n], gref[n]) for n in gref}
    m0, m1 = np.median(list(c0.values())), np.median(list(c1.values()))
    w1 = min(c1, key=c1.get)
    print(f"  full-tensor gradient cosine to fp64: folded median {m0:.4f} min {min(c0.values()):.4f}; "
          f"per-clip median {m1:.4f} min {c1[w1]:.4f} ({w1})")
    # bf16 trunks: the summed-vs-separate head gradients round differently; the per-clip mode must be
    # as close to fp64 as the folded one (the identity itself is exact in fp64:
    # tests/test_tube_oracle_golden.py::test_per_clip_audio_is_exact_in_fp64)
    # (per-clip rounds each clip's summed head gradient once where the folded batch rounds t copies
    # separately and averages their rounding errors in the fp32 wgrad accumulators: slightly noisier)
    assert m1 >= m0 - 0.05 and min(c1.values()) >= min(c0.values()) - 0.1, (m0, m1)
    # and both as close as the reference's own bf16-autocast trunks (median / worst parameter)
    names = [str(n) for n in g["param_names"]]
    cref = g["bf16ref_dev/grad_cos"]
    print(f"  bf16 reference: median {np.median(cref):.4f} min {cref.min():.4f}")
    for cc in (c0, c1):
        v = np.array([cc[n] for n in names])
        assert np.median(v) >= np.median(cref) - 0.05 and v.min() >= cref.min() - 0.1, (np.median(v), v.min())
    for k in s0:
        if "running" in k:
            torch.testing.assert_close(s1[k], s0[k], atol=1e-3, rtol=1e-2)
        elif k.endswith("num_batches_tracked"):
            assert int(s0[k]) == int(s1[k]) == 1


def test_fullmodel_buffers_and_eval(golden_dir):
    g = _golden(golden_dir, "fullmodel_tiny_b2t4")
    video, spec = _tube_inputs(g)
    m = _fullmodel()
    with torch.no_grad():
        m(spec.to(DEV), video.to(DEV))
    sd = m.state_dict()
    for k in [k for k in g if k.startswith("buf_f64/")]:
        n = k.split("/", 1)[1]
        ref = g[k]
        got = sd[n][:16].cpu().double().numpy()
        assert np.abs(got - ref).max() <= 2e-2 * max(1.0, np.abs(ref).max()), n
    assert int(sd["vidnet.bn1.num_batches_tracked"]) == 1
    m.eval()
    with torch.no_grad():
        A, logits = m(spec.to(DEV), video.to(DEV))
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    sd64 = {k: v.cpu() for k, v in sd64.items()}
    rA, rlog = tor.fullmodel_forward(sd64, tor.repeat_spectrogram(spec, 4).double(), video.double(), training=False)
    assert (A.cpu().double() - rA).abs().max() < 3e-2


def test_tube_train_step_graph_and_loss():
    from avt_amd.train import HardWayTrainStep

    video = tor.make_video(2, 4, 32).to(DEV)
    spec = orc.make_spectrogram(2, 65, 76).to(DEV)
    m_e, m_g = _fullmodel(), _fullmodel()
    s_e = HardWayTrainStep(m_e, lr=1e-4, weight_decay=1e-4)
    s_g = HardWayTrainStep(m_g, lr=1e-4, weight_decay=1e-4)
    le = [s_e.step(spec, video).item() for _ in range(4)]
    lg = [s_g.step(spec, video).item()]
    s_g.capture(spec.clone(), video.clone())
    lg += [s_g.step(spec, video).item() for _ in range(3)]
    print("eager", le, "graph", lg)
    assert np.all(np.isfinite(le)) and le[-1] < le[0], le
    np.testing.assert_allclose(lg, le, rtol=2e-3)
    # the vidnet is never updated (no gradient reaches it)
    before = tor.make_tube_state(0)
    sd = m_g.state_dict()
    for n in ("vidnet.conv1.weight", "vidnet.layer4.1.conv2.weight"):
        assert torch.equal(sd[n].cpu(), before[n]), n


@pytest.mark.parametrize("b,t,hw,C,normalized", [(2, 3, 7, 512, False), (1, 4, 14, 64, True), (3, 2, 5, 128, False)])
def test_hardway_attention_standalone_autograd(b, t, hw, C, normalized):
    """Standalone HardWayAttention()(audio_features, video_features) (model.py:38-60): fp32 outputs and
    gradients into both inputs against the fp64 oracle (autograd through orc.hardway_attention).
    The module takes the features as given (no normalisation inside), so un-normalised inputs are a case."""
    from avt_amd.model import HardWayAttention

    g = torch.Generator().manual_seed(b * 100 + t * 10 + hw)
    vid = torch.randn(b, C, t, hw, hw, generator=g, dtype=torch.float64) * 0.05
    aud = torch.randn(b * t, C, generator=g, dtype=torch.float64)
    if normalized:  # FullModel's call (model.py:31-35)
        vid = F.normalize(vid, dim=1)
        aud = F.normalize(aud, dim=1)
    else:
        aud = F.normalize(aud, dim=1) * 1.3
    wl = torch.randn(b * t, b * t + 2, generator=g, dtype=torch.float64)
    wa = torch.randn(b * t, 1, hw, hw, generator=g, dtype=torch.float64)

    vr, ar = vid.clone().requires_grad_(), aud.clone().requires_grad_()
    A_r, l_r = orc.hardway_attention(ar, vr)
    ((l_r * wl).sum() + (A_r * wa).sum()).backward()

    vd = vid.float().to(DEV).requires_grad_()
    ad = aud.float().to(DEV).requires_grad_()
    A, logits = HardWayAttention()(ad, vd)
    assert A.dtype == torch.float32 and logits.dtype == torch.float32 and A.requires_grad
    ((logits * wl.float().to(DEV)).sum() + (A * wa.float().to(DEV)).sum()).backward()
    # fp32 arithmetic against fp64: the logits carry 1/0.07 and sigmoids of (A - eps)/0.03
    assert rel_err(A, A_r.detach()) < 1e-5
    assert rel_err(logits, l_r.detach()) < 2e-4
    assert rel_err(vd.grad, vr.grad) < 2e-4
    assert rel_err(ad.grad, ar.grad) < 2e-4


@pytest.mark.parametrize("K,C,KT,R", [(64, 64, 3, 3), (128, 64, 3, 3), (512, 256, 3, 3), (512, 512, 3, 3),
                                        (128, 64, 1, 1), (16, 3, 3, 3), (8, 7, 3, 3), (32, 12, 3, 3)])
def test_pack_conv3d_weight_layout(K, C, KT, R):
    """avt_pack_conv3d_weight (fold 0): out[k][((kt*R + r)*S + s)*C + c] = bf16(w[k][c][kt][r][s]) -- the filter-row
    transpose through LDS (C % 8 == 0) and the element kernel (other C) both equal torch's permute + RNE cast, bitwise."""
    g = torch.Generator().manual_seed(K + C + KT)
    w = torch.randn(K, C, KT, R, R, generator=g)
    wp = torch.empty(K, KT * R * R * C, device=DEV, dtype=torch.bfloat16)
    wd = w.to(DEV)
    call("avt_pack_conv3d_weight", P(wd), P(wp), K, C, KT, R, R, 0, S())
    ref = w.permute(0, 2, 3, 4, 1).reshape(K, -1).to(torch.bfloat16)
    assert torch.equal(wp.cpu().view(torch.int16), ref.view(torch.int16))


def test_pack_conv3d_weights_batched_matches_single():
    """avt_pack_conv3d_weights_batched (one launch for every non-stem R3D conv) == avt_pack_conv3d_weight per conv,
    bitwise: 16-byte filter-row path, and the element path for C % 8 != 0 and for a misaligned source."""
    import struct

    # K, C, T, flat offset (floats)
    cases = [(64, 64, 27, 0), (128, 64, 1, 110592), (512, 512, 27, 118784), (16, 12, 27, 7196672),
             (8, 7, 9, 7201856), (32, 16, 27, 7202363)]
    total = max(o + K * C * T for K, C, T, o in cases)
    g = torch.Generator().manual_seed(9)
    flat = torch.randn(total, generator=g).to(DEV)
    descs, outs, singles = [], [], []
    for K, C, T, o in cases:
        w = flat[o:o + K * C * T]
        out = torch.empty(K, C * T, device=DEV, dtype=torch.bfloat16)
        descs.append(struct.pack("<QQiiii", w.data_ptr(), out.data_ptr(), K, C, T, 0))
        outs.append(out)
        one = torch.empty_like(out)
        kt, r = (3, 3) if T == 27 else (1, 3) if T == 9 else (1, 1)
        call("avt_pack_conv3d_weight", P(w), P(one), K, C, kt, r, r, 0, S())
        singles.append(one)
    assert len(descs[0]) == int(query("avt_pack3d_desc_bytes"))
    table = torch.frombuffer(bytearray(b"".join(descs)), dtype=torch.uint8).to(DEV)
    call("avt_pack_conv3d_weights_batched", P(table), len(descs), max(c[0] for c in cases),
         max(c[1] * c[2] for c in cases), S())
    torch.cuda.synchronize()
    for out, one in zip(outs, singles):
        assert torch.equal(out.view(torch.int16), one.view(torch.int16))
    with pytest.raises(RuntimeError):
        call("avt_pack_conv3d_weights_batched", P(table), len(descs), 512, 15361, S())


@pytest.mark.parametrize("shape", [(2, 16, 112, 112, 64), (1, 5, 7, 9, 8), (3, 1, 1, 2, 16), (2, 4, 6, 6, 64)])
def test_maxpool3d_matches_torch(shape):
    """avt_maxpool3d_fwd = nn.MaxPool3d(kernel_size=3, stride=2, padding=1) (resnet3D.py:129) on NDHWC bf16: bitwise
    equal to torch's max_pool3d of the same values (a max of bf16 values is exact), odd and unit extents, NaN and
    -0.0 / +0.0 ties (the first tap wins, as in torch)."""
    N, T, H, W, C = shape
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, T, H, W, C, generator=g).to(torch.bfloat16)
    x[..., 0] = torch.where(torch.rand(N, T, H, W, generator=g) < 0.5, torch.tensor(-0.0), torch.tensor(0.0)).bfloat16()
    if x.numel() > 64:
        x.view(-1)[37] = float("nan")
    To, Ho, Wo = (T - 1) // 2 + 1, (H - 1) // 2 + 1, (W - 1) // 2 + 1
    xd = x.to(DEV)
    y = torch.full((N, To, Ho, Wo, C), 7.0, device=DEV, dtype=torch.bfloat16)
    call("avt_maxpool3d_fwd", P(xd), P(y), N, T, H, W, C, S())
    ref = F.max_pool3d(x.float().permute(0, 4, 1, 2, 3).contiguous(), kernel_size=3, stride=2, padding=1)
    ref = ref.permute(0, 2, 3, 4, 1).to(torch.bfloat16)
    got = y.cpu()
    assert got.shape == ref.shape
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16)) or (
        torch.equal(torch.isnan(got), torch.isnan(ref)) and
        torch.equal(got.nan_to_num().view(torch.int16), ref.nan_to_num().view(torch.int16)))
    with pytest.raises(RuntimeError):
        call("avt_maxpool3d_fwd", P(xd), P(y), N, T, H, W, 12, S())


@pytest.mark.parametrize("standalone,max_pool", [(False, False), (True, False), (True, True)])
def test_r3d_forward_standalone(standalone, max_pool):
    """VERDICT r3 Missing #3: FullModel.vidnet(video) / a standalone generate_model(18, no_max_pool=True or False
    (the stem max-pool, VERDICT r5 gap 3), n_classes=1039)(video) return resnet3D.ResNet.forward's fc logits (resnet3D.py:197-213: layer4 ->
    AdaptiveAvgPool3d -> fc) on the same kernels, vs the fp64 restatement; forward-only (raises where
    gradients would be needed)."""
    from avt_amd.resnet3D import generate_model

    video = tor.make_video(2, 4, 64)
    sd = tor.make_tube_state(0)
    if standalone:
        net = generate_model(18, no_max_pool=not max_pool, n_classes=1039)
        net.load_state_dict({k[len("vidnet."):]: v for k, v in sd.items() if k.startswith("vidnet.")})
        net = net.to(DEV).train()
    else:
        net = _fullmodel().vidnet
    with pytest.raises(NotImplementedError):
        net(video.to(DEV))  # grad mode with parameters that require grad
    with torch.no_grad():
        logits = net(video.to(DEV))
    torch.cuda.synchronize()
    assert logits.shape == (2, 1039)
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    with torch.no_grad():
        feat = tor.r3d18_forward(sd64, "vidnet.", video.double(), training=True, max_pool=max_pool)  # [b,512,t,h,w]
        ref = F.linear(feat.mean(dim=(2, 3, 4)), sd64["vidnet.fc.weight"], sd64["vidnet.fc.bias"])
    err = rel_err(logits, ref)
    print(f"standalone={standalone} max_pool={max_pool}: R3D logits rel err {err:.3e}")
    assert err < 3e-2, err
    # train mode updated the running statistics and the batch counter, as the reference BN3d does
    bn1 = net.bn1
    assert int(bn1.num_batches_tracked) == 1
    assert not torch.equal(bn1.running_mean.cpu(), torch.zeros(64))
