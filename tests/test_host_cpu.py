"""Host-side logic on CPU: the C-ABI library loads and exports every declared symbol, the drop-in
module tree / state_dict / init match the reference, flat storage aliasing is right, and the
product path refuses to run without a GPU (no silent CPU fallback)."""
import os
import re

import numpy as np
import pytest
import torch

import avenet_oracle as orc
from avt_amd import _lib
from avt_amd.engine import FlatStore, trainable
from avt_amd.model import AVENet
from gen_golden import checksum

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = "".join(open(os.path.join(REPO, "include", h)).read() for h in ("avt.h", "avt_tuning.h"))
    return sorted(set(re.findall(r"\b(avt_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    lib = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} declared in avt.h but not bound in _lib.SIGNATURES"
    assert lib.avt_abi_version() == 1
    # pure host queries need no GPU
    # BN accumulators: 8-double header + one slot per 64 rows (+ 520 for persistent / reduce grids)
    assert _lib.query("avt_bn_acc_doubles", 6400, 64) == 8 + (100 + 520) * 64 * 3
    assert _lib.query("avt_bn_bwd_workspace", 6400, 64) == (8 + 64 + (100 + 520) * 64 * 2) * 8
    assert _lib.query("avt_hardway_bwd_ws_floats", 128, 512) == 64 * 128 * 512
    assert _lib.query("avt_pack_desc_bytes") == 48
    assert _lib.query("avt_hardway_save_floats", 8) == 8 * 20


def test_error_path_reports_message():
    # invalid shape is rejected on the host before any launch
    with pytest.raises(RuntimeError, match="null pointer"):
        _lib.call("avt_conv2d_fwd", None, None, None, None, 1, 8, 8, 64, 48, 3, 3, 1, 1, 576, None)


def test_state_dict_keys_shapes_match_reference_inventory():
    m = AVENet(orc.Args(), False)
    sd = m.state_dict()
    ref = orc.avenet_entries()
    assert list(sd.keys()) == [n for n, _, _ in ref]
    for n, shape, _ in ref:
        assert tuple(sd[n].shape) == tuple(shape), n
    assert sum(p.numel() for p in m.parameters()) == 23_422_928
    assert m._flat.n_train == 22_346_752
    assert sum(1 for n, _ in m.named_parameters() if trainable(n)) == len(orc.trainable_names(orc.make_state(0)))


def test_torch_seeded_init_matches_reference(golden_dir):
    g = np.load(os.path.join(golden_dir, "torch_init_seed0.npz"), allow_pickle=False)
    torch.manual_seed(0)
    m = AVENet(orc.Args(), False)
    sd = m.state_dict()
    for n, cs in zip(g["names"], g["checksums"]):
        np.testing.assert_allclose(checksum(sd[str(n)]), cs, rtol=1e-6, err_msg=str(n))


def test_flat_views_alias_storage_and_load_state_dict():
    m = AVENet(orc.Args(), False)
    ref = orc.make_state(0)
    m.load_state_dict(ref)
    w = m.imgnet.layer2[0].conv1.weight
    assert w.is_contiguous(memory_format=torch.channels_last)
    raw = m._flat.raw("imgnet.layer2.0.conv1.weight")
    assert raw.data_ptr() == w.data_ptr()
    assert torch.equal(raw.permute(0, 3, 1, 2), ref["imgnet.layer2.0.conv1.weight"])
    # in-place update through the flat buffer is visible through the parameter
    m._flat.flat[m._flat.poff["imgnet.layer2.0.conv1.weight"][0]] = 123.0
    assert w[0, 0, 0, 0].item() == 123.0
    rm = m.audnet.layer3[1].bn2.running_var
    assert rm.data_ptr() == m._flat.rawbuf("audnet.layer3.1.bn2.running_var").data_ptr()
    # trainable parameters occupy the front of the flat buffer
    offs = [m._flat.poff[n][0] for n in m._flat.pnames if trainable(n)]
    assert max(offs) < m._flat.n_train
    assert min(m._flat.poff[n][0] for n in m._flat.pnames if not trainable(n)) >= m._flat.n_train


def test_apply_rebinds_views():
    m = AVENet(orc.Args(), False)
    m = m.to(torch.device("cpu"))  # _apply path keeps aliasing
    assert m.imgnet.conv1.weight.data_ptr() == m._flat.raw("imgnet.conv1.weight").data_ptr()
    with pytest.raises(TypeError):
        m.double()


def test_no_cpu_fallback():
    m = AVENet(orc.Args(), False)
    with pytest.raises(RuntimeError, match="GPU"):
        m(torch.zeros(1, 3, 64, 64), torch.zeros(1, 1, 65, 76))


def test_grad_views_layout():
    m = AVENet(orc.Args(), False)
    g = torch.arange(m._flat.n_train, dtype=torch.float32)
    views = m._flat.param_grad_views(g)
    p = dict(m.named_parameters())
    for n, v in views.items():
        assert v.shape == p[n].shape and v.stride() == p[n].stride(), n


# ------------------------------------------------------------------ 3-D tube model (FullModel)
def test_fullmodel_state_dict_and_trainable_set():
    import tube_oracle as tor
    from avt_amd.model import FullModel

    m = FullModel(orc.Args())
    sd = m.state_dict()
    ref = tor.fullmodel_entries()
    assert list(sd.keys()) == [n for n, _, _ in ref]
    for n, shape, _ in ref:
        assert tuple(sd[n].shape) == tuple(shape), n
    names = [n for n in m._flat.pnames if m._flat.trainable(n)]
    assert sorted(names) == sorted(tor.trainable_names_tube())
    assert m._flat.n_train == sum(dict(m.named_parameters())[n].numel() for n in names)
    # vidnet conv weights keep the reference's OIDHW layout (contiguous 5-D views of the flat buffer)
    assert m.vidnet.conv1.weight.is_contiguous() and m.vidnet.layer1[0].conv1.weight.is_contiguous()


def test_fullmodel_torch_seeded_init_matches_reference(golden_dir):
    from avt_amd.model import FullModel

    g = dict(np.load(os.path.join(golden_dir, "fullmodel_torch_init_seed0.npz"), allow_pickle=False))
    torch.manual_seed(0)
    m = FullModel(orc.Args())
    sd = m.state_dict()
    assert list(sd.keys()) == [str(k) for k in g["keys"]]
    for n, cs in zip(g["names"], g["checksums"]):
        np.testing.assert_allclose(checksum(sd[str(n)]), cs, rtol=1e-10, atol=1e-10, err_msg=str(n))


def test_fullmodel_refuses_cpu():
    import tube_oracle as tor
    from avt_amd.model import FullModel

    m = FullModel(orc.Args())
    with pytest.raises(RuntimeError):
        m(orc.make_spectrogram(1, 65, 76), tor.make_video(1, 2, 32))


def test_flat_multistep_lr_matches_torch_schedule():
    """FlatMultiStepLR == torch.optim.lr_scheduler.MultiStepLR (train_hardway_1frame.py:118) epoch by
    epoch, and every change lands in the device hyper-parameter vector the graph-replayable Adam reads."""
    import types

    from avt_amd.optim import FlatAdam, FlatMultiStepLR

    flat = types.SimpleNamespace(n_train=8, flat=torch.zeros(8))
    opt = FlatAdam(flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4)
    sched = FlatMultiStepLR(opt, milestones=[60, 100, 150, 180], gamma=0.1)
    p = torch.nn.Parameter(torch.zeros(1))
    topt = torch.optim.Adam([p], lr=1e-3)
    tsched = torch.optim.lr_scheduler.MultiStepLR(topt, milestones=[60, 100, 150, 180], gamma=0.1)
    for epoch in range(200):
        assert abs(opt.lr - topt.param_groups[0]["lr"]) <= 1e-12 * max(1.0, topt.param_groups[0]["lr"]), epoch
        assert abs(float(opt._hyper[0]) - opt.lr) <= 1e-7 * opt.lr
        topt.step()
        tsched.step()
        sched.step()
    opt.betas = (0.8, 0.9)
    opt.eps, opt.wd = 1e-6, 0.0
    assert opt._hyper.tolist() == pytest.approx([opt.lr, 0.8, 0.9, 1e-6, 0.0])


def test_flat_multistep_lr_resume_does_not_decay_twice():
    """resuming a schedule (last_epoch=e, the optimizer lr restored from a checkpoint taken
    after epoch e) keeps the restored lr and then follows the uninterrupted torch MultiStepLR."""
    import types

    from avt_amd.optim import FlatAdam, FlatMultiStepLR

    ms = [60, 100, 150, 180]
    for e in (59, 68, 99, 120, 179):
        p = torch.nn.Parameter(torch.zeros(1))
        topt = torch.optim.Adam([p], lr=1e-6)
        tsched = torch.optim.lr_scheduler.MultiStepLR(topt, milestones=ms, gamma=0.1)
        for _ in range(e + 1):  # epochs 0..e, a scheduler step after each (train_hardway_1frame.py:138)
            topt.step()
            tsched.step()
        restored = topt.param_groups[0]["lr"]  # the checkpoint's lr: epoch e+1's
        for with_initial in (True, False):
            flat = types.SimpleNamespace(n_train=8, flat=torch.zeros(8))
            opt = FlatAdam(flat, lr=restored, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4)
            opt.initial_lr = 1e-6 if with_initial else None
            sched = FlatMultiStepLR(opt, milestones=ms, gamma=0.1, last_epoch=e)
            assert sched.base_lr == pytest.approx(1e-6, rel=1e-9), (e, with_initial)
            assert opt.lr == pytest.approx(restored, rel=1e-9), (e, with_initial)
            ref = torch.optim.lr_scheduler.MultiStepLR(torch.optim.Adam([torch.nn.Parameter(torch.zeros(1))],
                                                                        lr=1e-6), milestones=ms, gamma=0.1)
            for _ in range(e + 1):
                ref.step()
            for _ in range(60):
                ref.step()
                sched.step()
                assert opt.lr == pytest.approx(ref.get_last_lr()[0], rel=1e-9), (e, with_initial)


def test_flatstore_mirror_and_deepcopy_rebind():
    """FlatStore.mirror (the per-GPU store of an nn.DataParallel replica) copies every value and refuses
    module moves; a deep-copied AVENet's trunks belong to the copy."""
    import copy

    torch.manual_seed(0)
    m = AVENet(orc.Args(), False)
    mir = m._flat.mirror("cpu")
    assert torch.equal(mir.flat, m._flat.flat) and mir.flat.data_ptr() != m._flat.flat.data_ptr()
    assert torch.equal(mir.bflat, m._flat.bflat) and torch.equal(mir.nbt, m._flat.nbt)
    assert torch.equal(mir.raw("imgnet.layer1.0.conv1.weight"), m._flat.raw("imgnet.layer1.0.conv1.weight"))
    with pytest.raises(RuntimeError):
        mir.apply(lambda t: t)
    twin = copy.deepcopy(m)
    assert twin.imgnet._avt_parent[0]() is twin and twin.audnet._avt_parent[0]() is twin
    w = dict(twin.named_parameters())["imgnet.layer1.0.conv1.weight"]
    assert w.data_ptr() >= twin._flat.flat.data_ptr()
    assert w.data_ptr() < twin._flat.flat.data_ptr() + twin._flat.flat.numel() * 4
    with torch.no_grad():
        twin._flat.flat.zero_()
    assert dict(m.named_parameters())["imgnet.layer1.0.conv1.weight"].abs().sum() > 0


@pytest.mark.parametrize("knob", ["AVT_DIAG_SKIP", "AVT_HALO_DBG"])
def test_bench_refuses_wrong_results_knobs(knob):
    """bench.py exits non-zero, before touching a GPU, when a wrong-results timing diagnostic is set."""
    import subprocess
    import sys

    env = dict(os.environ, **{knob: "1"})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "1", "--warmup", "0"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "refusing" in (r.stderr + r.stdout) and knob in (r.stderr + r.stdout)


def test_bench_eager_copy_drops_every_captured_form():
    """bench.py's roofline profiles an eager copy of the train step.  At world > 1 the overlap schedule keeps its
    capture in _seg_graphs (the non-overlap one in _graph + _graph_opt); a copy that kept either would replay it and
    the profiler would see no conv launch (roofline.launches 0 at N > 1)."""
    import importlib.util

    import avtubes  # noqa: F401
    from avt_amd.train import HardWayTrainStep

    spec = importlib.util.spec_from_file_location("avt_bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    calls = []
    for captured in ({"_graph": object(), "_graph_opt": None, "_seg_graphs": None},
                     {"_graph": None, "_graph_opt": None, "_seg_graphs": [object(), object()]},
                     {"_graph": object(), "_graph_opt": object(), "_seg_graphs": None}):
        step = HardWayTrainStep.__new__(HardWayTrainStep)
        step.__dict__.update(captured)
        step._replay = lambda *a: calls.append("replay")
        step._eager_step = lambda *a: calls.append("eager")
        step.step()
        eager = bench.eager_copy(step)
        eager.step()
        assert eager._replay is step._replay  # same state otherwise
    assert calls == ["replay", "eager"] * 3, calls


def test_h1_skip_diagnostic_needs_opt_in():
    """AVT_DIAG_H1_SKIP makes the trunks compute a different network (timing diagnostic): importing the library
    under it fails unless AVT_DIAG_WRONG_RESULTS_OK=1 is set as well."""
    import subprocess
    import sys

    code = "import avtubes; import avt_amd.trunk as t; print('H1', t.DIAG_H1_SKIP)"
    env = {k: v for k, v in os.environ.items() if k != "AVT_DIAG_WRONG_RESULTS_OK"}
    env["AVT_DIAG_H1_SKIP"] = "1"
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WRONG results" in r.stderr
    env["AVT_DIAG_WRONG_RESULTS_OK"] = "1"
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "H1 True" in r.stdout, r.stderr
