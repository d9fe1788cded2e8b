"""Evaluation restatement (oracle/eval_oracle.py) and the host side of avt_amd.evaluate /
avt_amd.checkpoint, on CPU."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import avenet_oracle as orc
import eval_oracle as evo
from avt_amd import checkpoint as ckpt
from avt_amd import evaluate as ev
from avt_amd.model import AVENet
from avt_amd.optim import FlatAdam


@pytest.mark.parametrize("h,w,S", [(14, 14, 224), (7, 9, 224), (14, 14, 100), (3, 5, 17)])
def test_resize_restatement_matches_torch_bilinear(h, w, S):
    """The cv2 INTER_LINEAR restatement == torch's independent bilinear (align_corners=False) up to
    rounding (the formula is the same for upscaling; the order of fp32 operations differs)."""
    g = torch.Generator().manual_seed(50)
    m = torch.randn(h, w, generator=g)
    ours = evo.cv2_resize_linear(m.numpy(), S)
    ref = F.interpolate(m[None, None].double(), size=(S, S), mode="bilinear", align_corners=False)[0, 0].numpy()
    np.testing.assert_allclose(ours, ref, atol=2e-6, rtol=0)


def test_evaluator_and_auc_match_reference_formulas():
    rng = np.random.default_rng(51)
    e = ev.Evaluator()
    cious = []
    for _ in range(7):
        infer = rng.random((224, 224)).astype(np.float32)
        gt = evo.gt_map_flickr([[10, 20, 130, 200], [60, 40, 250, 120]])
        c, i, d = e.cal_CIOU(infer, gt, 0.5)
        rc, ri, rd = evo.cal_ciou(infer, gt, 0.5)
        assert (c, i, d) == (rc, ri, rd)
        cious.append(rc)
    assert abs(e.cal_AUC() - evo.cal_auc(cious)) < 1e-12
    assert e.final() == np.mean(np.array(cious) >= 0.5)


def test_gt_maps_match_reference():
    boxes = [[0, 0, 256, 256], [30, 40, 100, 220], [200, 10, 255, 60]]
    np.testing.assert_array_equal(ev.gt_map_flickr(boxes), evo.gt_map_flickr(boxes))
    nb = [[0.1, 0.2, 0.6, 0.9], [-0.1, 0.5, 0.3, 1.2]]
    np.testing.assert_array_equal(ev.gt_map_vggss(nb), evo.gt_map_vggss(nb))


def test_binarize_keeps_half_the_pixels():
    rng = np.random.default_rng(52)
    p = evo.binarize(rng.standard_normal((14, 14)).astype(np.float32))
    assert set(np.unique(p)) <= {0.0, 1.0}
    assert abs(p.mean() - 0.5) < 0.01


# ------------------------------------------------------------------------------------ checkpoints
def _cpu_model(seed=0):
    m = AVENet(orc.Args(), False)
    m.load_state_dict(orc.make_state(seed))
    return m


def test_checkpoint_roundtrip_reference_layout(tmp_path):
    m = _cpu_model(0)
    path = tmp_path / "model_1frm_10k_ep3.pth.tar"
    ck = ckpt.save_checkpoint(str(path), 3, m)
    ref_keys = [n for n, _, _ in orc.avenet_entries()]
    assert list(ck["model_state_dict"]) == ["module." + k for k in ref_keys]  # DataParallel layout
    m2 = _cpu_model(1)
    assert ckpt.load_checkpoint(str(path), m2) == 3
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k
    # partial dicts update (model_dict.update semantics); unknown keys raise
    m3 = _cpu_model(1)
    part = {"module.imgnet.conv1.weight": m.state_dict()["imgnet.conv1.weight"]}
    ckpt.load_checkpoint({"model_state_dict": part}, m3)
    assert torch.equal(m3.state_dict()["imgnet.conv1.weight"], m.state_dict()["imgnet.conv1.weight"])
    assert torch.equal(m3.state_dict()["audnet.conv1_a.weight"], _cpu_model(1).state_dict()["audnet.conv1_a.weight"])
    with pytest.raises(KeyError):
        ckpt.load_checkpoint({"model_state_dict": {"module.bogus": torch.zeros(1)}}, m3)


def test_flat_adam_state_converts_to_and_from_torch_adam():
    """A torch.optim.Adam state over the reference's parameter order (what the reference's
    checkpoints hold) -> the fused step's flat Adam -> back: identical tensors and step count."""
    m = _cpu_model(0)
    params = list(m.parameters())
    names = [n for n, _ in m.named_parameters()]
    topt = torch.optim.Adam(params, lr=4e-6, weight_decay=1e-4)
    g = torch.Generator().manual_seed(53)
    for _ in range(2):
        for n, p in zip(names, params):
            p.grad = torch.randn(p.shape, generator=g) if m._flat.trainable(n) else None
        topt.step()
    sd = topt.state_dict()
    fopt = FlatAdam(m._flat, lr=1.0)
    ckpt.load_flat_adam_state_dict(m, fopt, sd)
    assert fopt.t == 2 and fopt.lr == 4e-6 and fopt.wd == 1e-4
    back = ckpt.flat_adam_state_dict(m, fopt)
    assert set(back["state"]) == set(sd["state"])
    for i, st in sd["state"].items():
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(back["state"][i][k], st[k]), (names[i], k)
        assert float(back["state"][i]["step"]) == float(st["step"])
    # and torch's Adam accepts the converted dict
    topt2 = torch.optim.Adam(params, lr=1.0)
    topt2.load_state_dict(back)
    assert topt2.param_groups[0]["lr"] == 4e-6


def _ref_cal_ciou(infer, gtmap, thres):
    """utils.Evaluator.cal_CIOU (utils.py:209-214) transcribed line for line in numpy (the
    reference's own arithmetic, independent of both the product and eval_oracle)."""
    infer_map = np.zeros((224, 224))
    infer_map[infer >= thres] = 1
    ciou = np.sum(infer_map * gtmap) / (np.sum(gtmap) + np.sum(infer_map * (gtmap == 0)))
    return ciou, np.sum(infer_map * gtmap), (np.sum(gtmap) + np.sum(infer_map * (gtmap == 0)))


@pytest.mark.parametrize("n,seed", [(1, 60), (13, 61), (249, 62)])
def test_auc_matches_sklearn_on_reference_grid(n, seed):
    """utils.Evaluator.cal_AUC (utils.py:216-225) is sklearn.metrics.auc over x = [0.05 i, i=0..20]
    of the fraction of maps with cIoU >= 0.05 i: the product and the restatement against sklearn
    itself (importable here), incl. ties exactly on the grid and the 249-map test set size."""
    from sklearn import metrics

    rng = np.random.default_rng(seed)
    cious = list(rng.random(n))
    cious[: min(n, 3)] = [0.05 * k for k in (0, 10, 20)][: min(n, 3)]  # values on grid points
    x = [0.05 * i for i in range(21)]
    y = [np.sum(np.array(cious) >= 0.05 * i) / len(cious) for i in range(21)]
    ref = metrics.auc(x, y)
    e = ev.Evaluator()
    e.ciou = list(cious)
    assert abs(e.cal_AUC() - ref) < 1e-12, (e.cal_AUC(), ref)
    assert abs(ev.auc_from_cious(cious) - ref) < 1e-12
    assert abs(evo.cal_auc(cious) - ref) < 1e-12


@pytest.mark.parametrize("thres", [0.5, 0.01, 0.0])
def test_cal_ciou_matches_reference_transcription(thres):
    """Evaluator.cal_CIOU on random maps (and the restatement) vs the line-for-line numpy transcription
    of utils.py:209-214: identical (cIoU, intersection, denominator)."""
    rng = np.random.default_rng(63)
    for k in range(6):
        infer = rng.random((224, 224)).astype(np.float32)
        if k == 5:
            infer[:] = thres  # every pixel exactly on the threshold
        gt = (rng.random((224, 224)) < 0.3).astype(np.float64) * (0.5 if k % 2 else 1.0)
        ref = _ref_cal_ciou(infer, gt, thres)
        got = ev.Evaluator().cal_CIOU(infer, gt, thres)
        assert got[1] == ref[1] and got[2] == ref[2] and abs(got[0] - ref[0]) < 1e-15, (got, ref)
        rc = evo.cal_ciou(infer, gt, thres)
        assert rc[1] == ref[1] and rc[2] == ref[2] and abs(rc[0] - ref[0]) < 1e-15
