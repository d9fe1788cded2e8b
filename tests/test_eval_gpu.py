"""Localisation evaluation kernels (avt_localize_ciou / avt_pair_ciou via avt_amd.evaluate) against
the restated test protocol (oracle/eval_oracle.py), and checkpoint resume of the fused step."""
import numpy as np
import pytest
import torch

import avenet_oracle as orc
import eval_oracle as evo
from avt_amd import checkpoint as ckpt
from avt_amd import evaluate as ev
from avt_amd.model import AVENet
from avt_amd.train import HardWayTrainStep

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _heatmaps(n, h, w, seed):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((n, 1, h, w)).astype(np.float32) * 0.3 + 0.5
    A[0, 0, :, :] = 0.25                       # constant map: normalize_img leaves it unchanged
    A[1, 0, : h // 2] = A[1, 0, 0, 0]          # a plateau: ties around the median
    return A


def _gts(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        if i % 2:
            x0, y0 = rng.integers(0, 128, 2)
            x1, y1 = x0 + rng.integers(20, 128), y0 + rng.integers(20, 128)
            out.append(evo.gt_map_flickr([[x0, y0, x1, y1], [x0 + 10, y0 + 5, x1 + 30, y1]]))
        else:
            x0, y0 = rng.random(2) * 0.5
            out.append(evo.gt_map_vggss([[x0, y0, x0 + 0.4, y0 + 0.3]]))
    return np.stack(out)


@pytest.mark.parametrize("h,w", [(14, 14), (7, 9)])
def test_localize_matches_reference_protocol(h, w):
    n = 6
    A = _heatmaps(n, h, w, 60)
    gt = _gts(n, 61)
    stats, maps = ev.localize(torch.from_numpy(A).to(DEV), torch.from_numpy(gt).to(DEV), return_maps=True)
    torch.cuda.synchronize()
    stats, maps = stats.cpu().numpy(), maps.cpu().numpy()
    for i in range(n):
        pred = evo.binarize(A[i, 0])
        np.testing.assert_array_equal(maps[i], (pred >= 0.5).astype(np.uint8), err_msg=f"map {i}")
        c, inter, den = evo.cal_ciou(pred, gt[i], 0.5)
        assert (stats[i, 0], stats[i, 1], stats[i, 2]) == (c, inter, den), i


def test_mtc_and_auc():
    A = _heatmaps(5, 14, 14, 62)
    _, maps = ev.localize(torch.from_numpy(A).to(DEV), return_maps=True)
    preds = [evo.binarize(A[i, 0]) for i in range(5)]
    assert abs(ev.mtc(maps) - evo.mtc(preds)) < 1e-12
    cious = list(np.random.default_rng(63).random(40))
    assert abs(ev.auc_from_cious(cious) - evo.cal_auc(cious)) < 1e-12


def test_evaluate_hardway_on_model_heatmaps():
    """The test_hardway loop on the drop-in model's own A: kernel == protocol restatement."""
    m = AVENet(orc.Args(), False)
    m.load_state_dict(orc.make_state(0))
    m = m.to(DEV)
    img, aud = orc.make_image(4, 224), orc.make_spectrogram(4)
    gt = _gts(4, 64)
    with torch.no_grad():
        m.eval()
        A = m(img.to(DEV), aud.to(DEV))[0].cpu().numpy()
    ref = [evo.cal_ciou(evo.binarize(A[i, 0]), gt[i], 0.5)[0] for i in range(4)]
    c, auc = ev.evaluate_hardway(m, [(img.to(DEV), aud.to(DEV))], [gt])
    assert c == np.mean(np.array(ref) >= 0.5)
    assert abs(auc - evo.cal_auc(ref)) < 1e-12


def test_checkpoint_resume_of_fused_step(tmp_path):
    """save after two fused steps -> load into a fresh model/step -> the next step continues the
    same trajectory (same weights, moments, step count)."""
    img, aud = orc.make_image(4, 64).to(DEV), orc.make_spectrogram(4, 65, 76).to(DEV)

    def fresh():
        m = AVENet(orc.Args(), False)
        m.load_state_dict(orc.make_state(0))
        m = m.to(DEV).train()
        return m, HardWayTrainStep(m, lr=1e-4)

    m1, s1 = fresh()
    for _ in range(2):
        s1.step(img, aud)
    path = tmp_path / "ck.pth.tar"
    ckpt.save_checkpoint(str(path), 1, m1, s1)
    m2, s2 = fresh()
    assert ckpt.load_checkpoint(str(path), m2, s2) == 1
    assert s2.opt.t == 2
    s1.step(img, aud)
    s2.step(img, aud)
    torch.cuda.synchronize()
    for (n, a), (_, b) in zip(m1.state_dict().items(), m2.state_dict().items()):
        if n.endswith("num_batches_tracked"):
            assert int(a) == int(b) == 3, n
        else:  # identical state; only split-K/atomic ordering can differ (<= one lr-sized update)
            assert (a.double() - b.double()).abs().max().item() <= 1.2e-4, n
