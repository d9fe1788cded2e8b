"""Cross-trunk corruption finder (determinism diagnostic): runs one trunk's backward launch by launch on one
stream and, after every launch, compares the OTHER trunk's saved forward tensors with a copy taken before --
a change means a launch of this trunk wrote outside its own buffers.  usage: python tools/diag_oob.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import avtubes  # noqa: E402,F401
import avenet_oracle as orc  # noqa: E402
from avt_amd.model import AVENet, HardWayArgs  # noqa: E402
from avt_amd.train import HardWayTrainStep  # noqa: E402
from avt_amd.trunk import P, stream_ptr  # noqa: E402
from avt_amd._lib import call  # noqa: E402

DEV = torch.device("cuda")
img, aud = orc.make_image(6, 96).to(DEV), orc.make_spectrogram(6, 97, 110).to(DEV)
m = AVENet(HardWayArgs(), False)
m.load_state_dict(orc.make_state(3))
m = m.to(DEV).train()
step = HardWayTrainStep(m, lr=1e-4, weight_decay=1e-4)
for _ in range(2):
    step.step(img, aud)
torch.cuda.synchronize()
eng = step.engine
eng.concurrent = False


def tensors(obj, prefix, out):
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            out[prefix] = obj
    elif isinstance(obj, dict):
        for k, v in obj.items():
            tensors(v, f"{prefix}.{k}", out)
    elif isinstance(obj, (list, tuple)):
        for i, v in enumerate(obj):
            tensors(v, f"{prefix}[{i}]", out)
    return out


for victim in ("img", "aud"):
    out, tape = eng.forward(img, aud, training=True, with_ce=True, ce_scale=1.0)
    step.grad.zero_()
    gv, gan = eng.head_backward(tape, out["dlogits"])
    eng.store.grads = eng.flat.grad_views(step.grad)
    watch = tensors(tape[victim], victim, {})
    watch.update({"head." + k: v for k, v in tensors({k: tape[k] for k in ("v", "a", "an")}, "", {}).items()})
    watch["gv" if victim == "img" else "gan"] = gv if victim == "img" else gan
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in watch.items()}
    hi = eng.img.HI_BLOCK
    if victim == "img":  # run the AUDIO backward, watch the vision tensors
        a = tape["a"]
        B, C = tape["B"], tape["C"]
        ga = torch.empty_like(a)
        call("avt_audio_pool_norm_bwd", P(gan), P(tape["an"]), P(tape["amax"]), P(tape["anorm"]), P(ga), B,
             a.shape[1] * a.shape[2], C, stream_ptr())

        def chain():
            g, pm = yield from eng.aud.backward_blocks_iter(tape["aud"], ga, eng.store, hi, len(eng.aud.blocks))
            g, _ = yield from eng.aud.backward_blocks_iter(tape["aud"], g, eng.store, 0, hi, pm)
            yield from eng.aud.backward_stem_iter(tape["aud"], g, eng.store)
        gen = chain()
    else:
        def chain():
            g, pm = yield from eng.img.backward_blocks_iter(tape["img"], gv, eng.store, hi, len(eng.img.blocks))
            g, _ = yield from eng.img.backward_blocks_iter(tape["img"], g, eng.store, 0, hi, pm)
            yield from eng.img.backward_stem_iter(tape["img"], g, eng.store)
        gen = chain()
    n = 0
    bad = False
    while True:
        try:
            next(gen)
        except StopIteration:
            break
        n += 1
        torch.cuda.synchronize()
        for k, v in watch.items():
            if not torch.equal(v, ref[k]):
                d = (v.float() - ref[k].float()).abs()
                print(f"victim {victim}: after launch group {n} of the other trunk, {k} changed "
                      f"({int((d > 0).sum())} of {v.numel()} elements, shape {tuple(v.shape)})", flush=True)
                ref[k] = v.clone()
                bad = True
    eng.store.grads = None
    print(f"victim {victim}: {n} launch groups checked, {'CORRUPTED' if bad else 'clean'}", flush=True)
