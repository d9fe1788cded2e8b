"""Determinism and concurrency diagnostics of the train step (GPU; not imported by the tests or the product).

usage: python tools/diag.py <command> [args]
  rep          one conv launch repeated on the same inputs: distinct outputs (a data race shows as more than one).  args: [N H W C K] [launches]; env REP_FRESH=w|x rewrites the operands before each launch
  runs         which gradients differ between identical runs of the fused train step (3 runs x 3 steps; env DET_B, DET_FULL, DET_RUNS, DET_KEEP, DET_SHORT; AVT_CONCURRENT=0: one stream)
  calls        first divergence point between identical runs: the vision trunk's backward helper calls fingerprinted on the issuing stream (env DET_RUNS, DET_ONLY)
  oob          cross-trunk corruption finder: one trunk's backward launch by launch, the other trunk's saved tensors compared after every launch
  concurrency  concurrent (audio trunk on a side stream) vs sequential train steps: losses over several steps
  spread       run-to-run gradient spread of the fused and drop-in paths (1-frame and two-view)
"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import avtubes  # noqa: E402,F401
import avenet_oracle as orc  # noqa: E402
from avt_amd import trunk as T  # noqa: E402
from avt_amd._lib import call  # noqa: E402
from avt_amd.model import AVENet, HardWayArgs  # noqa: E402
from avt_amd.train import HardWayTrainStep, TwoViewTrainStep  # noqa: E402
from avt_amd.trunk import P, stream_ptr  # noqa: E402

DEV = torch.device("cuda")

def cmd_rep(argv):
    """one conv launch repeated on the same inputs: distinct outputs (a data race shows as more than one).  args: [N H W C K] [launches]; env REP_FRESH=w|x rewrites the operands before each launch"""
    a = [int(v) for v in argv[0:5]] if len(argv) > 4 else [32, 14, 14, 512, 512]
    n_launch = int(argv[5]) if len(argv) > 5 else 60
    N, H, W, C, K = a
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(5)
    dy = torch.randn(N, H, W, K, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(K, 3, 3, C, generator=g) * 0.05).to(dev)
    wf = torch.empty(K, 9 * C, device=dev, dtype=torch.bfloat16)
    wt = torch.empty(C, 9 * K, device=dev, dtype=torch.bfloat16)
    S = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
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


def cmd_runs(argv):
    """which gradients differ between identical runs of the fused train step (3 runs x 3 steps; env DET_B, DET_FULL, DET_RUNS, DET_KEEP, DET_SHORT; AVT_CONCURRENT=0: one stream)"""
    # DET_KEEP=1: keep every tensor a step allocates alive until the step has synchronised (no allocator reuse
    # inside a step: isolates cross-stream reuse of freed blocks)
    if os.environ.get("DET_KEEP"):
        _keep = []
        for _name in ("empty", "empty_like", "zeros", "zeros_like", "full"):
            _orig = getattr(torch, _name)

            def _wrap(*a, _o=_orig, **k):
                t = _o(*a, **k)
                _keep.append(t)
                return t
            setattr(torch, _name, _wrap)
    _B = int(os.environ.get("DET_B", "6"))
    if os.environ.get("DET_FULL"):  # the bench's input sizes (224 x 224 frames, 257 x 300 spectrograms)
        img, aud = orc.make_image(_B, 224).to(DEV), orc.make_spectrogram(_B, 257, 300).to(DEV)
    else:
        img, aud = orc.make_image(_B, 96).to(DEV), orc.make_spectrogram(_B, 97, 110).to(DEV)
    runs = []
    NR = int(os.environ.get("DET_RUNS", "3"))
    for r in range(NR):
        m = AVENet(HardWayArgs(), False)
        m.load_state_dict(orc.make_state(3))
        m = m.to(DEV).train()
        step = HardWayTrainStep(m, lr=1e-4, weight_decay=1e-4)
        per_step = []
        for _ in range(3):
            loss = step.step(img, aud).item()
            torch.cuda.synchronize()
            if os.environ.get("DET_KEEP"):
                _keep.clear()
            per_step.append((loss, step.grad.clone()))
        runs.append((m, per_step))
    m0 = runs[0][0]
    for s in range(3):
        g0 = runs[0][1][s][1]
        for r in range(1, NR):
            g = runs[r][1][s][1]
            if torch.equal(g, g0):
                print(f"step {s} run {r}: equal (loss {runs[r][1][s][0]} vs {runs[0][1][s][0]})", flush=True)
                continue
            v0, v = m0._flat.grad_views(g0), m0._flat.grad_views(g)
            bad = [(n, (v[n] - v0[n]).abs().max().item()) for n in v0 if not torch.equal(v[n], v0[n])]
            print(f"step {s} run {r}: {len(bad)} of {len(v0)} tensors differ; loss {runs[r][1][s][0]} vs "
                  f"{runs[0][1][s][0]}", flush=True)
            for n, d in bad[-3:] if os.environ.get("DET_SHORT") else bad[:40]:
                print(f"   {n:50s} max|d| {d:.3e}", flush=True)


def cmd_calls(argv):
    """first divergence point between identical runs: the vision trunk's backward helper calls fingerprinted on the issuing stream (env DET_RUNS, DET_ONLY)"""
    LOG = []


    def csum(t):
        # exact fingerprint (on the issuing stream): sum of the raw 16-bit words as int64, plus a weighted sum
        w = t.contiguous().view(-1)
        w = w.view(torch.int16) if w.element_size() == 2 else w.view(torch.int32)
        w = w.to(torch.int64)
        idx = torch.arange(w.numel(), device=w.device, dtype=torch.int64) % 1009 + 1
        return torch.stack([w.sum(), (w * idx).sum()])


    def wrap(name):
        orig = getattr(T.Trunk, name)

        def f(self, *a, **k):
            # DET_ONLY=substr: fingerprint only the vision calls whose conv/BN name contains substr (fewer extra
            # launches: less perturbation of the two streams' timing)
            tag = a[-2].name if name in ("_dgrad", "_wgrad") and hasattr(a[-2], "name") else \
                (getattr(a[-2], "prefix", "") if len(a) >= 2 else "")
            for x in a:
                if hasattr(x, "prefix") and not tag:
                    tag = x.prefix
            on = self.prefix.startswith("imgnet") and os.environ.get("DET_ONLY", "") in tag
            ins = [csum(x) for x in a if isinstance(x, torch.Tensor)] if on else []
            extra = [csum(v) for kk, v in k.items() if isinstance(v, torch.Tensor)] if on else []
            r = orig(self, *a, **k)
            outs = [csum(x) for x in (r if isinstance(r, tuple) else (r,)) if isinstance(x, torch.Tensor)] if on else []
            if on:
                LOG.append((name, ins + extra, outs, tag))
            return r
        setattr(T.Trunk, name, f)


    for n in ("_dgrad", "_wgrad", "_bn_relu_bwd", "_bn_bwd_mask", "_bn_bwd", "_bn_bwd_premasked"):
        wrap(n)

    img, aud = orc.make_image(6, 96).to(DEV), orc.make_spectrogram(6, 97, 110).to(DEV)
    runs = []
    for r in range(int(os.environ.get("DET_RUNS", "6"))):
        m = AVENet(HardWayArgs(), False)
        m.load_state_dict(orc.make_state(3))
        m = m.to(DEV).train()
        step = HardWayTrainStep(m, lr=1e-4, weight_decay=1e-4)
        steps = []
        for s in range(3):
            LOG.clear()
            step.step(img, aud)
            torch.cuda.synchronize()
            steps.append(([(n, [x.tolist() for x in i], [x.tolist() for x in o], tag) for n, i, o, tag in LOG],
                          step.grad.clone()))
        runs.append(steps)
    for r in range(1, len(runs)):
        for s in range(3):
            (a, ga), (b, gb) = runs[0][s], runs[r][s]
            if not torch.equal(ga, gb):
                print(f"run {r} step {s}: final gradients differ", flush=True)
            for j, (x, y) in enumerate(zip(a, b)):
                if x != y:
                    which = "inputs" if x[1] != y[1] else "outputs"
                    print(f"run {r} step {s}: first divergence at vision call {j} {x[0]} {x[3]} ({which}); "
                          f"in {[i for i, (p, q) in enumerate(zip(x[1], y[1])) if p != q]} "
                          f"out {[i for i, (p, q) in enumerate(zip(x[2], y[2])) if p != q]}", flush=True)
                    break
            else:
                continue
            break
    print("done", flush=True)


def cmd_oob(argv):
    """cross-trunk corruption finder: one trunk's backward launch by launch, the other trunk's saved tensors compared after every launch"""
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


def cmd_concurrency(argv):
    """concurrent (audio trunk on a side stream) vs sequential train steps: losses over several steps"""
    def run(conc, graph, steps=6, B=2):
        m = AVENet(orc.Args(), False)
        m.load_state_dict(orc.make_state(0))
        m = m.to(DEV).train()
        s = HardWayTrainStep(m, lr=1e-6)
        s.engine.concurrent = conc
        img, aud = orc.make_image(B, 64).to(DEV), orc.make_spectrogram(B, 65, 76).to(DEV)
        out = []
        for i in range(steps):
            out.append(round(s.step(img, aud).item(), 6))
            if graph and i == 0:
                s.capture(img.clone(), aud.clone())
        return out


    for conc, graph in [(False, False), (True, False), (True, False), (False, True), (True, True)]:
        print("concurrent", conc, "graph", graph, run(conc, graph))


    def run_two_shards(conc, steps=4):
        m = AVENet(orc.Args(), False)
        m.load_state_dict(orc.make_state(0))
        m = m.to(DEV).train()
        ref = HardWayTrainStep(m, lr=1e-6)
        ref.engine.concurrent = conc
        img, aud = orc.make_image(4, 64), orc.make_spectrogram(4, 65, 76)
        shards = [(img[r * 2:(r + 1) * 2].to(DEV), aud[r * 2:(r + 1) * 2].to(DEV)) for r in range(2)]
        out = [[], []]
        for _ in range(steps):
            gsum = torch.zeros_like(ref.grad)
            for r, (i, a) in enumerate(shards):
                out[r].append(round(ref._fwd_bwd(i, a).item(), 6))
                gsum += ref.grad
            ref.opt.step(gsum, grad_scale=0.5)
        return out


    for conc in (False, True, True):
        print("two shards concurrent", conc, run_two_shards(conc))


def cmd_spread(argv):
    """run-to-run gradient spread of the fused and drop-in paths (1-frame and two-view)"""
    def model():
        m = AVENet(orc.Args(), False)
        m.load_state_dict(orc.make_state(0))
        return m.to(DEV).train()


    def fused1(img, aud):
        m = model()
        s = HardWayTrainStep(m)
        s.opt.lr = 0.0
        s.step(img, aud)
        return s.grad.clone()


    def dropin1(img, aud):
        m = model()
        _, lg, _, _, _ = m(img, aud)
        torch.nn.CrossEntropyLoss()(lg, torch.zeros(lg.shape[0], dtype=torch.long, device=DEV)).backward()
        g = torch.zeros(m._flat.n_train, device=DEV)
        views = m._flat.grad_views(g)
        for n, p in m.named_parameters():
            if n in views and p.grad is not None:
                views[n].copy_(p.grad.permute(0, 2, 3, 1) if p.grad.dim() == 4 else p.grad)
        return g


    def fused2(fr, au, sp, dedup):
        m = model()
        s = TwoViewTrainStep(m, dedup_audio=dedup)
        s.opt.lr = 0.0
        s.step(fr, au, sp)
        return s.grad.clone()


    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()


    img, aud = orc.make_image(4, 64).to(DEV), orc.make_spectrogram(4, 65, 76).to(DEV)
    a, b = fused1(img, aud), fused1(img, aud)
    c, d = dropin1(img, aud), dropin1(img, aud)
    print("1-frame fused vs fused", rel(a, b), "dropin vs dropin", rel(c, d), "fused vs dropin", rel(a, c))
    fr, au, sp = orc.make_frames(2, 3, 64, 3).to(DEV), orc.make_frames(2, 3, 64, 4).to(DEV), orc.make_spectrogram(2, 65, 76).to(DEV)
    e, f = fused2(fr, au, sp, False), fused2(fr, au, sp, False)
    h = fused2(fr, au, sp, True)
    print("two-view fused vs fused", rel(e, f), "dedup vs folded", rel(h, e))


COMMANDS = {"rep": cmd_rep, "runs": cmd_runs, "calls": cmd_calls, "oob": cmd_oob, "concurrency": cmd_concurrency, "spread": cmd_spread}

if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in COMMANDS:
        sys.exit(__doc__)
    COMMANDS[sys.argv[1]](sys.argv[2:])
