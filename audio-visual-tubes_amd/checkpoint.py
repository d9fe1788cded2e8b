"""Reference-compatible checkpoints.

The reference saves (train_hardway_1frame.py:257-263, train_hardway.py, train_3D.py)
    torch.save({'epoch': epoch, 'model_state_dict': model.state_dict(),
                'optimizer_state_dict': optim.state_dict()}, path)
with ``model`` wrapped in nn.DataParallel (keys prefixed ``module.``) and ``optim`` a torch.optim.Adam
over ``model.parameters()``, and loads with ``model_dict.update(checkpoint['model_state_dict'])``
(train_hardway.py:94-100, test_hardway_dataset.py:66-70, test.py:64-68).

Here the same files are read and written: model keys with or without ``module.``; the optimizer
state either of a torch-API optimizer (``avt_amd.optim.Adam`` / ``torch.optim.Adam``: its own
state_dict) or of the fused steps' flat Adam (``HardWayTrainStep`` / ``TwoViewTrainStep``), which is
converted to and from torch.optim.Adam's layout (state indexed by position in model.parameters(),
conv moments in OIHW) so a checkpoint moves between the reference and this build in both directions.
Files are read with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

PREFIX = "module."


def _strip(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {(k[len(PREFIX):] if k.startswith(PREFIX) else k): v for k, v in sd.items()}


def _fused_opt(obj):
    """The FlatAdam of a fused train step (or the FlatAdam itself), else None."""
    from .optim import FlatAdam

    if isinstance(obj, FlatAdam):
        return obj
    opt = getattr(obj, "opt", None)
    return opt if isinstance(opt, FlatAdam) else None


def flat_adam_state_dict(model: torch.nn.Module, opt) -> dict:
    """torch.optim.Adam.state_dict() layout of a FlatAdam over ``model``'s parameters."""
    flat = opt.flat
    names = [n for n, _ in model.named_parameters()]
    step = float(opt.t)
    state = {}
    for i, n in enumerate(names):
        if not flat.trainable(n):
            continue  # never receives a gradient: torch's Adam holds no state for it either
        off, shape = flat.poff[n]
        k = 1
        for s in shape:
            k *= s
        views = []
        for buf in (opt.exp_avg, opt.exp_avg_sq):
            t = buf[off:off + k]
            t = t.view(shape[0], shape[2], shape[3], shape[1]).permute(0, 3, 1, 2) if len(shape) == 4 else t.view(shape)
            views.append(t.detach().clone().contiguous())
        state[i] = {"step": torch.tensor(step), "exp_avg": views[0], "exp_avg_sq": views[1]}
    group = {"lr": opt.lr, "betas": tuple(opt.betas), "eps": opt.eps, "weight_decay": opt.wd, "amsgrad": False,
             "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
             "params": list(range(len(names)))}
    if getattr(opt, "initial_lr", None) is not None:  # what torch's schedulers add to the group
        group["initial_lr"] = opt.initial_lr
    return {"state": state, "param_groups": [group]}


def load_flat_adam_state_dict(model: torch.nn.Module, opt, sd: dict) -> None:
    """Inverse of flat_adam_state_dict (e.g. a reference checkpoint's optimizer_state_dict)."""
    flat = opt.flat
    names = [n for n, _ in model.named_parameters()]
    groups = sd["param_groups"]
    if len(groups) != 1:
        raise ValueError("avt: expected one Adam param group (train_hardway*.py builds one)")
    g = groups[0]
    if len(g["params"]) != len(names):
        raise ValueError(f"avt: optimizer state covers {len(g['params'])} parameters, model has {len(names)}")
    opt.lr, opt.betas, opt.eps, opt.wd = g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]
    opt.initial_lr = g.get("initial_lr")
    steps = set()
    with torch.no_grad():
        opt.exp_avg.zero_()
        opt.exp_avg_sq.zero_()
        for pos, idx in enumerate(g["params"]):
            st = sd["state"].get(idx)
            if st is None:
                continue
            n = names[pos]
            if not flat.trainable(n):
                continue  # a stale moment of a parameter this step never updates
            off, shape = flat.poff[n]
            k = 1
            for s in shape:
                k *= s
            for buf, key in ((opt.exp_avg, "exp_avg"), (opt.exp_avg_sq, "exp_avg_sq")):
                src = st[key].to(buf.device, torch.float32)
                if len(shape) == 4:
                    src = src.permute(0, 2, 3, 1)
                buf[off:off + k].copy_(src.reshape(-1))
            steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError(f"avt: per-parameter Adam steps differ ({sorted(steps)}); the flat Adam keeps one")
        opt.t_dev.fill_(steps.pop() if steps else 0)


def save_checkpoint(path, epoch: int, model: torch.nn.Module, optimizer=None, data_parallel: bool = True) -> dict:
    """Write the reference's checkpoint dict; ``data_parallel`` adds the ``module.`` prefix the
    reference's nn.DataParallel-wrapped state_dict carries."""
    msd = model.state_dict()
    if data_parallel:
        msd = {PREFIX + k: v for k, v in msd.items()}
    ck = {"epoch": epoch, "model_state_dict": msd}
    if optimizer is not None:
        fused = _fused_opt(optimizer)
        ck["optimizer_state_dict"] = flat_adam_state_dict(model, fused) if fused is not None else optimizer.state_dict()
    if path is not None:
        torch.save(ck, path)
    return ck


def load_checkpoint(path_or_dict, model: torch.nn.Module, optimizer=None, map_location="cpu") -> Optional[int]:
    """``model_dict.update(checkpoint['model_state_dict'])`` then load (keys with or without
    ``module.``; keys the model lacks raise, like load_state_dict on the updated dict would).
    Optionally restores the optimizer state.  Returns the checkpoint's epoch (or None)."""
    ck = path_or_dict
    if not isinstance(ck, dict):
        ck = torch.load(path_or_dict, map_location=map_location, weights_only=True)
    sd = ck.get("model_state_dict", ck)
    model_dict = model.state_dict()
    upd = _strip(sd)
    unknown = sorted(set(upd) - set(model_dict))
    if unknown:
        raise KeyError(f"avt: checkpoint keys not in the model: {unknown[:5]}{' ...' if len(unknown) > 5 else ''}")
    model_dict.update(upd)
    model.load_state_dict(model_dict)
    if optimizer is not None and "optimizer_state_dict" in ck:
        fused = _fused_opt(optimizer)
        if fused is not None:
            load_flat_adam_state_dict(model, fused, ck["optimizer_state_dict"])
        else:
            optimizer.load_state_dict(ck["optimizer_state_dict"])
    return ck.get("epoch")
