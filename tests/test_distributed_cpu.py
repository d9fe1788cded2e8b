"""Data-parallel semantics on CPU with the gloo backend (world_size 2).

The reference wraps AVENet in nn.DataParallel (train_hardway_1frame.py:93): every replica builds
its own B_local x (B_local+2) logits (model.py:114-115 reads B per replica), normalises BN with its
local batch, and the loss is the mean CE over the gathered rows.  The MI355X build runs one process
per GPU and sums the flat gradient with one all-reduce (avt_amd.train.sync_gradients), folding
1/world into Adam.  Here the oracle computes per-rank gradients, the product's sync functions
combine them over gloo, and the result must equal the single-process DataParallel gradient."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import avenet_oracle as orc

B_LOCAL, S, F, T = 2, 64, 65, 76


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _local_grads(rank):
    sd = orc.make_state(0, torch.float64)
    sd32 = orc.make_state(0)
    for k in sd:
        if sd[k].is_floating_point():
            sd[k] = sd32[k].double()
    img = orc.make_image(2 * B_LOCAL, S).double()[rank * B_LOCAL:(rank + 1) * B_LOCAL]
    aud = orc.make_spectrogram(2 * B_LOCAL, F, T).double()[rank * B_LOCAL:(rank + 1) * B_LOCAL]
    loss, _, grads = orc.train_step(sd, img, aud, None)
    names = sorted(grads)
    flat = torch.cat([grads[n].flatten() for n in names])
    return loss, flat, sd


def _worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import avtubes  # noqa: F401
        from avt_amd.train import sync_buffers, sync_gradients

        torch.set_num_threads(2)
        loss, flat, sd = _local_grads(rank)
        scale = sync_gradients(flat)
        flat.mul_(scale)
        # BN buffers: each rank updated its own running stats; after sync all hold rank 0's
        rv = sd["imgnet.bn1.running_var"].clone()
        sync_buffers(rv)
        if rank == 0:  # numpy copies travel by value (no shared-memory fds outliving the worker)
            out_q.put((flat.numpy().copy(), rv.numpy().copy(), scale))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_dp_gradient_equivalence_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    flat, rv0, scale = q.get(timeout=600)
    flat, rv0 = torch.from_numpy(flat), torch.from_numpy(rv0)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert scale == 0.5
    # single-process DataParallel reference: mean of the per-replica local-negative losses
    torch.set_num_threads(4)
    sd = orc.make_state(0, torch.float64)
    sd32 = orc.make_state(0)
    for k in sd:
        if sd[k].is_floating_point():
            sd[k] = sd32[k].double()
    img = orc.make_image(2 * B_LOCAL, S).double()
    aud = orc.make_spectrogram(2 * B_LOCAL, F, T).double()
    names = orc.trainable_names(sd)
    leaves = {n: sd[n].detach().clone().requires_grad_(True) for n in names}
    total = 0
    for r in range(world):
        work = dict(sd)
        work.update(leaves)
        for k in list(work):
            if "running" in k or "num_batches" in k:
                work[k] = sd[k].clone()
        _, logits, _, _, _ = orc.avenet_forward(work, img[r * B_LOCAL:(r + 1) * B_LOCAL],
                                                aud[r * B_LOCAL:(r + 1) * B_LOCAL])
        total = total + orc.hardway_ce(logits) * B_LOCAL
    loss = total / (world * B_LOCAL)  # CE mean over the gathered rows
    gl = torch.autograd.grad(loss, [leaves[n] for n in names])
    ref = torch.cat([g.flatten() for _, g in sorted(zip(names, gl), key=lambda x: x[0])])
    assert torch.allclose(flat, ref, rtol=1e-9, atol=1e-12)
    # rank 0's running stats win
    _, _, sd_r0 = _local_grads(0)
    assert torch.equal(rv0, sd_r0["imgnet.bn1.running_var"])


def test_local_negatives_differ_from_global():
    """Sanity: per-replica negatives (the reference DP behaviour) are not the global-batch loss."""
    sd = orc.make_state(0)
    img = orc.make_image(2 * B_LOCAL, S)
    aud = orc.make_spectrogram(2 * B_LOCAL, F, T)
    _, lg_all, _, _, _ = orc.avenet_forward(dict(sd), img, aud)
    assert lg_all.shape == (2 * B_LOCAL, 2 * B_LOCAL + 2)
    sd = orc.make_state(0)
    _, lg_half, _, _, _ = orc.avenet_forward(dict(sd), img[:B_LOCAL], aud[:B_LOCAL])
    assert lg_half.shape == (B_LOCAL, B_LOCAL + 2)
