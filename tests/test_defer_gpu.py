"""Deferred optimizer step (engine.defer_update, bench.py --defer-update): each step's SGD runs at
the start of the next step on the weight-gradient stream.  Parameters, momenta and losses must be
BITWISE those of the immediate update, through a state_dict / evaluation / checkpoint read in
between (which flush the pending update)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(defer: bool, steps: int = 4):
    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.parallel.comm import NullComm
    from distributed_pytorch_amd.parallel.sync import make_sync

    g = torch.Generator().manual_seed(11)
    xs = [torch.zeros(64, 32, 32, 4) for _ in range(steps)]
    for x in xs:
        x[..., :3] = torch.randn(64, 32, 32, 3, generator=g)
    ts = [torch.randint(0, 10, (64,), generator=g) for _ in range(steps)]
    e = VGGEngine("VGG11", "cuda", max_batch=64, impl="x3")
    e.init_parameters(seed=3)
    e.defer_update = defer
    sync = make_sync("ddp", e, NullComm(), overlap=True, broadcast_init=False)
    losses, mid = [], None
    for k in range(steps):
        sync.begin_step()
        loss = e.forward_backward(xs[k].cuda(), ts[k].cuda(), grad_ready=sync.grad_ready,
                                  pre_forward=sync.pre_forward, params_free=sync.params_free)
        losses.append(loss.clone())
        sync.update(sync.finish())
        e.finish_step()
        if k == 1:
            mid = e.state_dict()  # an outside read between steps (flushes a deferred update)
    e.flush_update()
    torch.cuda.synchronize()
    e.check_signals()
    return (torch.stack(losses).cpu(), e.params.flat.clone(), e.mom.flat.clone(), e.wplanes.clone()
            if e.wplanes is not None else None, mid)


def test_deferred_update_bitwise():
    ref = _run(False)
    got = _run(True)
    assert torch.equal(ref[0], got[0]), "losses differ"
    assert torch.equal(ref[1], got[1]), "parameters differ"
    assert torch.equal(ref[2], got[2]), "momenta differ"
    if ref[3] is not None:
        assert torch.equal(ref[3], got[3]), "weight planes differ"
    for k in ref[4]:
        assert torch.equal(ref[4][k], got[4][k]), k


def test_deferred_update_pending_state():
    from distributed_pytorch_amd.engine import VGGEngine

    e = VGGEngine("VGG11", "cuda", max_batch=8, impl="x3")
    e.init_parameters(seed=1)
    e.defer_update = True
    x = torch.zeros(8, 32, 32, 4, device="cuda")
    t = torch.zeros(8, dtype=torch.long, device="cuda")
    e.forward_backward(x, t)
    e.sgd_step_deferred(1.0)
    e.finish_step()
    assert e._pending_upd is not None
    e.flush_update()
    assert e._pending_upd is None and not e._upd_wait
    e.forward_backward(x, t)
    e.sgd_step_deferred(1.0)
    e.finish_step()
    e.forward_backward(x, t)  # issues the pending update on the side stream, waits inside the forward
    assert e._pending_upd is None and not e._upd_wait
    torch.cuda.synchronize()
