"""Per-step health (VERDICT r5 "next round" 4a): every step snapshots the device error
words into pinned host memory without a synchronising read, and the NEXT step's finish raises if
any was set -- README's "fails the step" within one step, not at epoch end."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(impl="h2"):
    from distributed_pytorch_amd.engine import VGGEngine

    e = VGGEngine("VGG11", "cuda", max_batch=16, impl=impl)
    e.init_parameters(seed=1)
    torch.manual_seed(0)
    x = torch.zeros(16, 32, 32, 4, device="cuda")
    x[..., :3] = torch.randn(16, 32, 32, 3, device="cuda")
    t = torch.randint(0, 10, (16,), device="cuda")
    return e, x, t


def _step(e, x, t):
    e.forward_backward(x, t)
    e.sgd_step()
    e.finish_step()


def test_healthy_steps_pass():
    e, x, t = _engine()
    assert e.health
    for _ in range(4):
        _step(e, x, t)
    e.check_signals()
    names = e._health_names
    assert any("overflow" in n for n in names) and any("rendezvous" in n for n in names), names


@pytest.mark.parametrize("word", ["bn_tmo", "ksig_tmo"])
def test_timeout_word_fails_the_next_step(word):
    e, x, t = _engine()
    _step(e, x, t)
    _step(e, x, t)
    getattr(e, word).fill_(1)  # as if a bounded wait of this step had given up
    e.forward_backward(x, t)
    e.sgd_step()
    e.finish_step()  # snapshot of the bad step (slot k); checks step k-1: clean
    with pytest.raises(RuntimeError, match="health check"):
        _step(e, x, t)  # the next step's finish reads slot k
    getattr(e, word).zero_()


def test_fp16_pair_overflow_fails_the_next_step():
    from distributed_pytorch_amd import _ext

    C = _ext.require()
    C.h2_overflow(True)
    e, x, t = _engine()
    _step(e, x, t)
    torch.cuda.synchronize()
    try:
        # a weight beyond 65504 / H2_SW: the SGD kernel's fp16-pair split of it overflows
        e.params["layers.8.weight"][0, 0, 0, 0] = 1000.0
        _step(e, x, t)
        with pytest.raises(RuntimeError, match="fp16-pair overflow"):
            _step(e, x, t)
    finally:
        torch.cuda.synchronize()
        C.h2_overflow(True)


def test_health_off_switch(monkeypatch):
    monkeypatch.setenv("DPA_STEP_HEALTH", "0")
    e, x, t = _engine()
    assert not e.health
    _step(e, x, t)
    e.check_signals()
