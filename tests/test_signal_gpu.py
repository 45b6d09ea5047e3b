"""Kernel-start stream signals (signal.hip, common.h start_signal): the cross-stream dependency
the VGG engine uses instead of per-layer events on its critical-path stream."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from distributed_pytorch_amd import _ext

    return _ext.require()


def test_wait_orders_consumer_after_producer():
    """Stream B waits for a signal that stream A sets only after a long kernel; B's copy then
    sees A's data (written before the signal)."""
    C = _C()
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    sig = torch.zeros(1, dtype=torch.int32, device="cuda")
    tmo = torch.zeros(1, dtype=torch.int32, device="cuda")
    done = torch.zeros(1, dtype=torch.int32, device="cuda")
    src = torch.zeros(1 << 20, device="cuda")
    dst = torch.empty_like(src)
    torch.cuda.synchronize()
    with torch.cuda.stream(a):
        C.spin(20000, done)  # 20 ms: B's wait is certainly polling before the data exists
        src.fill_(7.0)
        C.set_signal(sig, 1)
    with torch.cuda.stream(b):
        C.wait_signal(sig, 1, 2_000_000, tmo)
        dst.copy_(src)
    torch.cuda.synchronize()
    assert int(tmo.item()) == 0
    assert int(done.item()) == 1
    assert torch.all(dst == 7.0)


def test_wait_gives_up_after_timeout():
    """A signal that never comes: the wait ends after its bound and reports it (no hang)."""
    C = _C()
    sig = torch.zeros(1, dtype=torch.int32, device="cuda")
    tmo = torch.zeros(1, dtype=torch.int32, device="cuda")
    C.wait_signal(sig, 5, 2000, tmo)  # 2 ms
    torch.cuda.synchronize()
    assert int(tmo.item()) == 1


def test_dgrad_signals_its_start():
    """conv_x3_dgrad with a signal word stores the value and computes the same result."""
    C = _C()
    g = torch.Generator().manual_seed(0)
    N, H, W, K, Cc = 4, 8, 8, 32, 16
    dz = torch.randn(N, H, W, K, generator=g).cuda()
    w = torch.randn(K, 3, 3, Cc, generator=g).cuda()
    dz3 = torch.empty(3, N, H, W, K, dtype=torch.bfloat16, device="cuda")
    w3 = torch.empty(3, K, 3, 3, Cc, dtype=torch.bfloat16, device="cuda")
    C.split_planes(dz.view(-1), dz3.view(3, -1))
    C.split_planes(w.view(-1), w3.view(3, -1))
    out0 = torch.empty(N, H, W, Cc, device="cuda")
    out1 = torch.empty_like(out0)
    sig = torch.zeros(1, dtype=torch.int32, device="cuda")
    C.conv_x3_dgrad(dz3, w3, out0, None, 1, 1)
    C.conv_x3_dgrad(dz3, w3, out1, None, 1, 1, sig=sig, sig_val=9)
    torch.cuda.synchronize()
    assert int(sig.item()) == 9
    assert torch.equal(out0, out1)
