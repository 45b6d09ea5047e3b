"""Time the small per-step kernels in isolation (fc head, BN stats/finalize, BN backward) at the
VGG-11 batch-256 shapes.   python tools/micro_small.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd import _ext  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    C = _ext.require()
    d = dict(device="cuda")
    B, Cin, J = 256, 512, 10
    x, w, b = torch.randn(B, Cin, **d), torch.randn(J, Cin, **d) * 0.05, torch.randn(J, **d)
    t = torch.randint(0, J, (B,), **d)
    lr, dl, dx = torch.empty(B, **d), torch.empty(B, J, **d), torch.empty(B, Cin, **d)
    dw, db, loss, acc = torch.empty(J, Cin, **d), torch.empty(J, **d), torch.zeros(1, **d), torch.zeros(1, **d)
    print(f"fc_ce_train      {timeit(lambda: C.fc_ce_train(x, w, b, t, lr, dl, dx, dw, db, loss, acc)):8.1f} us")
    for (N, H, Cc) in [(256, 32, 64), (256, 16, 128), (256, 8, 256), (256, 4, 512), (256, 2, 512)]:
        z = torch.randn(N, H, H, Cc, **d)
        part = torch.zeros(C.bn_part_floats(N * H * H, Cc, True), **d)
        g1, b1 = torch.ones(Cc, **d), torch.zeros(Cc, **d)
        outs = [torch.zeros(Cc, **d) for _ in range(4)]
        tf = timeit(lambda: C.bn_fwd_stats(z, 1, z, part, g1, b1, None, None, None, None, *outs, 0.1, 1e-5))
        a = torch.empty(N, H, H, Cc, **d)
        ta = timeit(lambda: C.bn_apply(z, a, outs[2], outs[3], False))
        print(f"bn N={N} H={H:2d} C={Cc:3d}: stats+finalize {tf:7.1f} us   apply {ta:7.1f} us")
    done = torch.zeros(1, dtype=torch.int32, device=db.device)
    print(f"empty-ish launch {timeit(lambda: C.spin(0, done)):8.1f} us")


if __name__ == "__main__":
    main()
