"""gemm_f32.hip (exact-fp32 matrix-core GEMM of the generic classifier head) vs fp64 matmul, in
every operand layout the head uses and on ragged shapes (bounds, split-K, bias)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K,ta,tb,bias", [
    (128, 1000, 2048, False, True, True),    # logits = feat @ W^T + b (ResNet-50 head)
    (128, 2048, 1000, False, False, False),  # dfeat = dl @ W
    (1000, 2048, 128, True, False, False),   # dW = dl^T @ feat
    (37, 53, 301, False, True, True),
    (64, 64, 32, True, True, False),
    (3, 5, 7, False, False, True),
])
def test_gemm_f32_matches_fp64(M, N, K, ta, tb, bias):
    from distributed_pytorch_amd.ops.functional import gemm_f32

    g = torch.Generator().manual_seed(M * 7 + N)
    a = torch.randn(*((K, M) if ta else (M, K)), generator=g)
    b = torch.randn(*((N, K) if tb else (K, N)), generator=g)
    bb = torch.randn(N, generator=g) if bias else None
    ref = (a.double().t() if ta else a.double()) @ (b.double().t() if tb else b.double())
    if bias:
        ref = ref + bb.double()
    out = gemm_f32(a.cuda(), b.cuda(), ta, tb, bb.cuda() if bias else None)
    torch.cuda.synchronize()
    err = ((out.double().cpu() - ref).abs().max() / ref.abs().max()).item()
    # fp32 products, fp32 accumulation over K: a few ulps of the largest partial sums
    assert err < 2e-6 * max(1.0, K / 256), err
    again = gemm_f32(a.cuda(), b.cuda(), ta, tb, bb.cuda() if bias else None)
    assert torch.equal(out, again)  # deterministic (fixed-order split-K)
