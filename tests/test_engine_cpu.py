"""CPU tests of the engine, data layer, checkpointing and bucket planning (no GPU needed).

The CPU backend (ops.cpu_ref) runs the same static schedule as the HIP kernels, so these pin the
engine's semantics against stock torch autograd on the reference module (model.VGG11)."""
import os

import pytest
import torch
import torch.nn.functional as F

from distributed_pytorch_amd.data import DeviceLoader, ShardSampler, synthetic_cifar
from distributed_pytorch_amd.engine import VGGEngine, conv_cfg
from distributed_pytorch_amd.models import VGG11, VGG13, VGGSpec
from distributed_pytorch_amd.parallel.sync import plan_buckets
from distributed_pytorch_amd.utils import checkpoint


def _x4(x):
    x4 = torch.zeros(x.shape[0], x.shape[2], x.shape[3], 4)
    x4[..., :3] = x.float().permute(0, 2, 3, 1)
    return x4


def test_state_dict_layout_matches_reference():
    m = VGG11()
    e = VGGEngine("VGG11", "cpu", max_batch=2)
    ref = m.state_dict()
    sd = e.state_dict()
    assert list(sd.keys()) == list(ref.keys())
    assert len(sd) == 58
    for k in ref:
        assert sd[k].shape == ref[k].shape and sd[k].dtype == ref[k].dtype, k
    assert sum(v.numel() for v in m.parameters()) == 9231114


def test_load_state_dict_roundtrip():
    torch.manual_seed(3)
    m = VGG11()
    e = VGGEngine("VGG11", "cpu", max_batch=2)
    e.load_state_dict(m.state_dict())
    for k, v in e.state_dict().items():
        assert torch.equal(v, m.state_dict()[k]), k
    m2 = VGG11()
    m2.load_state_dict(e.state_dict())
    # the "module." prefix written by DDP-mode checkpoints is accepted
    e.load_state_dict({"module." + k: v for k, v in m.state_dict().items()})


def test_engine_grads_match_autograd():
    torch.manual_seed(1)
    m = VGG11().double()
    e = VGGEngine("VGG11", "cpu", max_batch=6)
    e.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in m.state_dict().items()})
    x = torch.randn(6, 3, 32, 32, dtype=torch.float64)
    t = torch.randint(0, 10, (6,))
    loss = F.cross_entropy(m(x), t)
    loss.backward()
    l2 = e.forward_backward(_x4(x), t)
    assert abs(l2.item() - loss.item()) < 1e-4
    for n, p in m.named_parameters():
        g = e._to_torch_layout(n, e.grads[n]).double()
        assert (g - p.grad).abs().max().item() < 1e-4 * max(1.0, p.grad.abs().max().item()), n


def test_engine_training_matches_torch_sgd():
    torch.manual_seed(1)
    m = VGG11().double()
    e = VGGEngine("VGG11", "cpu", max_batch=8, lr=0.01)
    e.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in m.state_dict().items()})
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator().manual_seed(0)
    for _ in range(3):
        x = torch.randn(8, 3, 32, 32, generator=g, dtype=torch.float64)
        t = torch.randint(0, 10, (8,), generator=g)
        opt.zero_grad()
        F.cross_entropy(m(x), t).backward()
        opt.step()
        e.forward_backward(_x4(x), t)
        e.sgd_step()
        e.finish_step()
    sd = e.state_dict()
    for k, v in m.state_dict().items():
        if v.is_floating_point():
            assert (sd[k].double() - v).abs().max().item() < 2e-4 * max(1.0, v.abs().max().item()), k
        else:
            assert int(sd[k]) == int(v) == 3
    # optimizer state is torch-SGD-compatible
    osd = e.optimizer_state_dict()
    ref = opt.state_dict()
    assert osd["param_groups"][0]["params"] == ref["param_groups"][0]["params"]
    for i in ref["state"]:
        a, b = osd["state"][i]["momentum_buffer"].double(), ref["state"][i]["momentum_buffer"]
        assert a.shape == b.shape
        assert (a - b).abs().max().item() < 2e-3 * max(1.0, b.abs().max().item())


def test_eval_matches_module_eval():
    torch.manual_seed(2)
    m = VGG11()
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.normal_(0, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
    m.eval()
    e = VGGEngine("VGG11", "cpu", max_batch=5)
    e.load_state_dict(m.state_dict())
    x = torch.randn(5, 3, 32, 32)
    t = torch.randint(0, 10, (5,))
    e.begin_eval()
    logits = torch.zeros(5, 10)
    e.eval_batch(_x4(x), t, logits)
    with torch.no_grad():
        ref = m(x)
    assert (logits - ref).abs().max().item() < 1e-3
    assert int(e.eval_acc[1]) == int((ref.argmax(1) == t).sum())


def test_other_vgg_depths_build():
    for name in ("VGG13", "VGG16", "VGG19"):
        spec = VGGSpec.from_name(name)
        assert spec.convs[-1].pool and spec.fc_in == 512
    e = VGGEngine("VGG13", "cpu", max_batch=2)
    assert list(e.state_dict().keys()) == list(VGG13().state_dict().keys())
    x = torch.randn(2, 3, 32, 32)
    loss = e.forward_backward(_x4(x), torch.tensor([1, 2]))
    assert torch.isfinite(loss).all()


@pytest.mark.parametrize("W,n", [(1, 50000), (2, 50000), (3, 1001), (8, 50000), (4, 10)])
def test_shard_sampler_matches_torch(W, n):
    from torch.utils.data.distributed import DistributedSampler

    for r in range(W):
        ours = ShardSampler(n, W, r, shuffle=True, seed=0)
        ref = DistributedSampler(list(range(n)), num_replicas=W, rank=r, shuffle=True, seed=0, drop_last=False)
        for ep in (0, 3):
            ours.set_epoch(ep)
            ref.set_epoch(ep)
            assert ours.indices().tolist() == list(iter(ref))
        assert len(ours) == len(ref)


def test_iterations_per_epoch():
    # W=1→196, 2→98, 4→49, 8→25 iterations at batch 256
    ds = synthetic_cifar(50000, 0)
    for W, it in ((1, 196), (2, 98), (4, 49), (8, 25)):
        ld = DeviceLoader(ds, 256, "cpu", sampler=ShardSampler(50000, W, 0))
        assert len(ld) == it


def test_device_loader_cpu():
    ds = synthetic_cifar(300, 0)
    ld = DeviceLoader(ds, 128, "cpu", sampler=ShardSampler(300, 2, 1), train=True, seed=3)
    shapes = [(x.shape[0], t.shape[0]) for x, t in ld]
    assert shapes == [(128, 128), (22, 22)]
    x, t = next(iter(ld))
    assert x.shape == (128, 32, 32, 4) and float(x[..., 3].abs().max()) == 0.0
    ld2 = DeviceLoader(ds, 128, "cpu", sampler=ShardSampler(300, 2, 1), drop_last=True)
    assert len(list(ld2)) == 1 and len(ld2) == 1


def test_bucket_plan():
    e = VGGEngine("VGG11", "cpu", max_batch=2)
    order = [["fc1.weight", "fc1.bias"]] + [
        [f"{l.conv_key}.weight", f"{l.conv_key}.bias", f"{l.bn_key}.weight", f"{l.bn_key}.bias"]
        for l in reversed(e.spec.convs)]
    for mb in (0, 1, 10, 25, 1000):
        bs = plan_buckets(e.grads, order, mb)
        names = [n for b in bs for n in b.names]
        assert sorted(names) == sorted(e.grads.names())
        covered = sorted((b.lo, b.hi) for b in bs)
        assert covered[0][0] == 0 and covered[-1][1] == e.grads.numel
        for (a0, a1), (b0, b1) in zip(covered, covered[1:]):
            assert a1 == b0
    bs = plan_buckets(e.grads, order, 10)
    assert all(b.numel * 4 <= 10 * 2 ** 20 for b in bs)
    assert bs[-1].numel * 4 <= 2 * 2 ** 20  # small tail bucket
    assert len(plan_buckets(e.grads, order, 0)) == 34


def test_conv_cfg_heuristic():
    # VGG-11 shapes at batch 256 — sane tiles/splits, enough blocks
    for M, N, K in [(262144, 64, 36), (65536, 128, 576), (16384, 256, 2304), (1024, 512, 4608)]:
        tile, s = conv_cfg("fprop", M, N, K)
        assert tile in (0, 1) and s >= 1 and K // s >= 32
        tile, s = conv_cfg("wgrad", M, N, K)
        assert tile == 1 and 1 <= s <= 128


def test_checkpoint_roundtrip(tmp_path):
    torch.manual_seed(0)
    e = VGGEngine("VGG11", "cpu", max_batch=4)
    x = torch.randn(4, 3, 32, 32)
    e.forward_backward(_x4(x), torch.tensor([0, 1, 2, 3]))
    e.sgd_step()
    e.finish_step()
    p = checkpoint.save(str(tmp_path), 1, e, epoch=0, batch_idx=7, world=2, mode="ddp", ddp_prefix=True)
    assert os.path.basename(p) == "rank1.pt"
    raw = torch.load(p, weights_only=True)
    assert all(k.startswith("module.") for k in raw["model"])
    m = VGG11()
    m.load_state_dict({k[7:]: v for k, v in raw["model"].items()})
    e2 = VGGEngine("VGG11", "cpu", max_batch=4)
    obj = checkpoint.load(str(tmp_path), 1, e2)
    assert obj["batch_idx"] == 7
    assert torch.equal(e2.params.flat, e.params.flat)
    assert torch.equal(e2.mom.flat, e.mom.flat)
    assert e2.steps_taken >= 1
    # the next step from the restored state is identical
    for eng in (e, e2):
        eng.forward_backward(_x4(x), torch.tensor([0, 1, 2, 3]))
        eng.sgd_step()
        eng.finish_step()
    assert torch.allclose(e2.params.flat, e.params.flat, atol=0, rtol=0)


def test_cifar10_binary_reader(tmp_path):
    """The CIFAR-10 binary release layout (label byte + 3072 CHW bytes per record) is read into
    HWC uint8 images with int64 labels; a missing dataset falls back to synthetic data."""
    import numpy as np

    from distributed_pytorch_amd.data import cifar

    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    rng = np.random.default_rng(0)
    recs = {}
    for name, n in [(f"data_batch_{i}.bin", 3) for i in range(1, 6)] + [("test_batch.bin", 4)]:
        r = rng.integers(0, 256, size=(n, 3073), dtype=np.uint8)
        r[:, 0] = rng.integers(0, 10, size=n)
        r.tofile(d / name)
        recs[name] = r
    tr = cifar.load_cifar10(str(tmp_path), True)
    te = cifar.load_cifar10(str(tmp_path), False)
    assert tr.images.shape == (15, 32, 32, 3) and te.images.shape == (4, 32, 32, 3)
    r0 = recs["data_batch_1.bin"][0]
    assert int(tr.labels[0]) == int(r0[0])
    chw = r0[1:].reshape(3, 32, 32)
    assert np.array_equal(tr.images[0].numpy(), chw.transpose(1, 2, 0))
    a, b = cifar.get_datasets(str(tmp_path / "nope"), False, 64, 32)
    assert len(a) == 64 and len(b) == 32


@pytest.mark.parametrize("mode", ["ddp", "allreduce", "gather"])
def test_fused_step_matches_single_update(mode, monkeypatch):
    """Per-bucket SGD queued inside backward (params_free + grad_ready) gives the same parameters
    and momentum, bit for bit, as one SGD over the arena after backward."""
    from distributed_pytorch_amd.parallel import NullComm, make_sync

    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(4, 3, 32, 32, generator=g) for _ in range(2)]
    ts = [torch.randint(0, 10, (4,), generator=g) for _ in range(2)]
    out = []
    for fused in ("1", "0"):
        monkeypatch.setenv("DPA_FUSED_STEP", fused)
        e = VGGEngine("VGG11", "cpu", max_batch=4, lr=0.05)
        e.init_parameters(seed=2)
        sync = make_sync(mode, e, NullComm(), bucket_mb=1.0 if mode == "ddp" else None)
        assert sync.fuse_step == (fused == "1")
        stepped = []
        for x, t in zip(xs, ts):
            sync.begin_step()
            e.forward_backward(_x4(x), t, grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                               params_free=sync.params_free)
            stepped.append(all(b.stepped for b in sync.buckets))  # all queued inside backward
            sync.update(sync.finish())
            e.finish_step()
        if fused == "1":
            assert all(stepped)
        out.append((e.params.flat.clone(), e.mom.flat.clone()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


def test_halo_tile_geometry_rules():
    """engine.halo_ok mirrors conv_x3.hip run_halo: 64-channel-chunk tiles (22, 23) need C % 64,
    never run x3's three planes, and with fp16 pairs stage rows of at most 16 pixels (one bf16 plane
    keeps the BM/4 - 1 limit of the other tiles)."""
    from distributed_pytorch_amd.engine import HALO_GEOM, halo_ok

    for t in (22, 23):
        assert HALO_GEOM[t] == (256, 64)
        assert halo_ok("fprop", t, 16, 64, 128, 2) and not halo_ok("fprop", t, 17, 64, 128, 2)
        assert halo_ok("fprop", t, 56, 64, 64, 1) and not halo_ok("fprop", t, 64, 64, 64, 1)
        assert not halo_ok("fprop", t, 8, 64, 128, 3)
        assert not halo_ok("dgrad", t, 8, 96, 128, 2)
    # the 32-channel tiles are unchanged: rows up to BM/4 - 1 for every plane count
    assert halo_ok("fprop", 17, 63, 32, 64, 3) and not halo_ok("fprop", 17, 64, 32, 64, 3)
    assert halo_ok("dgrad", 21, 31, 32, 64, 2) and not halo_ok("dgrad", 21, 32, 32, 64, 2)
