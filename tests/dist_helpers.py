"""Worker functions for the multi-process (gloo, CPU) tests.  Spawned processes import this
module by name, so it must stay importable (tests/ is on sys.path in the children)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.nn.functional as F


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)


def _batches(rank, steps, n=4, seed=100):
    g = torch.Generator().manual_seed(seed + rank)
    out = []
    for _ in range(steps):
        x = torch.randn(n, 3, 32, 32, generator=g)
        t = torch.randint(0, 10, (n,), generator=g)
        out.append((x, t))
    return out


def _x4(x):
    x4 = torch.zeros(x.shape[0], 32, 32, 4)
    x4[..., :3] = x.permute(0, 2, 3, 1)
    return x4


def run_engine_mode(rank, world, port, mode, steps, outdir, bucket_mb=None, overlap=True, lr=0.01):
    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.parallel import TorchComm, make_sync

    _init(rank, world, port)
    comm = TorchComm(device=torch.device("cpu"))
    # deliberately different init on rank 1: the start-up broadcast must make replicas identical
    e = VGGEngine("VGG11", "cpu", max_batch=4, lr=lr)
    e.init_parameters(seed=1 + rank)
    sync = make_sync(mode, e, comm, bucket_mb=bucket_mb, overlap=overlap)
    losses = []
    for x, t in _batches(rank, steps):
        sync.begin_step()
        e.forward_backward(_x4(x), t, grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                           params_free=sync.params_free)
        sync.update(sync.finish())
        e.finish_step()
        losses.append(float(e.loss.item()))
    if mode == "ddp":
        wait = sync.pre_forward()  # what the first eval forward does
        if wait is not None:
            wait()
    sync.prepare_checkpoint()  # zero1: all-gather the momentum shards (no-op for the other modes)
    torch.save({"params": e.params.flat.clone(), "buffers": e.buffers.flat.clone(), "losses": losses,
                "mom": e.mom.flat.clone(), "sd": e.state_dict()}, os.path.join(outdir, f"{mode}_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def run_torch_ddp(rank, world, port, steps, outdir, lr=0.01):
    """Oracle: stock torch DistributedDataParallel on the reference module (main_ddp.py:137)."""
    from torch.nn.parallel import DistributedDataParallel

    from distributed_pytorch_amd.models import VGG11

    _init(rank, world, port)
    torch.manual_seed(1)
    m = DistributedDataParallel(VGG11())
    opt = torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
    losses = []
    for x, t in _batches(rank, steps):
        opt.zero_grad()
        loss = F.cross_entropy(m(x), t)
        loss.backward()
        opt.step()
        losses.append(float(loss.item()))
    m.eval()
    with torch.no_grad():
        m(torch.zeros(1, 3, 32, 32))  # first eval forward broadcasts rank 0's buffers
    torch.save({"sd": m.module.state_dict(), "losses": losses}, os.path.join(outdir, f"torchddp_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def run_cli_main(rank, world, port, script, args, outfile):
    """Run one of the CLI entry points in-process (rank from the reference-style CLI flags)."""
    import contextlib
    import io
    import runpy
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    torch.set_num_threads(1)
    sys.argv = [script, "--master-ip", "127.0.0.1", "--num-nodes", str(world), "--rank", str(rank), "--port",
                str(port)] + list(args)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        runpy.run_path(os.path.join(root, script), run_name="__main__")
    with open(outfile, "w") as f:
        f.write(buf.getvalue())


def run_uid_exchange(rank, world, port, outdir):
    """The RCCL bootstrap's store exchange, with a fake id generator (runs on CPU/gloo)."""
    from distributed_pytorch_amd.parallel.comm import exchange_unique_id

    _init(rank, world, port)
    store = dist.distributed_c10d._get_default_store()
    uid = exchange_unique_id(store, rank, lambda: bytes(range(128)), tag="test_uid")
    with open(os.path.join(outdir, f"uid_{rank}.bin"), "wb") as f:
        f.write(uid)
    dist.barrier()
    dist.destroy_process_group()


def run_generic_ddp(rank, world, port, steps, outdir, impl="ours"):
    """Generic DDP wrapper (parallel/ddp.py) on a small ResNet vs stock torch DDP on the same
    network (float64, gloo)."""
    from torch.nn.parallel import DistributedDataParallel as TorchDDP

    from distributed_pytorch_amd.models.resnet import ResNet, ResNetRef
    from distributed_pytorch_amd.parallel import TorchComm
    from distributed_pytorch_amd.parallel.ddp import DistributedDataParallel, FlatSGD

    _init(rank, world, port)
    torch.manual_seed(5 + rank)  # different init per rank: the wrap-time broadcast must unify them
    ours = ResNet([1, 1, 1, 1], 10).double()
    torch.manual_seed(5)
    ref = ResNetRef([1, 1, 1, 1], 10).double()
    if rank == 0:
        ref.load_state_dict(ours.state_dict())
    g = torch.Generator().manual_seed(40 + rank)
    data = [(torch.randn(3, 3, 32, 32, generator=g, dtype=torch.float64), torch.randint(0, 10, (3,), generator=g))
            for _ in range(steps)]
    if impl == "ours":
        m = DistributedDataParallel(ours, TorchComm(device=torch.device("cpu")), bucket_mb=0.5)
        opt = FlatSGD(m, lr=0.05, momentum=0.9, weight_decay=1e-4)
        for x, t in data:
            opt.zero_grad()
            loss = F.cross_entropy(m(x.permute(0, 2, 3, 1).contiguous()), t)
            loss.backward()
            opt.step(m.finish())
        sd = ours.state_dict()
        nb = m.num_buckets()
    else:
        m = TorchDDP(ref)
        opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        for x, t in data:
            opt.zero_grad()
            F.cross_entropy(m(x), t).backward()
            opt.step()
        sd = ref.state_dict()
        nb = 0
    torch.save({"sd": sd, "nb": nb}, os.path.join(outdir, f"gddp_{impl}_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def run_native_store(rank, world, port, outdir):
    """Native C++ TCP store: RCCL-id exchange, barrier and max-reduce without torch.distributed."""
    import json

    from distributed_pytorch_amd.parallel.comm import exchange_unique_id
    from distributed_pytorch_amd.parallel.store import NativeStore

    import datetime
    import time

    st = NativeStore("127.0.0.1", port, rank, world, timeout_s=60)
    uid = exchange_unique_id(st, rank, lambda: bytes(range(128)), tag="uid")
    st.barrier("b1")
    mx = st.all_max("m", 1.5 * rank + 0.25)
    cnt = st.add("c", 1)
    st.barrier("b2")
    n0 = st.num_keys()
    for i in range(10):  # barriers and max-reduces clean up after themselves
        st.barrier(f"loop{i}")
        st.all_max(f"lm{i}", float(i + rank))
    st.barrier("b3")
    n1 = st.num_keys()
    t0 = time.monotonic()
    try:
        st.wait(["never-set"], datetime.timedelta(seconds=0.5))
        waited = None
    except RuntimeError:
        waited = time.monotonic() - t0
    st.barrier("b4")
    with open(os.path.join(outdir, f"ns_{rank}.json"), "w") as f:
        json.dump({"uid": list(uid), "max": mx, "cnt": cnt, "keys_before": n0, "keys_after": n1,
                   "bounded_wait_s": waited}, f)
    st.close()  # rank 0 keeps serving until every client checked out


def run_resume_agree(rank, world, port, ckdir, outdir, batch_idx_by_rank, world_saved=None, reshard=False):
    """Each rank writes a checkpoint (its own batch index, or none if None), then resumes through
    train.resume exactly like a training run; records what happened."""
    import argparse
    import json

    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.parallel import DistContext, TorchComm
    from distributed_pytorch_amd.train import resume
    from distributed_pytorch_amd.utils import checkpoint

    _init(rank, world, port)
    comm = TorchComm(device=torch.device("cpu"))
    ctx = DistContext(rank, world, rank, torch.device("cpu"), comm, True)
    e = VGGEngine("VGG11", "cpu", max_batch=4)
    bi = batch_idx_by_rank[rank] if rank < len(batch_idx_by_rank) else None
    if bi is not None:
        e.init_parameters(seed=11)
        e.steps_taken = 7
        checkpoint.save(ckdir, rank, e, 0, bi, 0, world_saved or world, "ddp", ddp_prefix=True)
    dist.barrier()
    e = VGGEngine("VGG11", "cpu", max_batch=4)
    args = argparse.Namespace(resume=True, checkpoint_dir=ckdir, resume_reshard=reshard)
    try:
        out = {"ok": list(resume(ctx, e, "ddp", args, 100)), "steps_taken": e.steps_taken,
               "param_sum": float(e.params.flat.double().sum())}
    except checkpoint.ResumeMismatch as ex:
        out = {"error": str(ex)}
    with open(os.path.join(outdir, f"resume_{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()
