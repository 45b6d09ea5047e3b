"""Native RCCL communicator on real GPUs.

One GPU (always runs on the box):
* the watchdog's timeout path: a collective held behind a long kernel on the comm stream is declared
  dead after ``timeout_s``; the communicator is aborted and every later issue raises;
* K11 mean-of-W at W = 2/4/8 (gather mode's rank-0 reduction, main_gather.py:53-55);
* ``comm_count`` (ncclCommCount) of a 1-rank communicator.

Two or more GPUs (skipped on a 1-GPU box; RCCL refuses two ranks on one device): W = min(#GPUs, 4)
ranks started as plain processes through parallel/spawn.py, bootstrapped by the native store:
* every sync mode leaves bitwise-identical parameters on all ranks; the modes agree;
* ddp equals a single-process oracle that averages the W ranks' gradients (DDP semantics);
* ddp/zero1 BN buffers equal rank 0's after the eval pre-forward (main_ddp.py:137);
* a rank that dies mid-training makes the survivor exit 70 within DPA_COMM_TIMEOUT.
"""
import os
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "rccl_worker.py")


def _C():
    from distributed_pytorch_amd import _ext

    return _ext.require()


def test_watchdog_times_out_a_stuck_collective():
    C = _C()
    c = C.RcclComm(0, 1, C.rccl_unique_id(), 0, timeout_s=0.5, poll_s=0.05, exit_on_error=False)
    assert c.comm_count() == 1
    done = torch.zeros(1, dtype=torch.int32, device="cuda")
    t = torch.ones(1024, device="cuda")
    comm_stream = torch.cuda.ExternalStream(c.stream_ptr(), device="cuda:0")
    with torch.cuda.stream(comm_stream):
        C.spin(2_000_000, done)  # ~2 s on the comm stream: the next collective cannot complete before it
        c.all_reduce(t, "sum")
    deadline = time.time() + 10
    err = ""
    while not err and time.time() < deadline:
        time.sleep(0.05)
        err = c.async_error()
    assert "outstanding" in err and "timeout" in err, err
    with pytest.raises(RuntimeError, match="aborted"):
        c.all_reduce(t, "sum")
    assert c.comm_count() == -1
    comm_stream.synchronize()  # the spin kernel drains (bounded loop) before the test ends
    assert int(done.item()) == 1


@pytest.mark.parametrize("W", [2, 4, 8])
@pytest.mark.parametrize("n", [1, 4097, 9231114 // 8])
def test_mean_of_w(W, n):
    C = _C()
    g = torch.Generator().manual_seed(W * 7 + n)
    inp = torch.randn(W * n, generator=g) * 3
    out = torch.empty(n, device="cuda")
    C.mean_of_w(inp.cuda(), out, W)
    torch.cuda.synchronize()
    ref = inp.view(W, n).double().mean(0)
    d = (out.cpu().double() - ref).abs().max().item()
    assert d <= 4e-7 * max(1.0, ref.abs().max().item()), d
    assert torch.allclose(out.cpu(), torch.stack(list(inp.view(W, n))).mean(0), rtol=1e-6, atol=1e-6)


# ---------------------------------------------------------------------------------------- multi-GPU
def _ngpu():
    return torch.cuda.device_count()


multi = pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (RCCL refuses two ranks on one device)")


def _run_ranks(W, args, env_extra=None, timeout=300):
    from distributed_pytorch_amd.parallel import spawn

    return spawn.launch(WORKER, args, W, timeout_s=timeout, extra_env=env_extra or {})


@pytest.fixture(scope="module")
def mode_runs(tmp_path_factory):
    W = min(_ngpu(), 4)
    d = str(tmp_path_factory.mktemp("rccl"))
    out = {}
    for mode in ("gather", "allreduce", "ddp", "zero1"):
        rc = _run_ranks(W, [mode, "3", d], {"DPA_COMM_TIMEOUT": "120"})
        assert rc == 0, f"{mode}: ranks exited with {rc}"
        out[mode] = [torch.load(os.path.join(d, f"{mode}_{r}.pt"), weights_only=True) for r in range(W)]
    return W, out


@multi
@pytest.mark.parametrize("mode", ["gather", "allreduce", "ddp", "zero1"])
def test_rccl_replicas_bitwise_identical(mode_runs, mode):
    W, out = mode_runs
    r0 = out[mode][0]
    assert r0["comm"] == "rccl" and r0["world"] == W and r0["rccl_world"] == W
    for r in range(1, W):
        assert torch.equal(out[mode][r]["params"], r0["params"]), f"{mode}: rank {r} diverged"


@multi
def test_rccl_modes_agree(mode_runs):
    _, out = mode_runs
    a = out["gather"][0]["params"]
    for m in ("allreduce", "ddp", "zero1"):
        b = out[m][0]["params"]
        assert (a - b).abs().max().item() <= 1e-5 * max(1.0, a.abs().max().item()), m


@multi
def test_rccl_ddp_matches_gradient_average_oracle(mode_runs):
    """DDP semantics without any communicator: one process runs every rank's batch, averages the W
    gradients and steps (the reference's main_ddp.py:137 result, computed serially)."""
    from distributed_pytorch_amd.engine import VGGEngine

    W, out = mode_runs
    runs = out["ddp"]
    e = VGGEngine("VGG11", "cuda", max_batch=32, impl="x3", lr=0.01)
    e.init_parameters(seed=1)
    steps = len(runs[0]["losses"])
    acc = torch.zeros_like(e.grads.flat)
    for s in range(steps):
        acc.zero_()
        for r in range(W):
            x, t = runs[r]["data"][s]
            e.forward_backward(x.cuda(), t.cuda())
            torch.cuda.synchronize()
            assert abs(float(e.loss.item()) - runs[r]["losses"][s]) <= 1e-5 * max(1.0, runs[r]["losses"][s])
            acc += e.grads.flat
        e.grads.flat.copy_(acc)
        e.sgd_step(1.0 / W)
        e.finish_step()
    torch.cuda.synchronize()
    p = e.params.flat.cpu()
    q = runs[0]["params"]
    assert (p - q).abs().max().item() <= 1e-5 * max(1.0, q.abs().max().item())


@multi
@pytest.mark.parametrize("mode", ["ddp", "zero1"])
def test_rccl_ddp_buffers_from_rank0(mode_runs, mode):
    W, out = mode_runs
    for r in range(1, W):
        assert torch.equal(out[mode][r]["buffers"], out[mode][0]["buffers"])
    # modes A/B keep per-rank BN statistics
    assert not torch.equal(out["allreduce"][1]["buffers"], out["allreduce"][0]["buffers"])


@multi
def test_rccl_lost_peer_makes_survivor_exit_70(tmp_path):
    """Rank 1 dies after its first step; rank 0's next collective never completes (or RCCL reports
    the lost peer).  The native watchdog must end rank 0 with exit code 70 within the timeout instead
    of hanging."""
    from distributed_pytorch_amd.parallel import spawn

    port, store_port = spawn.free_port_pair()
    procs = []
    for r in range(2):
        env = spawn.rank_env(r, 2, port, store_port)
        env.update({"DPA_COMM_TIMEOUT": "5", "DPA_PG_TIMEOUT": "60"})
        procs.append(subprocess.Popen([sys.executable, WORKER, "ddp", "50", str(tmp_path), "--fault-rank", "1",
                                       "--fault-step", "1"], env=env, start_new_session=True))
    t0 = time.monotonic()
    try:
        rc1 = procs[1].wait(timeout=120)
        rc0 = procs[0].wait(timeout=120)
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
                p.wait()
    assert rc1 == 13
    assert rc0 == 70, rc0
    assert time.monotonic() - t0 < 120
