"""Multi-process data-parallel tests on CPU (gloo, world_size 2) — the SURVEY §4 oracle:
all three sync modes must leave identical parameters on every rank, agree with each other, and
agree with stock torch DistributedDataParallel on the reference module."""
import os
import re

import pytest
import torch
import torch.multiprocessing as mp

import dist_helpers as H

WORLD = 2
STEPS = 3


def _spawn(fn, *args):
    port = H.free_port()
    mp.start_processes(fn, args=(WORLD, port) + args, nprocs=WORLD, join=True, start_method="spawn")


@pytest.fixture(scope="module")
def mode_results(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("modes"))
    for mode in ("gather", "allreduce", "ddp", "zero1"):
        _spawn(H.run_engine_mode, mode, STEPS, d)
    _spawn(H.run_torch_ddp, STEPS, d)
    out = {}
    for name in ("gather", "allreduce", "ddp", "zero1", "torchddp"):
        out[name] = [torch.load(os.path.join(d, f"{name}_{r}.pt"), weights_only=True) for r in range(WORLD)]
    return out


@pytest.mark.parametrize("mode", ["gather", "allreduce", "ddp", "zero1"])
def test_replicas_identical(mode_results, mode):
    r0, r1 = mode_results[mode]
    assert torch.equal(r0["params"], r1["params"]), f"{mode}: parameters diverged across ranks"


def test_modes_agree(mode_results):
    a = mode_results["gather"][0]["params"]
    for m in ("allreduce", "ddp", "zero1"):
        b = mode_results[m][0]["params"]
        assert (a - b).abs().max().item() < 1e-5 * max(1.0, a.abs().max().item()), m
    # per-rank losses identical across modes (same data, same params each step)
    for r in range(WORLD):
        la = mode_results["gather"][r]["losses"]
        for m in ("allreduce", "ddp", "zero1"):
            lb = mode_results[m][r]["losses"]
            assert all(abs(x - y) < 1e-4 for x, y in zip(la, lb))


def test_zero1_checkpoint_momentum_is_complete(mode_results):
    """After prepare_checkpoint, every zero1 rank holds the full momentum arena (not just its
    shards) and it equals DDP's (same math, sharded update)."""
    ref = mode_results["ddp"][0]["mom"]
    for r in range(WORLD):
        m = mode_results["zero1"][r]["mom"]
        assert (m - ref).abs().max().item() <= 1e-5 * max(1.0, ref.abs().max().item()), r


def test_ddp_matches_torch_ddp(mode_results):
    ours = mode_results["ddp"][0]["sd"]
    ref = mode_results["torchddp"][0]["sd"]
    for k, v in ref.items():
        if v.is_floating_point():
            d = (ours[k].double() - v.double()).abs().max().item()
            assert d < 5e-4 * max(1.0, v.abs().max().item()), (k, d)
        else:
            assert int(ours[k]) == int(v)
    lo = mode_results["ddp"][0]["losses"]
    lr = mode_results["torchddp"][0]["losses"]
    assert all(abs(x - y) < 1e-3 for x, y in zip(lo, lr)), (lo, lr)


def test_ddp_eval_buffers_from_rank0(mode_results):
    # DDP semantics: the first eval forward broadcasts rank 0's BN buffers
    b0, b1 = mode_results["ddp"][0]["buffers"], mode_results["ddp"][1]["buffers"]
    assert torch.equal(b0, b1)
    # modes A/B keep per-rank BN statistics
    g0, g1 = mode_results["allreduce"][0]["buffers"], mode_results["allreduce"][1]["buffers"]
    assert not torch.equal(g0, g1)


def test_overlap_and_bucketing_do_not_change_results(tmp_path):
    d = str(tmp_path)
    _spawn(H.run_engine_mode, "ddp", 2, d, 1.0, False)
    a = torch.load(os.path.join(d, "ddp_0.pt"), weights_only=True)["params"]
    _spawn(H.run_engine_mode, "ddp", 2, d, 0.0, True)
    b = torch.load(os.path.join(d, "ddp_0.pt"), weights_only=True)["params"]
    assert torch.equal(a, b)


LOSS_RE = re.compile(r"^Epoch: 1, Iteration: (\d+)-(\d+), Average Loss: \d+\.\d{3}$")
TIME_RE = re.compile(r"^Avg Time for iteration (\d+)-(\d+): [0-9.e-]+ seconds\.$")
TEST_RE = re.compile(r"^Test set: Average loss: \d+\.\d{4}, Accuracy: \d+/(\d+) \(\d+%\)$")


@pytest.mark.parametrize("script", ["main_gather.py", "main_all_reduce.py", "main_part3.py"])
def test_cli_entrypoints_log_format(tmp_path, script):
    args = ["--device", "cpu", "--synthetic", "--batch-size", "8", "--max-iters", "41", "--train-size", "2000",
            "--test-size", "40"]
    outs = [str(tmp_path / f"out{r}.txt") for r in range(WORLD)]
    port = H.free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=H.run_cli_main, args=(r, WORLD, port, script, args, outs[r])) for r in range(WORLD)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(600)
        assert p.exitcode == 0
    for o in outs:
        lines = [l for l in open(o).read().splitlines() if l.strip()]
        loss_lines = [l for l in lines if l.startswith("Epoch:")]
        time_lines = [l for l in lines if l.startswith("Avg Time")]
        test_lines = [l for l in lines if l.startswith("Test set:")]
        assert [LOSS_RE.match(l).groups() for l in loss_lines] == [("1", "20"), ("21", "40")]
        assert [TIME_RE.match(l).groups() for l in time_lines] == [("2", "40")]
        assert len(test_lines) == 1 and TEST_RE.match(test_lines[0]).group(1) == "40"


def test_rccl_bootstrap_store_exchange(tmp_path):
    _spawn(H.run_uid_exchange, str(tmp_path))
    a = open(tmp_path / "uid_0.bin", "rb").read()
    b = open(tmp_path / "uid_1.bin", "rb").read()
    assert a == b == bytes(range(128))


def test_generic_ddp_matches_torch_ddp(tmp_path):
    """parallel/ddp.py (flat arenas, hook-issued buckets, fused FlatSGD) on a ResNet built from the
    kernel layers == torch DistributedDataParallel + SGD on the stock-torch ResNet."""
    d = str(tmp_path)
    _spawn(H.run_generic_ddp, 3, d, "ours")
    _spawn(H.run_generic_ddp, 3, d, "torch")
    ours = [torch.load(os.path.join(d, f"gddp_ours_{r}.pt"), weights_only=True) for r in range(WORLD)]
    ref = torch.load(os.path.join(d, "gddp_torch_0.pt"), weights_only=True)["sd"]
    assert ours[0]["nb"] > 1  # really bucketed
    for k, v in ref.items():
        a, b = ours[0]["sd"][k], ours[1]["sd"][k]
        if "running" not in k and "num_batches" not in k:
            assert torch.equal(a, b), f"{k}: replicas diverged"
        err = (a.double() - v.double()).abs().max() / v.double().abs().max().clamp_min(1e-12)
        assert err < 1e-6, (k, float(err))


def test_native_tcp_store(tmp_path):
    import json

    d = str(tmp_path)
    _spawn(H.run_native_store, d)
    res = [json.load(open(os.path.join(d, f"ns_{r}.json"))) for r in range(WORLD)]
    for r in res:
        assert r["uid"] == list(range(128))
        assert r["max"] == 1.5 * (WORLD - 1) + 0.25
    assert sorted(r["cnt"] for r in res) == list(range(1, WORLD + 1))
    for r in res:  # 10 barriers + 10 max-reduces leave at most one barrier's 3 keys in flight
        assert r["keys_after"] <= r["keys_before"] + 3, r
        assert r["bounded_wait_s"] is not None and 0.3 < r["bounded_wait_s"] < 5.0, r


def _run_ranks(script, args, outdir, world):
    port = H.free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=H.run_cli_main, args=(r, world, port, script, args, os.path.join(outdir, f"log{r}.txt")))
          for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(600)
        assert p.exitcode == 0


@pytest.mark.parametrize("script,world", [("main_part3.py", WORLD), ("main_all_reduce.py", WORLD)])
def test_preempt_and_resume_is_bitwise_identical(tmp_path, script, world):
    """a run stopped mid-epoch (--stop-after-iters, per-rank checkpoint) and resumed
    (--resume) ends with exactly the parameters, SGD momenta and position of an uninterrupted run."""
    base = ["--device", "cpu", "--synthetic", "--batch-size", "8", "--train-size", "96", "--test-size", "16",
            "--epochs", "2", "--no-eval"]  # 6 iterations per epoch per rank at W=2
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    _run_ranks(script, base + ["--checkpoint-dir", a], str(tmp_path), world)
    _run_ranks(script, base + ["--checkpoint-dir", b, "--stop-after-iters", "8"], str(tmp_path), world)
    mid = torch.load(os.path.join(b, "rank0.pt"), weights_only=True)
    assert (mid["epoch"], mid["batch_idx"]) == (1, 2)  # stopped inside the second epoch
    _run_ranks(script, base + ["--checkpoint-dir", b, "--resume"], str(tmp_path), world)
    for r in range(world):
        ca = torch.load(os.path.join(a, f"rank{r}.pt"), weights_only=True)
        cb = torch.load(os.path.join(b, f"rank{r}.pt"), weights_only=True)
        assert (ca["epoch"], ca["batch_idx"]) == (cb["epoch"], cb["batch_idx"]) == (2, 0)
        assert ca["model"].keys() == cb["model"].keys()
        for k in ca["model"]:
            assert torch.equal(ca["model"][k], cb["model"][k]), (r, k)
        for (ia, sa), (ib, sb) in zip(sorted(ca["optimizer"]["state"].items()), sorted(cb["optimizer"]["state"].items())):
            assert ia == ib and torch.equal(sa["momentum_buffer"], sb["momentum_buffer"]), (r, ia)


@pytest.mark.parametrize("kind", ["exit", "hang"])
def test_lost_rank_fails_peers_instead_of_hanging(tmp_path, monkeypatch, kind):
    """SURVEY §5.3 fault injection: rank 1 dies (or stops issuing collectives) at iteration 3; the
    surviving rank must fail with an error within the process-group timeout, never hang."""
    import time as _time

    monkeypatch.setenv("DPA_FAULT", f"1:3:{kind}")
    monkeypatch.setenv("DPA_PG_TIMEOUT", "20")
    args = ["--device", "cpu", "--synthetic", "--batch-size", "8", "--train-size", "160", "--test-size", "16",
            "--no-eval"]
    port = H.free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=H.run_cli_main, args=(r, WORLD, port, "main_part3.py", args,
                                                   str(tmp_path / f"log{r}.txt"))) for r in range(WORLD)]
    t0 = _time.monotonic()
    for p in ps:
        p.start()
    ps[0].join(240)
    took = _time.monotonic() - t0
    alive = ps[0].is_alive()
    for p in ps:
        if p.is_alive():
            p.kill()
            p.join()
    assert not alive, "surviving rank hung after its peer was lost"
    assert ps[0].exitcode != 0, "surviving rank finished as if nothing happened"
    if kind == "exit":
        assert ps[1].exitcode == 13
    assert took < 200, took
