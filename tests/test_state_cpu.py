"""Checkpoint/resume safety and the CIFAR-10 loader's restricted unpickler (CPU)."""
import json
import os
import pickle

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import dist_helpers as H
from distributed_pytorch_amd.data.cifar import load_cifar10, safe_load_batch
from distributed_pytorch_amd.engine import VGGEngine
from distributed_pytorch_amd.utils import checkpoint


def test_checkpoint_refuses_other_topology(tmp_path):
    e = VGGEngine("VGG11", "cpu", max_batch=4)
    checkpoint.save(str(tmp_path), 0, e, 0, 37, 0, world=2, mode="ddp", ddp_prefix=True)
    with pytest.raises(checkpoint.ResumeMismatch, match="world size 2 -> 1"):
        checkpoint.load(str(tmp_path), 0, VGGEngine("VGG11", "cpu", max_batch=4), world=1, mode="ddp")
    with pytest.raises(checkpoint.ResumeMismatch, match="sync mode"):
        checkpoint.load(str(tmp_path), 0, VGGEngine("VGG11", "cpu", max_batch=4), world=2, mode="gather")
    obj = checkpoint.load(str(tmp_path), 0, VGGEngine("VGG11", "cpu", max_batch=4), world=2, mode="ddp")
    assert obj["batch_idx"] == 37


def test_checkpoint_reshard_restarts_the_epoch(tmp_path):
    e = VGGEngine("VGG11", "cpu", max_batch=4)
    e.init_parameters(seed=5)
    e.steps_taken = 3
    checkpoint.save(str(tmp_path), 0, e, 2, 37, 0, world=4, mode="ddp", ddp_prefix=True)
    e2 = VGGEngine("VGG11", "cpu", max_batch=4)
    with pytest.warns(UserWarning, match="restarting epoch 2 at batch 0"):
        obj = checkpoint.load(str(tmp_path), 0, e2, world=8, mode="ddp", reshard=True)
    assert obj["epoch"] == 2 and obj["batch_idx"] == 0 and e2.steps_taken == 3
    assert torch.equal(e2.params.flat, e.params.flat)


def _spawn(fn, world, *args):
    mp.start_processes(fn, args=(world, H.free_port()) + args, nprocs=world, join=True, start_method="spawn")


@pytest.mark.parametrize("case", ["different_iteration", "rank_without_checkpoint", "agree"])
def test_resume_point_must_agree_across_ranks(tmp_path, case):
    ck, out = str(tmp_path / "ck"), str(tmp_path)
    by_rank = {"different_iteration": [40, 20], "rank_without_checkpoint": [40, None], "agree": [40, 40]}[case]
    _spawn(H.run_resume_agree, 2, ck, out, by_rank)
    res = [json.load(open(os.path.join(out, f"resume_{r}.json"))) for r in range(2)]
    if case == "agree":
        assert res[0]["ok"] == res[1]["ok"] == [0, 40]
    else:  # every rank refuses (none is left waiting in a collective the others never issue)
        assert all("error" in r and "disagree" in r["error"] for r in res), res


def test_resume_topology_change_fails_on_every_rank(tmp_path):
    ck, out = str(tmp_path / "ck"), str(tmp_path)
    _spawn(H.run_resume_agree, 2, ck, out, [40, 40], 4)
    res = [json.load(open(os.path.join(out, f"resume_{r}.json"))) for r in range(2)]
    assert all("error" in r and "world size 4 -> 2" in r["error"] for r in res), res


def test_resume_reshard_onto_a_larger_world(tmp_path):
    """2 -> 4 ranks with --resume-reshard: ranks 2 and 3 have no file of their own and load rank 0's;
    every rank restarts the saved epoch at batch 0 with the same weights and step count."""
    ck, out = str(tmp_path / "ck"), str(tmp_path)
    _spawn(H.run_resume_agree, 4, ck, out, [40, 40], 2, True)
    res = [json.load(open(os.path.join(out, f"resume_{r}.json"))) for r in range(4)]
    assert all("ok" in r for r in res), res
    assert all(r["ok"] == [0, 0] and r["steps_taken"] == 7 for r in res), res
    assert len({r["param_sum"] for r in res}) == 1


def test_agree_pieces_are_exact():
    big = (1, 3, (1 << 40) + 1, (1 << 24) + 1)
    assert checkpoint._unpieces(checkpoint._pieces(big)) == list(big)
    assert checkpoint._unpieces(checkpoint._pieces((-1, -1, -1, -1))) == [-1, -1, -1, -1]
    p1, p2 = checkpoint._pieces((1, 0, 0, 1 << 24)), checkpoint._pieces((1, 0, 0, (1 << 24) + 1))
    assert torch.tensor(p1, dtype=torch.float32).tolist() != torch.tensor(p2, dtype=torch.float32).tolist()


def _write_py_release(root, payload_train, payload_test):
    d = root / "cifar-10-batches-py"
    d.mkdir()
    for i in range(1, 6):
        (d / f"data_batch_{i}").write_bytes(pickle.dumps(payload_train))
    (d / "test_batch").write_bytes(pickle.dumps(payload_test))


def test_cifar_python_release_loads(tmp_path):
    rng = np.random.default_rng(0)
    batch = {b"batch_label": b"x", b"labels": [1, 2, 3], b"data": rng.integers(0, 255, (3, 3072), dtype=np.uint8),
             b"filenames": [b"a.png", b"b.png", b"c.png"]}
    _write_py_release(tmp_path, batch, batch)
    tr = load_cifar10(str(tmp_path), True)
    assert tr.images.shape == (15, 32, 32, 3) and tr.labels.tolist() == [1, 2, 3] * 5
    assert torch.equal(tr.images[0].permute(2, 0, 1).reshape(-1), torch.from_numpy(batch[b"data"][0]))


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned > /dev/null",))


def test_cifar_loader_refuses_code_in_pickles(tmp_path):
    p = tmp_path / "evil"
    p.write_bytes(pickle.dumps({b"data": _Evil(), b"labels": []}))
    with pytest.raises(pickle.UnpicklingError, match="refusing"):
        safe_load_batch(str(p))


def test_json_metrics_carry_scaling_efficiency(tmp_path, capsys):
    from distributed_pytorch_amd.train import main_single

    p = tmp_path / "m.jsonl"
    main_single(["--device", "cpu", "--synthetic", "--train-size", "12", "--test-size", "4", "--batch-size", "4",
                 "--no-eval", "--json-metrics", str(p), "--single-gpu-img-s", "100"])
    rec = json.loads(p.read_text().splitlines()[-1])
    assert rec["world"] == 1 and rec["comm"] == "null" and rec["iters_run"] == 3
    assert abs(rec["scaling_efficiency"] - rec["images_per_sec_rank"] / 100) < 1e-12
