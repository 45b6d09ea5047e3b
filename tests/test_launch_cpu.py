"""The single-node N-rank launcher (parallel/spawn.py) and the self-launching bench: what the
round-end driver runs as ``python bench.py --gpus N`` must start N ranks, report one JSON line,
and turn a failed or hung rank into a non-zero exit instead of a hang."""
import json
import os
import signal
import subprocess
import sys
import textwrap
import time

import pytest

from distributed_pytorch_amd.parallel import spawn
from distributed_pytorch_amd.utils.benchlib import strip_flag
from distributed_pytorch_amd.utils.profiling import rocprof_command

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _script(tmp_path, body):
    p = tmp_path / "child.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_launch_sets_rank_env(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    s = _script(tmp_path, f"""
        import os, json
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                "DPA_STORE_PORT", "{spawn.SPAWNED_ENV}")
        with open(os.path.join({str(out)!r}, os.environ["RANK"] + ".json"), "w") as f:
            json.dump({{k: os.environ[k] for k in keys}}, f)
        """)
    assert spawn.launch(s, [], 3, timeout_s=60) == 0
    envs = [json.loads((out / f"{r}.json").read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert len({e["MASTER_PORT"] for e in envs}) == 1 and envs[0]["MASTER_PORT"] != envs[0]["DPA_STORE_PORT"]
    assert all(e[spawn.SPAWNED_ENV] == "1" for e in envs)


def test_launch_failing_rank_stops_the_others(tmp_path):
    s = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)
        """)
    t0 = time.monotonic()
    rc = spawn.launch(s, [], 3, timeout_s=100, grace_s=5)
    assert rc == 3
    assert time.monotonic() - t0 < 30


def test_launch_timeout(tmp_path):
    s = _script(tmp_path, "import time\ntime.sleep(120)\n")
    t0 = time.monotonic()
    assert spawn.launch(s, [], 2, timeout_s=2, grace_s=2) == 124
    assert time.monotonic() - t0 < 30


def test_needs_spawn(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv(spawn.SPAWNED_ENV, raising=False)
    assert spawn.needs_spawn(2) and not spawn.needs_spawn(1)
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert not spawn.needs_spawn(2)  # torchrun already started the ranks


def test_profile_command_puts_python_right_after_dashes():
    cmd = rocprof_command(["bench.py", "--steps", "5"], outdir="gpurun_out/p")
    i = cmd.index("--")
    assert cmd[0] == "rocprofv3" and "--kernel-trace" in cmd and "--stats" in cmd
    assert cmd[i + 1] == sys.executable and cmd[i + 2:] == ["bench.py", "--steps", "5"]
    assert strip_flag(["--profile", "--steps", "5"], "--profile") == ["--steps", "5"]


@pytest.mark.slow
def test_bench_self_launch_two_ranks_cpu():
    """``bench.py --gpus 2`` with no launcher environment: 2 gloo ranks on CPU through the same
    spawn path the driver's 8-GPU run takes; one JSON line with the scaling fields."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", spawn.SPAWNED_ENV)}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--batch", "4", "--steps", "2", "--warmup", "1", "--solo-steps", "1",
                        "--comm-tune-steps", "1", "--comm-tune-budget", "500"],  # (a loaded CPU: every plan timed)
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "per_gpu_img_s", "scaling_efficiency", "rccl_world",
              "replicas_identical"):
        assert k in rec, k
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["parallelism"] == "dp2" and rec["config"]["launcher"] == "spawn"
    assert rec["config"]["global_batch"] == 8
    assert rec["replicas_identical"] is True
    assert rec["rccl_world"] is None  # gloo process group: no RCCL communicator exists
    assert rec["scaling_efficiency"] is not None and rec["value"] > 0
    # the warmup-time gradient-sync plan choice: every candidate timed, one chosen, reported
    tune = rec["config"]["comm_tune"]
    assert len(tune["ms_per_step"]) == 5 and all(v > 0 for v in tune["ms_per_step"].values())
    ch = tune["chosen"]
    assert rec["config"]["per_bucket_update"] == ch["per_bucket_update"]
    key = f"b{ch['bucket_mb']}_t{ch['tail_mb']}_{'fused' if ch['per_bucket_update'] else 'after'}"
    best, default = min(tune["ms_per_step"].values()), next(iter(tune["ms_per_step"].values()))
    assert tune["ms_per_step"][key] == best or (tune["ms_per_step"][key] == default and best > 0.99 * default)
    # the tuning steps leave no trace: the same run without tuning ends with the same parameters
    r2 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
                         "--batch", "4", "--steps", "2", "--warmup", "1", "--solo-steps", "0", "--diag-steps", "0",
                         "--comm-tune", "off"], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r2.returncode == 0, r2.stderr[-3000:]
    rec2 = json.loads([l for l in r2.stdout.splitlines() if l.startswith("{")][-1])
    assert rec2["config"]["comm_tune"] is None
    assert rec2["param_checksum"] == rec["param_checksum"] and rec2["final_loss"] == rec["final_loss"]


def test_bench_single_rank_reports_no_rccl_world():
    """A 1-GPU-style run has a null communicator: ``rccl_world`` must be None (not 1), and without
    --torch-baseline the stock-torch comparison fields are None (never a stale constant)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", spawn.SPAWNED_ENV)}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--batch", "4",
                        "--steps", "1", "--warmup", "1", "--diag-steps", "0"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == 1 and rec["config"]["comm"] == "null"
    assert rec["rccl_world"] is None
    assert rec["vs_torch_eager_fp32"] is None and rec["torch_eager_fp32_img_s"] is None


def test_comm_world_only_for_rccl():
    from distributed_pytorch_amd.parallel import NullComm
    from distributed_pytorch_amd.utils.benchlib import comm_world

    class FakeRccl:
        world = 4

        def comm_count(self):
            return 4

    assert comm_world(NullComm()) is None
    assert comm_world(FakeRccl()) == 4


def _alive(pid: int) -> bool:
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except FileNotFoundError:
        return False


@pytest.mark.parametrize("sig", [signal.SIGTERM, signal.SIGKILL])
def test_launcher_stop_takes_ranks_down(tmp_path, sig):
    """Stopping the self-launcher (SIGTERM: its handler runs the teardown; SIGKILL: the ranks'
    parent-death signal) leaves no rank running."""
    child = tmp_path / "child.py"
    child.write_text("import os, sys, time\n"
                     "open(os.path.join(sys.argv[1], 'pid' + os.environ['RANK']), 'w').write(str(os.getpid()))\n"
                     "time.sleep(120)\n")
    launcher = tmp_path / "launcher.py"
    launcher.write_text(f"import sys\nsys.path.insert(0, {ROOT!r})\n"
                        "from distributed_pytorch_amd.parallel import spawn\n"
                        f"sys.exit(spawn.launch({str(child)!r}, [{str(tmp_path)!r}], 2, timeout_s=300))\n")
    p = subprocess.Popen([sys.executable, str(launcher)], start_new_session=True)
    try:
        t_end = time.time() + 60
        files = [tmp_path / "pid0", tmp_path / "pid1"]
        while not all(f.exists() and f.read_text() for f in files):
            assert time.time() < t_end and p.poll() is None, "ranks did not start"
            time.sleep(0.1)
        pids = [int(f.read_text()) for f in files]
        assert all(_alive(q) for q in pids)
        os.kill(p.pid, sig)
        rc = p.wait(30)
        if sig == signal.SIGTERM:
            assert rc == 128 + signal.SIGTERM
        t_end = time.time() + 30
        while any(_alive(q) for q in pids):
            assert time.time() < t_end, "a rank outlived its launcher"
            time.sleep(0.1)
    finally:
        if p.poll() is None:
            p.kill()


def test_native_store_port_via_torchrun_agent_store(tmp_path):
    """Under torchrun the native store's port is published through the elastic agent's store (a
    TCPStore at MASTER_PORT): rank 0 binds an ephemeral port, the others read it."""
    import torch.distributed as dist

    from distributed_pytorch_amd import _ext

    if not _ext.available():
        pytest.skip("native extension not built")
    port = spawn.free_port()
    agent = dist.TCPStore("127.0.0.1", port, None, True)  # stands in for the torchrun agent's store
    out = tmp_path / "out"
    out.mkdir()
    s = _script(tmp_path, f"""
        import os, sys
        sys.path.insert(0, {ROOT!r})
        from distributed_pytorch_amd.parallel.launch import native_store_from_env
        r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        st = native_store_from_env(r, w)
        st.set(f"k{{r}}", str(r * 10))
        st.barrier("b")
        vals = [int(st.get(f"k{{q}}")) for q in range(w)]
        open(os.path.join({str(out)!r}, f"{{r}}.txt"), "w").write(f"{{st.port}} {{vals}}")
        st.close()
        """)
    env = {"TORCHELASTIC_USE_AGENT_STORE": "True", "TORCHELASTIC_RUN_ID": "t1", "MASTER_PORT": str(port)}
    procs = []
    for r in range(3):
        e = dict(os.environ, RANK=str(r), WORLD_SIZE="3", MASTER_ADDR="127.0.0.1", **env)
        e.pop("DPA_STORE_PORT", None)
        procs.append(subprocess.Popen([sys.executable, s], env=e))
    assert all(p.wait(timeout=120) == 0 for p in procs)
    res = [(out / f"{r}.txt").read_text().split(" ", 1) for r in range(3)]
    assert len({p for p, _ in res}) == 1 and int(res[0][0]) not in (port, port + 1)
    assert all(v == "[0, 10, 20]" for _, v in res)
    del agent


def test_native_store_under_real_torchrun(tmp_path):
    """The same exchange under an actual torch.distributed.run launch (static rendezvous, the
    driver's form): the elastic agent's store is reachable at MASTER_PORT and every rank gets the
    native store."""
    from distributed_pytorch_amd import _ext

    if not _ext.available():
        pytest.skip("native extension not built")
    out = tmp_path / "out"
    out.mkdir()
    s = _script(tmp_path, f"""
        import os, sys
        sys.path.insert(0, {ROOT!r})
        from distributed_pytorch_amd.parallel.launch import native_store_from_env
        r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        assert os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True", dict(os.environ)
        st = native_store_from_env(r, w)
        st.set(f"k{{r}}", str(r + 1))
        st.barrier("b")
        tot = sum(int(st.get(f"k{{q}}")) for q in range(w))
        open(os.path.join({str(out)!r}, f"{{r}}.txt"), "w").write(str(tot))
        st.close()
        """)
    env = dict(os.environ)
    for k in ("DPA_STORE_PORT", "WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
           "127.0.0.1", "--master-port", str(spawn.free_port()), s]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert [(out / f"{q}.txt").read_text() for q in range(3)] == ["6", "6", "6"]


def test_comm_plans_per_mode():
    """The warmup tuner's candidate gradient-sync plans: DDP tries bucket sizes, the tail bucket and
    the update placement (default plan first); per-tensor all-reduce keeps its granularity and only
    tries the update placement; gather / zero1 are not tuned; --bucket-mb pins the bucket size."""
    sys.path.insert(0, ROOT)
    import bench

    p = bench.comm_plans(bench.parse(["--mode", "ddp"]))
    assert p[0] == (10.0, 2.0, False, 0, False) and len(p) == 5 and len(set(p)) == 5
    assert {q[0] for q in p} == {10.0, 25.0, 5.0} and any(q[2] for q in p)
    assert any(q[1] < 2 for q in p) and all(q[3] == 0 and not q[4] for q in p)
    p = bench.comm_plans(bench.parse(["--mode", "ddp", "--bucket-mb", "8"]))
    assert {q[0] for q in p} == {8.0} and p[0] == (8.0, 2.0, False, 0, False)
    assert bench.comm_plans(bench.parse(["--mode", "allreduce"])) == [(None, 2.0, False, 0, False),
                                                                      (None, 2.0, True, 0, False)]
    assert bench.comm_plans(bench.parse(["--mode", "gather"])) == []
    assert bench.comm_plans(bench.parse(["--mode", "zero1"])) == []
    p = bench.comm_plans(bench.parse(["--mode", "ddp"]), ipc=True)  # ipc block budgets
    assert p[-3:] == [(10.0, 2.0, False, 0, 32), (10.0, 2.0, False, 0, 16), (10.0, 2.0, False, 0, 64)]
    assert len(p) == 8
    p = bench.comm_plans(bench.parse(["--mode", "ddp", "--ipc-blocks", "8"]), ipc=True)
    assert p[-1] == (10.0, 2.0, False, 0, 8) and len(p) == 6


def test_comm_plans_rccl_channel_budgets(monkeypatch):
    """with a native RCCL communicator the tuner also tries the default plan on
    channel-limited communicators (--rccl-channels); 'off' or a pinned DPA_RCCL_CHANNELS drops them."""
    sys.path.insert(0, ROOT)
    import bench

    monkeypatch.delenv("DPA_RCCL_CHANNELS", raising=False)
    p = bench.comm_plans(bench.parse(["--mode", "ddp"]), rccl=True)
    assert p[0] == (10.0, 2.0, False, 0, False)
    assert p[-2:] == [(10.0, 2.0, False, 16, False), (10.0, 2.0, False, 8, False)]
    p = bench.comm_plans(bench.parse(["--mode", "allreduce", "--rccl-channels", "4"]), rccl=True)
    assert p == [(None, 2.0, False, 0, False), (None, 2.0, True, 0, False), (None, 2.0, False, 4, False)]
    assert len(bench.comm_plans(bench.parse(["--mode", "ddp", "--rccl-channels", "off"]), rccl=True)) == 5
    monkeypatch.setenv("DPA_RCCL_CHANNELS", "12")
    assert len(bench.comm_plans(bench.parse(["--mode", "ddp"]), rccl=True)) == 5
    assert bench.comm_plans(bench.parse(["--mode", "gather"]), rccl=True) == []


def test_ipc_collective_pieces_cover_the_tensor():
    """csrc/runtime/ipc_comm.cpp IpcComm::pieces: a collective larger than what the staging buffer
    (all-reduce) or the inbox (bounced inputs) holds runs as consecutive pieces that cover it
    exactly, each a multiple of 4 words except the last (16-byte aligned offsets), each fitting its
    buffer; registered inputs of the copy collectives are one piece."""
    from distributed_pytorch_amd import _ext

    C = _ext.require()
    AR, BC, GA, RS, AG = 0, 1, 2, 3, 4
    for op, world, stage, inbox, n, reg in ((AR, 2, 1000, 1 << 20, 4099, True), (AR, 8, 65536, 1 << 22, 9_225_000, True),
                                            (AR, 4, 1 << 22, 1 << 22, 12345, True), (AR, 8, 1 << 22, 40_000, 9_231_114, False),
                                            (BC, 2, 4, 40_000, 100_003, False), (BC, 8, 4, 40_000, 100_003, True),
                                            (GA, 4, 4, 4096, 65_537, False), (RS, 2, 4, 40_000, 40_028, False),
                                            (RS, 8, 4, 40_000, 40_028, True), (AG, 3, 4, 40_000, 40_031, False)):
        ps = C.ipc_pieces(op, n, world, stage, inbox, reg)
        pos = 0
        for off, k in ps:
            assert off == pos and k > 0 and off % 4 == 0, (op, ps)
            pos += k
            if op == AR:
                sl = C.ipc_slice(k, world)
                assert sl <= stage and (reg or sl * world <= inbox), (op, k, sl)
            elif op == RS and not reg:
                assert k * world <= inbox
            elif not reg:
                assert k <= inbox
        assert pos == n, (op, n, ps)
        if reg and op != AR:
            assert len(ps) == 1
    assert C.ipc_pieces(AR, 0, 4, 1 << 20, 1 << 20, True) == []

def _bench8(extra_env, args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", spawn.SPAWNED_ENV)}
    env.update(OMP_NUM_THREADS="1", **extra_env)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--device", "cpu", "--batch", "2",
                        "--steps", "1", "--warmup", "1", "--solo-steps", "0", "--diag-steps", "0",
                        "--comm-tune-steps", "1"] + args, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_comm_tuner_eight_ranks_plan_dropped_on_one_rank():
    """VERDICT r5 item 6 (first 8-GPU contact): the warmup comm tuner at W = 8 (gloo ranks on CPU,
    the same bench.py code path).  A plan whose set-up fails on ONE rank (injected on rank 5) is
    dropped on EVERY rank -- the ranks keep identical plan lists, nothing hangs -- every other plan
    is timed, one is chosen, and the replicas end identical."""
    rec = _bench8({"DPA_TEST_TUNE_DROP": "5:1"}, [])
    tune = rec["config"]["comm_tune"]
    assert rec["n_gpus"] == 8 and rec["replicas_identical"] is True, rec
    assert tune["dropped_plans"] == 1 and tune["untimed_plans"] == 0 and not tune["budget_hit"], tune
    assert len(tune["ms_per_step"]) == 4 and "b25.0_t2.0_after" not in tune["ms_per_step"], tune
    assert tune["tune_seconds"] > 0 and tune["tune_seconds"] < tune["budget_s"], tune


def test_comm_tuner_eight_ranks_budget():
    """A spent wall-clock budget (agreed over the ranks) stops the tuner at the same plan on every
    rank; the default plan, always timed first, carries the run."""
    rec = _bench8({}, ["--comm-tune-budget", "0"])
    tune = rec["config"]["comm_tune"]
    assert rec["replicas_identical"] is True, rec
    assert tune["budget_hit"] is True and list(tune["ms_per_step"]) == ["b10.0_t2.0_after"], tune
    assert tune["chosen"] == {"bucket_mb": 10.0, "tail_mb": 2.0, "per_bucket_update": False, "rccl_channels": None,
                              "ipc_blocks": None}, tune
    assert tune["untimed_plans"] == 4, tune
