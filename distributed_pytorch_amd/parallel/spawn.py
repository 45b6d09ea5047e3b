"""Single-node N-rank launcher: ``python bench.py --gpus N`` without torchrun.

The reference starts one trainer per node by hand or through torchrun (README.md:4,
start_ddp.sh:1, main_ddp.py:93-104).  Here one node holds 8 MI355X, so the benches and the CLI
can start their own ranks: the parent picks a free rendezvous port on 127.0.0.1, starts N fresh
child processes of the same script with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set (the torchrun contract, so the children take the same ``env://``
path as under torchrun), and supervises them:

* the parent never touches the GPU (no HIP call, no ``torch.cuda`` query): children are fresh
  processes, never an exec of a GPU-initialised one;
* if any child exits non-zero (or is killed), the others are terminated (SIGTERM, then SIGKILL
  after a grace period) and the launcher returns that child's exit code;
* a wall-clock limit bounds the whole job (exit code 124 on expiry, as ``timeout``).

Each child runs in its own process group so that the teardown reaches any helper processes it
started; only the exact process groups started here are signalled.

The teardown also runs when the launcher itself is told to stop: SIGTERM / SIGHUP / SIGINT raise
into it (exit code 128 + signal).  And if the launcher dies without running it (SIGKILL, a crashed
interpreter), every child gets SIGTERM from the kernel (``PR_SET_PDEATHSIG``), so no rank is left
holding a GPU while its peers hang in a collective until the watchdog.
"""
from __future__ import annotations

import ctypes
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional, Sequence

SPAWNED_ENV = "DPA_SPAWNED"  # set in every child: the script must not spawn again


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def free_port_pair(host: str = "127.0.0.1", tries: int = 64) -> tuple:
    """Two free ports: MASTER_PORT (torch's store, if any) and the native store's port."""
    for _ in range(tries):
        a, b = free_port(host), free_port(host)
        if a != b:
            return a, b
    raise RuntimeError("no free port pair found")


def rank_env(rank: int, world: int, port: int, store_port: int, base: Optional[Dict[str, str]] = None,
             host: str = "127.0.0.1") -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": host,
                "MASTER_PORT": str(port), "DPA_STORE_PORT": str(store_port), SPAWNED_ENV: "1"})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
    return env


class _Stopped(Exception):
    def __init__(self, signum: int):
        super().__init__(signum)
        self.signum = signum


_STOP_SIGNALS = (signal.SIGTERM, signal.SIGHUP, signal.SIGINT)


def _die_with_parent(parent: int):
    """preexec_fn of every rank (runs in the child between fork and exec): SIGTERM when the launcher
    dies; exit at once if it is already gone.  The launcher blocks the stop signals while it starts
    ranks and exec keeps the signal mask, so the child unblocks them here."""
    signal.pthread_sigmask(signal.SIG_UNBLOCK, _STOP_SIGNALS)
    try:
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGTERM), 0, 0, 0)  # PR_SET_PDEATHSIG
    except OSError:
        pass
    if os.getppid() != parent:
        os._exit(1)


def _kill_group(p: subprocess.Popen, sig: int):
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def launch(script: str, argv: Sequence[str], nprocs: int, timeout_s: float = 1800.0, grace_s: float = 10.0,
           extra_env: Optional[Dict[str, str]] = None, python: Optional[str] = None) -> int:
    """Run ``python script *argv`` as ``nprocs`` ranks on this node; return the job's exit code
    (0 if every rank exited 0, else the first failing rank's code; 124 on timeout)."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    port, store_port = free_port_pair()
    procs: List[subprocess.Popen] = []
    py = python or sys.executable
    parent = os.getpid()
    old_handlers = {}
    if threading.current_thread() is threading.main_thread():
        def _on_signal(signum, _frame):
            raise _Stopped(signum)

        for sg in _STOP_SIGNALS:
            old_handlers[sg] = signal.signal(sg, _on_signal)
    code = 0
    failed: Optional[int] = None
    main = threading.current_thread() is threading.main_thread()
    try:
        # Stop signals stay pending while ranks start: one arriving between a fork and the append
        # below would otherwise leave a rank the teardown never signals.  They are
        # delivered (and raise into the teardown) once every started rank is in `procs`.
        if main:
            signal.pthread_sigmask(signal.SIG_BLOCK, _STOP_SIGNALS)
        try:
            for r in range(nprocs):
                env = rank_env(r, nprocs, port, store_port)
                if extra_env:
                    env.update(extra_env)
                procs.append(subprocess.Popen([py, script, *argv], env=env, start_new_session=True,
                                              preexec_fn=lambda: _die_with_parent(parent)))
        finally:
            if main:
                signal.pthread_sigmask(signal.SIG_UNBLOCK, _STOP_SIGNALS)
        deadline = time.monotonic() + timeout_s
        while True:
            alive = 0
            for r, p in enumerate(procs):
                rc = p.poll()
                if rc is None:
                    alive += 1
                elif rc != 0 and failed is None:
                    failed = r
                    code = rc if rc > 0 else 128 - rc  # killed by signal s -> 128 + s
                    print(f"[launch] rank {r} exited with {rc}; stopping the other ranks", file=sys.stderr,
                          flush=True)
            if failed is not None or alive == 0:
                break
            if time.monotonic() > deadline:
                print(f"[launch] job exceeded {timeout_s:.0f} s; stopping all ranks", file=sys.stderr, flush=True)
                code = 124
                break
            time.sleep(0.05)
    except _Stopped as e:
        print(f"[launch] launcher received signal {e.signum}; stopping all ranks", file=sys.stderr, flush=True)
        code = 128 + e.signum
    except KeyboardInterrupt:
        code = 130
    finally:
        # a second signal during the teardown must not abort it half-way
        for sg in old_handlers:
            signal.signal(sg, signal.SIG_IGN)
        live = [p for p in procs if p.poll() is None]
        for p in live:
            _kill_group(p, signal.SIGTERM)
        t_end = time.monotonic() + grace_s
        for p in live:
            try:
                p.wait(max(0.0, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                _kill_group(p, signal.SIGKILL)
                p.wait()
        for sg, h in old_handlers.items():
            signal.signal(sg, h)
    return code


def is_spawned_child() -> bool:
    return os.environ.get(SPAWNED_ENV) == "1"


def needs_spawn(requested_world: int) -> bool:
    """True when the caller asked for N>1 ranks but was started as a single plain process (no
    torchrun / launcher environment)."""
    return requested_world > 1 and "WORLD_SIZE" not in os.environ and not is_spawned_child()
