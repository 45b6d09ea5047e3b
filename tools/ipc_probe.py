"""Probe: can a process map another process's device buffer on the SAME GPU (hipIpcGetMemHandle /
hipIpcOpenMemHandle through torch's vendored HIP runtime)?  VERDICT r3 item 5 asks for this check
before building a peer-memory collective that a one-GPU lease can exercise.

    python tools/ipc_probe.py            # parent: never touches the GPU, starts 2 rank processes

Rank 0 allocates a float32 buffer, exports its handle through a file; rank 1 opens it, checks the
contents with a copy, writes new contents through a torch kernel on the mapped pointer
(``__cuda_array_interface__``), and rank 0 checks them.  Prints one JSON line.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

N = 1 << 20


def _hip():
    import torch

    return ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))


class _Handle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_ubyte * 64)]


class _Cai:
    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 2}


def _wait(path: str, timeout: float = 60.0):
    t0 = time.monotonic()
    while not os.path.exists(path):
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(path)
        time.sleep(0.01)


def rank0(d: str) -> dict:
    import torch

    hip = _hip()
    x = torch.arange(N, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    h = _Handle()
    rc = hip.hipIpcGetMemHandle(ctypes.byref(h), ctypes.c_void_p(x.data_ptr()))
    out = {"get_rc": rc}
    if rc != 0:
        open(os.path.join(d, "fail"), "w").close()
        return out
    base, size = ctypes.c_void_p(), ctypes.c_size_t()
    hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(x.data_ptr()))
    out["offset"] = x.data_ptr() - (base.value or x.data_ptr())  # the handle names the whole allocation
    with open(os.path.join(d, "h.tmp"), "wb") as f:
        f.write(ctypes.string_at(ctypes.addressof(h), 64))  # (a c_char field would stop at a NUL)
        f.write(int(out["offset"]).to_bytes(8, "little"))
    os.rename(os.path.join(d, "h.tmp"), os.path.join(d, "handle"))
    _wait(os.path.join(d, "done"))
    torch.cuda.synchronize()
    ok = bool(torch.equal(x, torch.arange(N, dtype=torch.float32, device="cuda") * 2 + 1))
    out["rank0_sees_peer_kernel_write"] = ok
    return out


def rank1(d: str) -> dict:
    import torch

    torch.cuda.init()
    hip = _hip()
    _wait(os.path.join(d, "handle"))
    h = _Handle()
    raw = open(os.path.join(d, "handle"), "rb").read()
    ctypes.memmove(ctypes.addressof(h), raw, 64)
    off = int.from_bytes(raw[64:72], "little")
    ptr = ctypes.c_void_p()
    rc = hip.hipIpcOpenMemHandle(ctypes.byref(ptr), h, ctypes.c_uint(1))
    out = {"open_rc": rc}
    if rc != 0:
        open(os.path.join(d, "done"), "w").close()
        return out
    y = torch.as_tensor(_Cai(ptr.value + off, N), device="cuda")
    out["rank1_reads_peer_buffer"] = bool(torch.equal(y, torch.arange(N, dtype=torch.float32, device="cuda")))
    y.mul_(2).add_(1)  # torch kernels writing through the mapped pointer
    torch.cuda.synchronize()
    open(os.path.join(d, "done"), "w").close()
    del y
    out["close_rc"] = hip.hipIpcCloseMemHandle(ptr)
    return out


def main() -> int:
    if len(sys.argv) > 2 and sys.argv[1] == "--rank":
        r, d = int(sys.argv[2]), sys.argv[3]
        res = (rank0 if r == 0 else rank1)(d)
        with open(os.path.join(d, f"r{r}.json"), "w") as f:
            json.dump(res, f)
        return 0
    d = tempfile.mkdtemp(prefix="ipc_probe_")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rank", str(r), d], env=env) for r in (0, 1)]
    codes = []
    for p in ps:
        try:
            codes.append(p.wait(timeout=180))
        except subprocess.TimeoutExpired:
            p.kill()
            codes.append(-9)
    res = {"exit_codes": codes}
    for r in (0, 1):
        pth = os.path.join(d, f"r{r}.json")
        if os.path.exists(pth):
            res.update(json.load(open(pth)))
    print(json.dumps(res), flush=True)
    return 0 if all(c == 0 for c in codes) else 1


if __name__ == "__main__":
    sys.exit(main())
