"""In-tree build of the native extension ``distributed_pytorch_amd/_C.so``.

Compiles every HIP kernel (``csrc/kernels/*.hip``) for gfx950 with ``hipcc`` and the host
runtime (``csrc/runtime/*.cpp`` + ``csrc/bindings.cpp``) with the host compiler, then links one
shared object against the HIP runtime and RCCL that PyTorch-ROCm itself vendors in
``torch/lib`` so a process has exactly one ``libamdhip64`` and one ``librccl``.

No hipify, no ``torch.utils.cpp_extension`` JIT cache: the ``.so`` lives next to this file so
it travels to the GPU box with the repo snapshot.

Usage::

    python -m distributed_pytorch_amd._build            # incremental
    python -m distributed_pytorch_amd._build --force    # rebuild everything
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import re
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
# DPA_NO_PACKED_FP32=1: every kernel built without gfx950's packed fp32 instructions (A/B build,
# written to build/native_nopk/_C.so; load it with DPA_EXT_SO=<path>, _ext.py)
# DPA_BUILD_TAG=<tag>: any A/B build of the working tree, to build/native_<tag>/_C.so likewise
NOPK = os.environ.get("DPA_NO_PACKED_FP32", "0") == "1"
TAG = os.environ.get("DPA_BUILD_TAG") or ("nopk" if NOPK else "")
BUILD_DIR = os.path.join(os.path.dirname(PKG_DIR), "build", "native_" + TAG if TAG else "native")
OUT_SO = os.path.join(BUILD_DIR, "_C.so") if TAG else os.path.join(PKG_DIR, "_C.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch  # noqa: F401  (only for paths)

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib")


def _sources():
    kern = sorted(os.path.join(CSRC, "kernels", f) for f in os.listdir(os.path.join(CSRC, "kernels")) if f.endswith(".hip"))
    host = sorted(os.path.join(CSRC, "runtime", f) for f in os.listdir(os.path.join(CSRC, "runtime")) if f.endswith(".cpp"))
    host.append(os.path.join(CSRC, "bindings.cpp"))
    return kern, host


_INC = re.compile(r'^\s*#\s*include\s*"([^"]+)"', re.M)


def _deps(src, seen=None):
    """The in-tree headers ``src`` includes, transitively (quoted includes resolved against the
    including file's directory, then csrc/): a source is rebuilt only when one of ITS headers
    changes."""
    seen = set() if seen is None else seen
    with open(src, encoding="utf-8", errors="replace") as f:
        text = f.read()
    for inc in _INC.findall(text):
        for base in (os.path.dirname(src), CSRC):
            h = os.path.normpath(os.path.join(base, inc))
            if os.path.isfile(h):
                if h not in seen:
                    seen.add(h)
                    _deps(h, seen)
                break
    return sorted(seen)


def _digest(path, extra):
    h = hashlib.sha1()
    with open(path, "rb") as f:
        h.update(f.read())
    for e in extra:
        with open(e, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _compile_cmd(src, obj, torch_inc):
    common = ["-O3", "-fPIC", "-std=c++17", "-I" + CSRC, "-I" + os.path.join(ROCM, "include"),
              "-D__HIP_PLATFORM_AMD__=1", "-Wno-unused-result"]
    if src.endswith(".hip"):
        nopk = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"] if NOPK else []
        return [os.path.join(ROCM, "bin", "hipcc"), "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
                "-c", src, "-o", obj] + common + nopk
    py_inc = sysconfig.get_paths()["include"]
    incs = ["-I" + p for p in torch_inc] + ["-I" + py_inc]
    return ["g++", "-c", src, "-o", obj, "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
            "-D_GLIBCXX_USE_CXX11_ABI=1", "-DUSE_ROCM=1", "-fvisibility=hidden"] + common + incs


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    tdir, torch_inc, torch_lib = _torch_paths()
    os.makedirs(BUILD_DIR, exist_ok=True)
    kern, host = _sources()
    jobs = jobs or max(1, min(8, os.cpu_count() or 1, int(os.environ.get("MAX_JOBS", "8"))))
    todo, objs = [], []
    for src in kern + host:
        rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
        obj = os.path.join(BUILD_DIR, rel + ".o")
        stamp = obj + ".sha1"
        dig = _digest(src, _deps(src))
        objs.append(obj)
        if force or not os.path.exists(obj) or not os.path.exists(stamp) or open(stamp).read() != dig:
            todo.append((src, obj, stamp, dig))

    def run(item):
        src, obj, stamp, dig = item
        cmd = _compile_cmd(src, obj, torch_inc)
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
        with open(stamp, "w") as f:
            f.write(dig)
        return src

    if todo:
        with cf.ThreadPoolExecutor(jobs) as ex:
            for s in ex.map(run, todo):
                print(f"[build] compiled {os.path.relpath(s, PKG_DIR)}", flush=True)
    need_link = bool(todo) or not os.path.exists(OUT_SO) or any(os.path.getmtime(o) > os.path.getmtime(OUT_SO) for o in objs)
    if need_link:
        tmp = OUT_SO + ".tmp"
        cmd = [os.path.join(ROCM, "bin", "hipcc"), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + [
            "-L" + torch_lib, "-Wl,-rpath," + torch_lib, "-Wl,--no-as-needed",
            "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            os.path.join(torch_lib, "librccl.so"), os.path.join(torch_lib, "libamdhip64.so")]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        shutil.move(tmp, OUT_SO)
        print(f"[build] linked {OUT_SO}", flush=True)
    return OUT_SO


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build(a.force, a.verbose, a.jobs)


if __name__ == "__main__":
    sys.exit(main())
