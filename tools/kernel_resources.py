"""Per-kernel register / LDS / spill table from hipcc -Rpass-analysis=kernel-resource-usage.

    python tools/kernel_resources.py distributed_pytorch_amd/csrc/kernels/conv_x3.hip [--filter Li3E]
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
           "-I", os.path.join(ROOT, "distributed_pytorch_amd", "csrc"), "-c", a.src, "-o", "/tmp/_kr.o",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur, rows = None, []
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|SGPRs): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).split()[0]] = int(m.group(2))
    print(f"{'VGPR':>5} {'AGPR':>5} {'SGPR':>5} {'scr':>4} {'occ':>4} {'LDS':>7}  kernel")
    for r in rows:
        if a.filter in r["name"]:
            print(f"{r.get('VGPRs', 0):5d} {r.get('AGPRs', 0):5d} {r.get('SGPRs', 0):5d} {r.get('ScratchSize', 0):4d} "
                  f"{r.get('Occupancy', 0):4d} {r.get('LDS', 0):7d}  {r['name'][:110]}")


if __name__ == "__main__":
    sys.exit(main())
