"""Build the HIP C-ABI library in-tree (gfx950 only).

    python unbiased-quantization-distributed-mean-estimation_amd/build_ext.py

Output: unbiased-quantization-distributed-mean-estimation_amd/_build/libuq_dme.so
(git-ignored; it travels to the GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(PKG_DIR, "csrc", "uq_dme.hip")
OUT_DIR = os.path.join(PKG_DIR, "_build")
SO = os.path.join(OUT_DIR, "libuq_dme.so")

# -ffp-contract=off: the reference evaluates m*p, floor, subtract, (L1*sign)*(k)/m as
#   separate f32 ops; a fused multiply-add would change bits.
# -fhip-fp32-correctly-rounded-divide-sqrt: x/den and t/m must be IEEE divisions.
# -fno-gpu-flush-denormals-to-zero: torch CPU keeps f32 denormals.
HIPCC_FLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
    "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fno-gpu-flush-denormals-to-zero", "-Wall",
]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def needs_build() -> bool:
    if not os.path.exists(SO):
        return True
    deps = [os.path.join(PKG_DIR, "csrc", f) for f in os.listdir(os.path.join(PKG_DIR, "csrc"))]
    deps.append(os.path.join(PKG_DIR, "..", "include", "uq_dme.h"))
    src_m = max(os.path.getmtime(f) for f in deps)
    return os.path.getmtime(SO) < src_m


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return SO
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = SO + ".tmp"
    cmd = [hipcc(), *HIPCC_FLAGS, "-o", tmp, SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, SO)
    return SO


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
