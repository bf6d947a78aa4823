"""Build the HIP C-ABI library in-tree (gfx950 only).

    python unbiased-quantization-distributed-mean-estimation_amd/build_ext.py

Output: unbiased-quantization-distributed-mean-estimation_amd/_build/libuq_dme.so
(git-ignored; it travels to the GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(PKG_DIR, "csrc", "uq_dme.hip")
# host-only C++, g++, linked into the same library: the MT19937 jump polynomials, and numpy's
# legacy RandomState samplers for the NMSE harness (uq_legacy_rng.cpp: -ffp-contract=off, every
# product and sum rounded on its own as in numpy's baseline build; log/exp from the host libm)
HOST_SRCS = [os.path.join(PKG_DIR, "csrc", f) for f in ("uq_mt_poly.cpp", "uq_legacy_rng.cpp")]
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


HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-ffp-contract=off", "-fno-fast-math"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


HEADER = os.path.join(PKG_DIR, "..", "include", "uq_dme.h")
ID_FILE = SO + ".build_id"


def build_id() -> str:
    """SHA-256 over the library's sources (csrc/*, include/uq_dme.h) and the compile flags:
    the identity of the binary they produce.  The library reports the id it was built from
    (uq_build_id), so a stale binary is detected by content, not by file times."""
    h = hashlib.sha256()
    csrc = os.path.join(PKG_DIR, "csrc")
    for f in sorted(os.listdir(csrc)) + [None]:
        path = HEADER if f is None else os.path.join(csrc, f)
        h.update((os.path.basename(path) + "\0").encode())
        with open(path, "rb") as fh:
            h.update(fh.read())
    h.update("\0".join(HIPCC_FLAGS + HOST_FLAGS).encode())
    return h.hexdigest()


def needs_build() -> bool:
    if not os.path.exists(SO) or not os.path.exists(ID_FILE):
        return True
    with open(ID_FILE) as f:
        return f.read().strip() != build_id()


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return SO
    os.makedirs(OUT_DIR, exist_ok=True)
    bid = build_id()
    tmp = SO + ".tmp"
    objs = [os.path.join(OUT_DIR, os.path.basename(f)[:-4] + ".o") for f in HOST_SRCS]
    cmds = [[os.environ.get("CXX", "g++"), *HOST_FLAGS, "-c", "-o", o, f] for f, o in zip(HOST_SRCS, objs)]
    cmds.append([hipcc(), *HIPCC_FLAGS, f'-DUQ_BUILD_ID="{bid}"', "-o", tmp, SRC, "-x", "none", *objs, "-lpthread"])
    for cmd in cmds:
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    os.replace(tmp, SO)
    with open(ID_FILE, "w") as f:
        f.write(bid + "\n")
    return SO


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
