"""Source tree for timing-only ablation builds.

The product kernels (csrc/) carry no experiment switches.  The switches the round-1
ablations used (-DUQ_ABL_COPY, -DUQ_ABL_NOIO, -DUQ_CODES_FIRST, -DUQ_Q_AUX=..., -DUQ_TIE_PROF,
-DUQ_NORM_ABL_*, -DUQ_FOLD_PROF, ...) live in tools/exp/ablations.patch; patched_csrc() copies
csrc/ to a scratch directory, applies that patch and returns the directory, so an
experiment builds `<dir>/uq_dme.hip` with its -D flags.  Results of ablated builds are wrong
by construction; they are timing probes only."""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd", "csrc")
PATCH = os.path.join(ROOT, "tools", "exp", "ablations.patch")


def patched_csrc() -> str:
    top = tempfile.mkdtemp(prefix="uq_abl_")
    d = os.path.join(top, "pkg", "csrc")            # the sources include "../../include/uq_dme.h"
    os.makedirs(d)
    os.symlink(os.path.join(ROOT, "include"), os.path.join(top, "include"))
    for f in os.listdir(CSRC):
        shutil.copy(os.path.join(CSRC, f), d)
    subprocess.run(["patch", "-s", "-p1", "-d", d, "-i", PATCH], check=True)
    return d
