"""A/B timing of source variants of the product library in one GPU process each.

    python tools/exp/variants.py build <spec.json>     # here (CPU): tools/exp/_var/<name>/libuq_dme.so
    python tools/exp/variants.py run <name> -- <tool.py> [tool args]   # on the GPU box

spec.json: {"<name>": [[file, old, new], ...], ...} -- exact substitutions in a scratch copy of
csrc/ (each `old` must occur); "base" with no substitutions is the tree as it is; a value
{"git": "<rev>"} takes csrc/ as of that revision.  `run` points
the package's loader at the variant's library, then runs the tool's main() in this process.
Timing probes only: variants are not tested and never shipped."""
import json
import os
import runpy
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd")
OUT = os.path.join(ROOT, "tools", "exp", "_var")
sys.path.insert(0, ROOT)


def build(spec_path):
    from importlib import util
    spec = util.spec_from_file_location("build_ext", os.path.join(PKG, "build_ext.py"))
    be = util.module_from_spec(spec)
    spec.loader.exec_module(be)
    variants = json.load(open(spec_path))
    shutil.rmtree(OUT, ignore_errors=True)
    os.makedirs(OUT)
    objs = []                                      # the tree's host code (no GPU work) in every variant
    for f in be.HOST_SRCS:
        objs.append(os.path.join(OUT, os.path.basename(f)[:-4] + ".o"))
        subprocess.run(["g++", *be.HOST_FLAGS, "-c", "-o", objs[-1], f], check=True)
    procs = []
    for name, subs in variants.items():
        top = os.path.join(OUT, name)
        src = os.path.join(top, "pkg", "csrc")
        os.makedirs(src)
        os.symlink(os.path.join(ROOT, "include"), os.path.join(top, "include"))
        if isinstance(subs, dict):                  # {"git": rev}: csrc/ as of that revision
            rel = os.path.relpath(os.path.join(PKG, "csrc"), ROOT)
            names = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", subs["git"], rel + "/"],
                                   check=True, capture_output=True, text=True).stdout.split()
            for path in names:
                blob = subprocess.run(["git", "-C", ROOT, "show", f"{subs['git']}:{path}"], check=True,
                                      capture_output=True).stdout
                open(os.path.join(src, os.path.basename(path)), "wb").write(blob)
            subs = []
        else:
            for f in os.listdir(os.path.join(PKG, "csrc")):
                shutil.copy(os.path.join(PKG, "csrc", f), src)
        for f in os.listdir(src):                  # host sources are linked from objs
            if f.endswith(".cpp"):
                os.remove(os.path.join(src, f))
        for fname, old, new in subs:
            p = os.path.join(src, fname)
            t = open(p).read()
            assert old in t, (name, fname, old[:60])
            open(p, "w").write(t.replace(old, new))
        so = os.path.join(top, "libuq_dme.so")
        procs.append((name, subprocess.Popen([be.hipcc(), *be.HIPCC_FLAGS, "-o", so, os.path.join(src, "uq_dme.hip"),
                                              "-x", "none", *objs, "-lpthread"])))
    bad = [n for n, p in procs if p.wait() != 0]
    if bad:
        raise SystemExit(f"variant builds failed: {bad}")
    print("built", [n for n, _ in procs])


def run(name, tool, args):
    import uqdme  # noqa: F401  (registers uqdme_amd; the library loads on first use)
    from uqdme_amd import build_ext
    build_ext.SO = os.path.join(OUT, name, "libuq_dme.so")
    sys.argv = [tool, *args]
    runpy.run_path(tool, run_name="__main__")


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2])
    else:
        i = sys.argv.index("--")
        run(sys.argv[2], sys.argv[i + 1], sys.argv[i + 2:])
