"""Build libppls_amd.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build() and the tests.

    python -m ppls_amd.build [--force]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libppls_amd.so")
ARCH = os.environ.get("PPLS_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["ppls_kernels.hip", "ppls_variances.hip", "ppls_xprod.hip", "ppls_linalg.hip", "ppls_ozaki.hip",
           "ppls_capi.cpp"]
# Per-file flags.  ppls_kernels.hip: the panel dots kernel keeps its MFMA accumulators in VGPRs
# (the default AGPR form copied them VGPR <-> AGPR on every tile; its only MFMA user).
FILE_FLAGS = {"ppls_kernels.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function", "-Wno-inline-asm",
          "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
# experiment builds only (e.g. tools/variant_ab.sh: -DPPLS_REG_RMAX=6 into a copied tree)
CFLAGS += [f for f in os.environ.get("PPLS_EXTRA_CFLAGS", "").split() if f]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _local_includes(path, seen=None):
    """The in-tree headers a source includes, transitively (quoted #include lines)."""
    seen = set() if seen is None else seen
    with open(path) as f:
        for line in f:
            m = re.match(r'\s*#\s*include\s+"([^"]+)"', line)
            if m:
                h = os.path.normpath(os.path.join(os.path.dirname(path), m.group(1)))
                if os.path.exists(h) and h not in seen:
                    seen.add(h)
                    _local_includes(h, seen)
    return seen


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    objs, procs = [], []
    for src in SOURCES:   # the translation units compile in parallel
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, os.path.splitext(src)[0] + ".o")
        objs.append(o)
        newest_dep = max([_mtime(h) for h in _local_includes(s)] + [-1.0])
        if force or _mtime(o) < max(_mtime(s), newest_dep):
            cmd = [HIPCC, *CFLAGS, *FILE_FLAGS.get(src, []), "-x", "hip", "-c", s, "-o", o]
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append((subprocess.Popen(cmd), o))
    failed = False
    for pr, o in procs:
        if pr.wait() != 0:
            failed = True
            if os.path.exists(o):
                os.remove(o)
    if failed:
        raise subprocess.CalledProcessError(1, "hipcc")
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs,
               "-L/opt/rocm/lib", "-lrccl", "-lrocsolver", "-lrocblas", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
