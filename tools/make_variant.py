"""Experiment build: copy the product tree to abtest/<name> and build it with extra compiler flags
(e.g. -DPPLS_XP_TPB=2), for tools/variant_ab.sh.  Not part of the product.

    python tools/make_variant.py <name> "<flags>"
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    name, flags = sys.argv[1], sys.argv[2]
    out = os.path.join(ROOT, "abtest", name)
    if os.path.exists(out):
        shutil.rmtree(out)
    for d in ("ppls_amd", "tools", "oracle", "include", "tests"):
        shutil.copytree(os.path.join(ROOT, d), os.path.join(out, d),
                        ignore=shutil.ignore_patterns("_build", "__pycache__", "*.so", "*.o"))
    for f in ("bench.py", "__graft_entry__.py"):
        shutil.copy(os.path.join(ROOT, f), out)
    env = dict(os.environ, PPLS_EXTRA_CFLAGS=flags)
    subprocess.run([sys.executable, "-m", "ppls_amd.build", "--force"], cwd=out, check=True, env=env)
    print("built", os.path.join(out, "ppls_amd", "libppls_amd.so"), "with", flags)


if __name__ == "__main__":
    main()
