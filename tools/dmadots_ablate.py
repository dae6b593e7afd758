"""Ablation builds of the LDS-DMA dots kernel (round 5), to name what bounds it at full C5:
abtest/<name>/ = a copy of the product with ppls_panel_dmadots_kernel patched, built with its own
libppls_amd.so.  Results of the ablated builds are wrong by construction; only their times count.
Not part of the product.

    python tools/dmadots_ablate.py nomfma|nolds|nob      then on the GPU: tools/variant_ab.sh dma_<name> c5

  nomfma: each MFMA replaced by one fp64 VALU FMA into the accumulator (the loads, LDS reads and
          conversions stay)
  nolds:  the A operands taken from registers instead of the LDS image (the DMA still lands)
  nob:    no B loads (B = constants; the waits stay)
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MFMA = "            acc[bk] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)a[s], bw, acc[bk], 0, 0, 0);"
LDSR = "            av[bk][h] = *(const float4*)(buf + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));"
BLD = "        for (int s = 0; s < NBW; ++s) b[s] = ppls_load16_uncounted(wb, boff + 256u * s);"
PATCH = {
    "nomfma": (MFMA, "            acc[bk][s & 3] = fma((double)a[s], bw, acc[bk][s & 3]);"),
    "nolds": (LDSR, "            av[bk][h] = make_float4((float)row, (float)c, (float)tc, 1.f);"),
    "nob": (BLD, "        for (int s = 0; s < NBW; ++s) b[s] = ppls_d2v{(double)tc, (double)s};"),
}


def main():
    name = sys.argv[1]
    out = os.path.join(ROOT, "abtest", "dma_" + name)
    if os.path.exists(out):
        shutil.rmtree(out)
    for d in ("ppls_amd", "tools", "oracle", "include"):
        shutil.copytree(os.path.join(ROOT, d), os.path.join(out, d),
                        ignore=shutil.ignore_patterns("_build", "__pycache__", "*.so", "*.o"))
    for f in ("bench.py", "__graft_entry__.py"):
        shutil.copy(os.path.join(ROOT, f), out)
    src = os.path.join(out, "ppls_amd", "csrc", "ppls_kernels.hip")
    s = open(src).read()
    old, new = PATCH[name]
    i = s.index("void ppls_panel_dmadots_kernel(")
    j = s.index("\n}\n", i)
    body = s[i:j]
    assert body.count(old) == 1, "dots kernel changed: update the patch"
    s = s[:i] + body.replace(old, new) + s[j:]
    open(src, "w").write(s)
    subprocess.run([sys.executable, "-m", "ppls_amd.build", "--force"], cwd=out, check=True)
    print("built", os.path.join(out, "ppls_amd", "libppls_amd.so"))


if __name__ == "__main__":
    main()
