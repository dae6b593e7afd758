"""Experiment build for the C5 A/B of fp32 MFMA in the panel dots pass (round-4 verdict item 4).

Writes abtest/f32dots/: a copy of the product sources whose ppls_panel_mfmadots_kernel multiplies on
v_mfma_f32_16x16x4_f32 instead of v_mfma_f64_16x16x4_f64 -- A = the stored fp32 X values, B = W
rounded to fp32, fp32 accumulation over one 128-B column tile (32 fp32 columns = 8 MFMA steps), then
added into the fp64 accumulators -- and builds its libppls_amd.so.  The f32 MFMA's result lanes hold
rows 4 (l >> 4) + reg (the f64 one: (l >> 4) + 4 reg), so the A operand of lane l is read from tile
row rho(l & 15), rho(i) = (i >> 2) + 4 (i & 3), which puts every result where the f64 layout has it.
Not part of the product.  Then on the GPU:

    tools/variant_ab.sh f32dots c5 c5s          (kernel times, ms per iteration)
    python tools/f32dots_check.py base|f32dots  (a full C5 fit; W, loglik to gpurun_out/)
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "abtest", "f32dots")

OLD_A = "const float4 v = *(const float4*)(wl + (16 * bk + i16) * RS + kq * KQ * ES + h * 16);"
NEW_A = ("const float4 v = *(const float4*)(wl + (16 * bk + ((i16 >> 2) + 4 * (i16 & 3))) * RS + kq * KQ * ES"
         " + h * 16);")
OLD_M = """#pragma unroll
          for (int s2 = 0; s2 < KQ; ++s2)
            acc[bk] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)a[s2], bw[s2], acc[bk], 0, 0, 0);"""
NEW_M = """f4 af = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s2 = 0; s2 < KQ; ++s2)
            af = __builtin_amdgcn_mfma_f32_16x16x4f32((float)a[s2], (float)bw[s2], af, 0, 0, 0);
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[bk][u] += (double)af[u];"""


def main():
    if os.path.exists(OUT):
        shutil.rmtree(OUT)
    for d in ("ppls_amd", "tools", "oracle", "include"):
        shutil.copytree(os.path.join(ROOT, d), os.path.join(OUT, d),
                        ignore=shutil.ignore_patterns("_build", "__pycache__", "*.so", "*.o"))
    for f in ("bench.py", "__graft_entry__.py"):
        shutil.copy(os.path.join(ROOT, f), OUT)
    src = os.path.join(OUT, "ppls_amd", "csrc", "ppls_kernels.hip")
    s = open(src).read()
    assert s.count(OLD_A) == 1 and s.count(OLD_M) == 1, "dots kernel changed: update the patch"
    s = s.replace(OLD_A, NEW_A).replace(OLD_M, NEW_M)
    open(src, "w").write(s)
    subprocess.run([sys.executable, "-m", "ppls_amd.build", "--force"], cwd=OUT, check=True)
    print("built", os.path.join(OUT, "ppls_amd", "libppls_amd.so"))


if __name__ == "__main__":
    main()
