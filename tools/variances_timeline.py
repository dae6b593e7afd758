"""Timeline of each variances.PPLS_simult call from a rocprofv3 kernel trace (+ memory-copy trace):
span from the call's Cxt pass (`ppls_xtmu_kernel`) to its last seLoad kernel, split into the MFMA
Gram, the Cxt pass, rocSOLVER/rocBLAS kernels, our small kernels, copies and idle GPU time.

    python tools/variances_timeline.py <rocprofv3 output dir> [--prefix run]
"""
import csv
import os
import sys


def load(path):
    return list(csv.DictReader(open(path))) if os.path.exists(path) else []


def main():
    d = sys.argv[1]
    pre = sys.argv[sys.argv.index("--prefix") + 1] if "--prefix" in sys.argv else "run"
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
           r["Kernel_Name"].replace("(anonymous namespace)::", "")) for r in load(f"{d}/{pre}_kernel_trace.csv")]
    cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", ""))
          for r in load(f"{d}/{pre}_memory_copy_trace.csv")]
    ks.sort()
    starts = [i for i, k in enumerate(ks) if k[2].startswith("void ppls_xtmu_kernel")]
    for ci, i0 in enumerate(starts):
        i1 = starts[ci + 1] if ci + 1 < len(starts) else len(ks)
        ends = [i for i in range(i0, i1) if "symdiag" in ks[i][2] or "negdiag" in ks[i][2]]
        if not ends:
            continue
        t0, t1 = ks[i0][0], ks[ends[-1]][1]
        cat = {"gram": 0, "xtmu": 0, "solver": 0, "ppls": 0, "copy": 0}
        n_solver = 0
        ev = [k for k in ks[i0:ends[-1] + 1]] + [c for c in cs if t0 <= c[0] <= t1]
        for s, e, nm in ev:
            if nm.startswith("copy"):
                cat["copy"] += e - s
            elif "gram_mfma" in nm:
                cat["gram"] += e - s
            elif "xtmu" in nm:
                cat["xtmu"] += e - s
            elif "ppls" in nm:
                cat["ppls"] += e - s
            else:
                cat["solver"] += e - s
                n_solver += 1
        # solver region: first to last rocSOLVER/rocBLAS kernel of the call
        sol = [k for k in ks[i0:ends[-1] + 1] if "ppls" not in k[2]]
        sspan = (sol[-1][1] - sol[0][0]) if sol else 0
        busy = sum(cat.values())
        print(f"call {ci}: span {(t1 - t0) / 1e6:7.2f} ms | gram {cat['gram'] / 1e6:6.2f} xtmu {cat['xtmu'] / 1e6:5.2f} "
              f"solver {cat['solver'] / 1e6:6.2f} ({n_solver} kernels over {sspan / 1e6:6.2f} ms) "
              f"ppls {cat['ppls'] / 1e6:5.2f} copies {cat['copy'] / 1e6:5.2f} | idle {(t1 - t0 - busy) / 1e6:6.2f} ms")


if __name__ == "__main__":
    main()
