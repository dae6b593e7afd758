"""HBM/MALL traffic of the cross-product tile kernel per launch from the rocprofv3 PMC passes
written by tools/profile.sh (bench.py's xprod section runs in the same profiled command).

    python tools/pmc_xprod_summary.py <tag> <config> [note] [--bytes B]

--bytes: S's bytes (8 P^2 with P the padded ldx + ldy, as ppls_xprod_info reports it; default from
p and q rounded to even, which is exact for the split sweep's 16-B rows but not for the panel
sweep's padded ones: C5 has P = 10,240 + 512).

Reads gpurun_out/prof_<tag>/pmc_{FETCH_SIZE,WRITE_SIZE}/run_counter_collection.csv and the kernel
trace's stats (average duration), writes profiles/pmc_xprod_<config>_dp1.json.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE (kB) exact.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pmc_summary import ROOT, per_launch, profiled_tree  # noqa: E402


def avg_us(stats, sub):
    for r in csv.DictReader(open(stats)):
        if sub in r["Name"]:
            return float(r["AverageNs"]) / 1e3, r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    return None, None


def main():
    args = list(sys.argv[1:])
    nbytes = None
    if "--bytes" in args:
        i = args.index("--bytes")
        nbytes = float(args[i + 1])
        del args[i:i + 2]
    tag, config = args[0], args[1]
    note = args[2] if len(args) > 2 else ""
    import bench
    cfg = bench.CONFIGS[config]
    ldx, ldy = (cfg["p"] + 1) // 2 * 2, (cfg["q"] + 1) // 2 * 2
    P = ldx + ldy
    alg = nbytes if nbytes else 8.0 * P * P
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    names, n, fetch = per_launch(os.path.join(base, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE",
                                 ("xprod_tile",))
    _, _, write = per_launch(os.path.join(base, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE",
                             ("xprod_tile",))
    us, kname = avg_us(os.path.join(base, "trace", "run_kernel_stats.csv"), "xprod_tile")
    gms, _ = avg_us(os.path.join(base, "trace", "run_kernel_stats.csv"), "gram_mfma")
    _, _, gfetch = per_launch(os.path.join(base, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE",
                              ("gram_mfma",))
    read = 2.0 * fetch * 1024
    out = dict(
        workload=f"{config}_dp1 (bench.py, tools/profile.sh {tag})",
        kernels={
            kname or "ppls_xprod_tile_kernel": dict(
                launches=n, FETCH_SIZE_kB_per_launch=fetch, WRITE_SIZE_kB_per_launch=write,
                read_bytes_per_launch=read, write_bytes_per_launch=write * 1024, algorithmic_bytes=alg,
                ratio=read / alg, avg_us=us,
                note="FETCH_SIZE x 2 x 1024 (gfx950 16-B/lane correction); Infinity-Cache hits are counted "
                     "too, so this does not separate MALL from HBM; writes: M (P x 2r) and the X'mu_T, Y'mu_U rows"),
            "ppls_gram_mfma_kernel (setup)": dict(
                read_bytes_per_launch=2.0 * gfetch * 1024, avg_ms=(gms / 1e3) if gms else None,
                note="each 128 x 128 output tile streams its two 128-column panels over all rows: L2/MALL "
                     "absorb most; compute-bound (pmc_compute_*.json)")},
        source=f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, gpurun_out/prof_{tag}; {note}",
        profiled_tree=profiled_tree())
    path = os.path.join(ROOT, "profiles", f"pmc_xprod_{config}_dp1.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, f"{read / alg:.4f} x algorithmic, {us} us")


if __name__ == "__main__":
    main()
