import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from bench import CONFIGS, make_truth_and_theta0
from ppls_amd import Context
for cfgname in sys.argv[1:]:
    cfg = CONFIGS[cfgname]; n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0); truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    ctx.em_begin(th0)
    for rep in range(3):
        for nt in (0, 1):
            for ab in (0, 1):
                ctx.set_option("nt", nt); ctx.set_option("ablate", ab)
                ctx.em_iterate(2); ctx.synchronize()
                ctx.set_option("timing", 1); ctx.sweep_timing(reset=True)
                ctx.em_iterate(10); ctx.synchronize()
                ms, k = ctx.sweep_timing(reset=True); ctx.set_option("timing", 0)
                print(f"{cfgname} nt={nt} ablate={ab}: sweep {ms/k:.4f} ms  {8*n*(p+q)/(ms/k*1e-3)/1e12:.3f} TB/s", flush=True)
    ctx.set_option("ablate", 0); ctx.close()
