import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from bench import CONFIGS, make_truth_and_theta0
from ppls_amd import Context
cfg = CONFIGS["c5s"]
n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
ctx = Context(0)
ctx.set_option("dtype", 1)
truth, th0 = make_truth_and_theta0(p, q, r)
ctx.generate_synthetic(n, p, q, truth, seed=20261015)
ctx.set_option("team_rows", 1 << 20)
ctx.set_option("ftrace", 1)
ctx.em_begin(th0)
for it in range(30):
    ctx.em_iterate(1)
    tr = ctx.finalize_trace()
    print(it, {b: (v[10] if len(v) > 10 else None, v[7] if len(v) > 7 else None, v[8] if len(v) > 8 else None) for b, v in tr.items()}, flush=True)
