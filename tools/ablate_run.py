"""Run 60 EM iterations of a bench config on whatever libppls_amd.so this tree holds, tolerating
the numerical failures of ablated (deliberately wrong) builds; for kernel traces of tools/*_ablate.py
variants:  rocprofv3 --kernel-trace --stats -- python3 abtest/<v>/tools/ablate_run.py c5"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402

cfg = CONFIGS[sys.argv[1]]
ctx = Context(0)
if cfg.get("storage") == "f32":
    ctx.set_option("dtype", 1)
truth, th0 = make_truth_and_theta0(cfg["p"], cfg["q"], cfg["r"])
ctx.generate_synthetic(int(os.environ.get("AB_N", cfg["n"])), cfg["p"], cfg["q"], truth, seed=20261015)
done = 0
t0 = time.perf_counter()
for _ in range(60):
    try:
        ctx.em_begin(th0)
        ctx.em_iterate(1)
        ctx.synchronize()
        done += 1
    except Exception as e:   # an ablated build's garbage: the kernels still ran
        err = str(e)
print(f"{ROOT}: {done} of 60 single iterations without error, {time.perf_counter() - t0:.2f} s", flush=True)
ctx.close()
