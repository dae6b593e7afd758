"""The driver's multi-GPU bench command path, rehearsed on one GPU.

`python bench.py --gpus N` without a launcher spawns N rank processes (bench.spawn_ranks); the
driver's 8-GPU run takes exactly that path.  Two ranks oversubscribe GPU 0 with the host reducer
(gloo) in place of RCCL (RCCL refuses two ranks on one device), at one GPU's C4 share: the line must
say n_gpus 2 and bitwise-identical ranks, and its log-likelihood must equal the one-rank run of the
same config (EM_W_multi.R:689-712, :732-733 are row sums: sharding only reorders them).  A run whose
ranks disagree must print no value and exit 3.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

ARGS = ["--config", "c4s", "--steps", "10", "--xprod-steps", "50", "--no-cpu"]


def _bench(extra, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE")}
    env.update(env_extra or {})
    pr = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *extra, *ARGS], cwd=ROOT, env=env,
                        capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in pr.stdout.splitlines() if ln.startswith("{")]
    return pr, (json.loads(lines[-1]) if lines else None)


def test_bench_two_ranks_spawn_path_equals_one_rank():
    pr2, two = _bench(["--gpus", "2", "--comm", "host", "--oversubscribe"])
    assert pr2.returncode == 0, pr2.stderr[-3000:]
    pr1, one = _bench(["--gpus", "1"])
    assert pr1.returncode == 0, pr1.stderr[-3000:]
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["ranks_bitwise_identical"] is True
    assert two["comm"]["backend"] == "host reducer over gloo"
    assert "dp2" in two["config"]["parallelism"]
    assert abs(two["loglik_last"] - one["loglik_last"]) <= 1e-12 * abs(one["loglik_last"])
    # the cross-product form: S summed over the two shards by one all-reduce, then the same iterates
    assert two["xprod"]["setup_allreduce_ms"] > 0 and one["xprod"]["setup_allreduce_ms"] == 0
    assert two["xprod"]["loglik_rel_diff_vs_streaming"] < 1e-12
    # the whole PPLS_simult call on the sharded data: the same fit as on one rank
    for mode in ("stream", "xprod", "auto"):
        a, b = two["call"][mode], one["call"][mode]
        assert a["em_steps"] == b["em_steps"] and a["init_steps"] == b["init_steps"]
        assert abs(a["loglik_last"] - b["loglik_last"]) <= 1e-10 * abs(b["loglik_last"])
    assert two["call"]["xprod"]["read_S"] and not two["call"]["stream"]["read_S"]
    # per-rank spreads (a scaling run explains itself): every rank's sweep kernel time and rows, the
    # all-reduce of S; the statistics all-reduce is timed on the RCCL path only (None here)
    pr_ = two["per_rank"]
    assert len(pr_["sweep_kernel_ms"]["per_rank"]) == 2
    assert 0 < pr_["sweep_kernel_ms"]["min"] <= pr_["sweep_kernel_ms"]["max"]
    assert sum(pr_["rows"]["per_rank"]) == 125_000
    assert pr_["xprod_setup_allreduce_ms"]["min"] > 0
    assert pr_["allreduce_us"]["per_rank"] == [None, None]
    assert "per_rank" not in one
    # the Gram that forms S is reported on its useful flops, and beside the MFMA peak
    g = one["xprod"]["gram_roofline"]
    assert g["bound"] == "mfma" and 0 < g["frac"] < 1 and g["flops_per_launch"] < g["tile_flops_per_launch"]
    assert one["roofline"]["mfma_gemm"]["kernel"].startswith("ppls_gram_mfma")


def test_bench_diverging_ranks_fail_loudly():
    pr, line = _bench(["--gpus", "2", "--comm", "host", "--oversubscribe", "--no-call"],
                      {"PPLS_BENCH_TEST_DIVERGE": "1"})
    assert pr.returncode == 3, (pr.returncode, pr.stderr[-2000:])
    assert line is None   # no value printed
    assert "ranks hold different estimates" in pr.stderr
