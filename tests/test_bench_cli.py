"""bench.py's command-line contract that needs no GPU: a multi-rank request that cannot be honoured
fails before any GPU work, with exit status 2."""
import os
import subprocess
import sys

from conftest import ROOT


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=300)


def test_oversubscribe_needs_host_comm():
    pr = _run("--gpus", "2", "--oversubscribe")
    assert pr.returncode == 2 and "--comm host" in pr.stderr and pr.stdout == ""


def test_more_ranks_than_gpus_is_refused():
    # no GPU here: 0 visible devices, so even one rank per GPU cannot be honoured
    pr = _run("--gpus", "2", "--comm", "host")
    assert pr.returncode == 2 and "GPU" in pr.stderr and pr.stdout == ""
