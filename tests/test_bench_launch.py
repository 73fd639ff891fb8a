"""bench.py's multi-rank launch: `--gpus N` without an external launcher must
start N ranks itself (torch.distributed.run as a child process) and report
n_gpus = N.  The CPU test runs the launch/timing protocol over gloo
(`--launch-check`); the GPU test runs the whole bench with 2 ranks on the one
GPU of the box (gloo, ED_BENCH_ONE_DEVICE) and relies on bench.py's own
fixture assertions (c2 E0 per rank seed, configs[3] eigenvalues, configs[4]
G(iw)).  Reference: the sector loop the farm replaces, ED_DIAG.f90:71-249."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, env=env, timeout=timeout)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    return _json_line(p.stdout)


@pytest.mark.parametrize("n", [1, 2])
def test_launch_spawns_n_ranks(n):
    out = _run(["--gpus", str(n), "--launch-check"])
    assert out["n_gpus"] == n
    assert out["ranks"] == list(range(n))
    assert sorted(out["local_ranks"]) == list(range(n))


def test_launch_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stdout + p.stderr)


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu():
    out = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--niter", "256", "--no-roofline", "--no-cpu"],
               env_extra={"ED_BENCH_BACKEND": "gloo", "ED_BENCH_ONE_DEVICE": "1"}, timeout=600)
    assert out["n_gpus"] == 2
    assert out["validation"]["rel_dev"] < 1e-10
    assert out["farm_c4"]["n_gpus"] == 2 and out["farm_c4"]["parity"]["E0_rel_dev"] < 1e-10
    assert out["nonsu2_c5"]["parity"]["G_iw_max_rel_dev"] < 1e-10
    assert out["split_n28"]["backend"] == "gloo"
