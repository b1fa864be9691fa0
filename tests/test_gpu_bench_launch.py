"""bench.py --gpus N starts its own ranks (no external launcher): the parent never
touches the GPU and spawns N fresh rank processes. Rehearsed here with the gloo backend
on the box's one GPU (TT_DIST_BACKEND=gloo; the 8-GPU node runs the same code over
RCCL). Checks the driver contract: exactly one JSON line, from rank 0, n_gpus = N,
whole-job value, finite losses."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("loss", ["hardneg_margin", "infonce"])
def test_bench_spawns_two_ranks_without_launcher(loss):
    env = dict(os.environ, TT_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "512", "--vocab", "20000", "--loss", loss, "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 1024
    assert rec["value"] > 0 and all(abs(x) < 1e3 for x in rec["loss_first_last"])
