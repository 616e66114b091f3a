"""bench.py's own multi-rank branch (VERDICT r2 "Missing" 3 / "Next round" 7), launched exactly as
the driver launches the N-GPU bench (python -m torch.distributed.run --nnodes=1 --nproc-per-node N
--master-addr 127.0.0.1 ... bench.py --gpus N), with world 2 on the one GPU of the box: the
gloo backend (--dist-backend gloo; RCCL cannot put two ranks on one GPU) carries the same
barrier, max-over-ranks timing and gradient all-reduce hook as the RCCL run. Checked: rank 0
prints ONE JSON line with n_gpus 2, the whole job's env count (2 x envs per GPU), a finite
value equal to envs x ranks x steps / the timed seconds, and the extra whole-job reading
(--total-reading: the same total env count split over the ranks)."""
import json
import math
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_world2_gloo_prints_one_line(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    E, steps = 512, 4
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--grid", "64", "--people", "569", "--robots", "8", "--envs", str(E), "--steps", str(steps),
           "--warmup", "2", "--age-steps", "40", "--stagger", "40", "--other-steps", "0", "--start-steps", "0",
           "--env-steps", "3", "--no-cpu", "--total-reading", str(E)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == steps and rec["scaling"] == "weak"
    cfg = rec["config"]
    assert cfg["envs_per_gpu"] == E and cfg["envs_total"] == 2 * E and cfg["dist_backend"] == "gloo"
    assert math.isfinite(rec["value"]) and rec["value"] > 0
    assert abs(rec["value"] - 2 * E * steps / (rec["ms_per_step"] * steps * 1e-3)) <= 1e-6 * rec["value"]
    tot = rec["total_envs_reading"]
    assert tot is not None and tot["envs_total"] == E and tot["envs_per_gpu"] == E // 2
    assert math.isfinite(tot["steps_per_s"]) and tot["steps_per_s"] > 0
    assert rec["last_loss"] is not None and math.isfinite(rec["last_loss"])
