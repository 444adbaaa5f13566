"""bench.py's N > 1 path, executed: two ranks launched by torch.distributed.run exactly as the
driver launches the 8-GPU run, sharing the one leased GPU over the gloo backend (RCCL needs one
GPU per rank). The ranks capture the segmented data-parallel step (trainer._capture_dp) and
time its replays with the per-bucket all-reduces between the segment graphs; rank 0 prints the
one JSON line. Shapes are reduced (224x224, per-GPU batch 8) to keep the two replicas' autotuning
short; the parity of the same step is tests/test_dp_gpu.py."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
def test_bench_world2_gloo_line(cuda):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
           "--backend", "gloo", "--size", "224", "--batch", "8", "--no-extra-configs",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 16
    assert out["config"]["parallelism"] == "dp2" and out["config"]["backend"] == "gloo"
    assert out["config"]["graph"] is True
    assert out["config"]["ranks_seen"] == 2
    assert out["value"] > 0 and out["steps"] == 3
    assert out["loss"] == out["loss"]  # finite
    # the replicas' parameters agree bit for bit after the timed steps
    d = out["distributed"]
    assert d["replicas_identical"] is True, d
    assert d["param_checksums"]["min"] == d["param_checksums"]["max"]
    assert d["timeout_s"] > 0


@pytest.mark.timeout(300)
def test_bench_dead_rank_exits_nonzero(cuda):
    """A rank that dies before the first step: the surviving rank's first collective fails (the
    peer's socket closes, or the bounded timeout passes) and the job exits non-zero instead of
    hanging (bench.py --dist-timeout, dp.exit_on_failure)."""
    import time
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
           "--backend", "gloo", "--size", "64", "--batch", "2", "--no-extra-configs",
           "--no-cpu-baseline", "--dist-timeout", "60", "--debug-fail-rank", "1"]
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode != 0, r.stdout[-2000:]
    assert time.time() - t0 < 250
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(600)
def test_bench_self_spawns_ranks(cuda):
    """`python bench.py --gpus 2` with no launcher (no WORLD_SIZE), as the driver invokes the
    N = 1 bench: bench.py starts the two ranks itself and rank 0 prints the one line."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "2", "--backend", "gloo", "--size", "224", "--batch", "8",
           "--no-extra-configs", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["ranks_seen"] == 2
    assert out["config"]["backend"] == "gloo" and out["config"]["global_batch"] == 16
    assert out["value"] > 0
