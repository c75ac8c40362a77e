"""The multi-GPU path of bench.py driving the real prover — MI355X (-m gpu).

Two ranks launched exactly as the driver launches N>1 (`python -m torch.distributed.run
--nproc-per-node 2 --master-addr 127.0.0.1 … bench.py --gpus 2`), both on device 0 (a lease has one
GPU; bench.py maps rank -> device as local_rank mod device count).  Each rank proves its own clients'
witnesses through libzkfl (the metric circuit at a reduced step count, the input.json leg and the
config-5 round shard k -> rank k mod 2), GPU-verifies every proof, and rank 0 reports the summed
counts.  torch.distributed (gloo) carries only the barrier, the max-over-ranks time and the counts;
there is no collective on the data path.
"""
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


def test_two_ranks_real_prover_one_device(tmp_path):
    env = dict(os.environ)
    env["ZKFL_HW_QUEUES"] = "12"        # two processes share the device's hardware queues
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--slots", "4", "--e2e-steps", "1",
           "--c5-rounds", "2", "--c5-weak-rounds", "1", "--extra-circuit", "none", "--merkle-log2n", "0",
           "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    log = p.stdout + "\n" + p.stderr
    (tmp_path / "bench2.log").write_text(log)
    assert p.returncode == 0, log[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, log[-4000:]          # one JSON line, from rank 0
    rep = json.loads(lines[0])
    assert rep["ranks"] == 2 and rep["n_gpus"] == 1           # two ranks, one distinct device
    assert rep["steps"] == 2 and rep["scaling"] == "weak"
    assert rep["proofs_timed"] == 2 * 2 * 4 and rep["verified"] == rep["proofs_timed"]
    assert rep["value"] > 0 and rep["config"]["parallelism"] == "replicas2"
    assert rep["end_to_end"]["proofs"] == 2 * 4
    assert rep["end_to_end"]["verified"] == 2 * 4
    c5 = rep["c5"]
    assert c5["proofs"] == 32 and c5["verified"] == 32 and c5["scaling"] == "strong"
    w = rep["c5_weak"]
    assert w["proofs"] == 2 * 16 and w["verified"] == 32 and w["scaling"] == "weak"
    # both ranks really ran the prover on device 0 (their own log lines)
    for r in (0, 1):
        assert f"[bench r{r}] 8 proofs in" in log and f"device 0 of" in log


def test_two_ranks_without_launcher(tmp_path):
    """`bench.py --gpus 2` with no torchrun: bench.py starts the two ranks itself (before any HIP
    call in the parent) and rank 0 reports both."""
    env = dict(os.environ)
    env["ZKFL_HW_QUEUES"] = "12"
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--slots", "2", "--e2e-steps", "0", "--c5-rounds", "0", "--merkle-log2n", "0", "--extra-circuit", "none",
           "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    log = p.stdout + "\n" + p.stderr
    (tmp_path / "bench2_nolauncher.log").write_text(log)
    assert p.returncode == 0, log[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, log[-4000:]
    rep = json.loads(lines[0])
    assert rep["ranks"] == 2 and rep["proofs_timed"] == 2 * 1 * 2 and rep["verified"] == 4
    for r in (0, 1):
        assert f"[bench r{r}] 2 proofs in" in log
