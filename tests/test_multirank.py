"""bench.py's N>1 control plane (barrier, max-over-ranks timing, summed verification counts, weak-scaling
value, rank-0 report) on 2 gloo ranks with a stub prover (CPU).  The same path driving the real
prover on the GPU is tests/test_gpu_multirank.py; there is no data-path collective (independent
proofs per rank)."""
import json
import os
import socket
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _StubKey:
    """Stands in for native.ProvingKey: 'proves' by sleeping a rank-dependent time."""

    def __init__(self, rank):
        self.rank = rank

    def prove_batch(self, ws, rs=None):
        time.sleep(0.01 * (1 + self.rank) * len(ws))
        return [bytes(256)] * len(ws)


class _StubCtx:
    def synchronize(self):
        pass

    def profile_reset(self):
        pass

    def set_profiling(self, on):
        pass

    def profile(self, name):
        return (0.0, 0, 0.0, 0.0)


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    pin = bench.pin_host_cores(rank, world)   # the N>1 rule: each rank its share of the host cores
    dist.init_process_group("gloo", rank=rank, world_size=world)
    key = _StubKey(rank)
    elapsed, proofs, _ = bench.timed_run(key, [0], list(range(8)), None, _StubCtx(), dist)
    verified = bench._sum_over_ranks(len(proofs), dist)
    host = bench.host_report(rank, rank, dist, pin, {"main": 0.5 + rank})
    prof = {k: (0.0, 0, 0.0, 0.0) for k in bench.PROFILED}

    class A:
        steps, warmup, slots = 8, 1, 1
    if rank == 0:
        rep = bench.report(A, world, elapsed, 8 * world, verified, prof, 1, None, {"workload": "stub"}, {"host": host})
        with open(out_path, "w") as f:
            json.dump(rep, f)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_report(tmp_path):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    out = str(tmp_path / "rep.json")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    rep = json.load(open(out))
    # the slowest rank (rank 1: 8 * 20 ms) bounds the job; value counts both ranks' proofs
    assert rep["n_gpus"] == 2 and rep["steps"] == 8 and rep["scaling"] == "weak"
    assert rep["ms_per_step"] >= 8 * 20 / 8 * 0.9
    assert abs(rep["value"] - 2 * 8 / (rep["ms_per_step"] * 8 / 1e3)) < 1e-3 * rep["value"] + 1e-6
    assert rep["metric"].startswith("Groth16 proofs/sec") and rep["verified"] == 16
    # per-rank host facts (bench.host_report): the node's CPUs, each rank's pinning and host CPU
    host = rep["host"]
    assert host["node_cpus"] == os.cpu_count() and [r["rank"] for r in host["ranks"]] == [0, 1]
    allowed = len(os.sched_getaffinity(0))
    for r in host["ranks"]:
        assert r["host_cpu_ms_per_proof"] == {"main": 0.5 + r["rank"]}
        assert r["pin"]["allowed_cpus"] == allowed
        if allowed >= 2:   # two ranks: disjoint halves of the allowed cores
            assert r["pin"]["pinned"] and r["pin"]["cpus"] == allowed // 2 + (allowed % 2) * r["rank"]


def test_pin_single_rank_untouched():
    """One rank on the node keeps the process's affinity (the N=1 headline is not re-pinned)."""
    sys.path.insert(0, ROOT)
    import bench
    before = os.sched_getaffinity(0)
    info = bench.pin_host_cores(0, 1)
    assert not info["pinned"] and os.sched_getaffinity(0) == before
    assert bench._cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]


def test_bench_refuses_world_size_mismatch():
    """WORLD_SIZE from a launcher must equal --gpus (checked before anything touches HIP)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in p.stderr
