"""bench.py's N>1 control plane (barrier, max-over-ranks timing, summed verification counts, weak-scaling
value, rank-0 report) on 2 and 8 gloo ranks with a stub prover (CPU), and the host-core pinning of 8
ranks on a faked 8-GPU node.  The same path driving the real
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
    import torch
    torch.set_num_threads(1)
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


def test_eight_rank_gloo_report(tmp_path):
    """The driver's 8-GPU run, rehearsed on the CPU: 8 ranks, each its stub proofs, rank 0's line
    counts all 64 proofs at the slowest rank's time, and every rank's host facts reach it."""
    pytest.importorskip("torch")
    import torch.multiprocessing as mp
    out = str(tmp_path / "rep8.json")
    mp.start_processes(_worker, args=(8, _free_port(), out), nprocs=8, join=True, start_method="spawn")
    rep = json.load(open(out))
    assert rep["n_gpus"] == 8 and rep["verified"] == 64 and rep["scaling"] == "weak"
    assert rep["ms_per_step"] >= 8 * 80 / 8 * 0.9           # rank 7: 8 proofs x 80 ms
    assert abs(rep["value"] - 8 * 8 / (rep["ms_per_step"] * 8 / 1e3)) < 1e-3 * rep["value"] + 1e-6
    ranks = rep["host"]["ranks"]
    assert [r["rank"] for r in ranks] == list(range(8))
    assert [r["host_cpu_ms_per_proof"]["main"] for r in ranks] == [0.5 + r for r in range(8)]
    allowed = len(os.sched_getaffinity(0))
    if allowed >= 8:   # this container: 8 cores, one each
        assert all(r["pin"]["pinned"] and r["pin"]["cpus"] == allowed // 8 for r in ranks)


# A node of the driver's kind: 8 GPUs, 2 per NUMA node, 64 host cores per NUMA node
_NODE = [list(range(64 * (g // 2), 64 * (g // 2) + 64)) for g in range(8)]


def _shares(monkeypatch, env=None):
    sys.path.insert(0, ROOT)
    import bench
    out = []
    for r in range(8):
        for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
            monkeypatch.delenv(var, raising=False)
        for k, v in (env(r) if env else {}).items():
            monkeypatch.setenv(k, v)
        info = bench.pin_host_cores(r, 8, topo=_NODE, allowed=range(256), apply=False)
        assert info["pinned"] and info["source"].startswith("GPU-local"), info
        out.append(info["share"])
    return out


def _check_node_shares(shares):
    for r, sh in enumerate(shares):
        assert len(sh) == 32 and set(sh) <= set(_NODE[r]), (r, sh[:4])   # half of its GPU's NUMA node
    flat = [c for sh in shares for c in sh]
    assert len(flat) == len(set(flat)) == 256                                 # disjoint, all cores used


def test_pin_eight_ranks_gpu_local(monkeypatch):
    """8 ranks on a faked 8-GPU node (2 GPUs per NUMA node), every GPU visible to every rank
    (rank r drives device r): disjoint shares of 32 cores, each on its own GPU's NUMA node."""
    _check_node_shares(_shares(monkeypatch))


def test_pin_eight_ranks_one_visible_gpu_each(monkeypatch):
    """The same node with a launcher that shows each rank only its own GPU (ROCR_VISIBLE_DEVICES=r):
    the peers are counted on the node's topology, so each rank still gets half of its NUMA node
    (it used to count all 8 ranks as peers on one GPU's cores)."""
    _check_node_shares(_shares(monkeypatch, lambda r: {"ROCR_VISIBLE_DEVICES": str(r)}))
    _check_node_shares(_shares(monkeypatch, lambda r: {"HIP_VISIBLE_DEVICES": str(r)}))


def test_pin_unknown_topology_even_split(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    shares = [bench.pin_host_cores(r, 8, topo=[], allowed=range(256), apply=False)["share"] for r in range(8)]
    assert [len(s) for s in shares] == [32] * 8 and sorted(c for s in shares for c in s) == list(range(256))


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
