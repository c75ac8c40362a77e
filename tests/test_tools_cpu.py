"""Host-side measurement tools (CPU, no device): the PMC request-size attribution
(tools/pmc_attrib.py) on synthetic rocprofv3 databases, and the wave tracer's timeline helpers
(tools/wtrace.py) on synthetic wave records."""
import json
import os
import sqlite3
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

G1 = "void zkfl::k_msm_accumulate<zkfl::FqOps29, 3, zkfl::FqOps>(unsigned short const*)"
G2 = "void zkfl::k_msm_accumulate<zkfl::Fq2Pair29, 2, zkfl::Fq2Ops>(unsigned short const*)"


def _db(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    c = sqlite3.connect(path)
    c.execute("create table counters_collection (kernel_name text, counter_name text, value real)")
    c.executemany("insert into counters_collection values (?, ?, ?)", rows)
    c.commit()
    c.close()


def test_pmc_attrib_exact_bytes(tmp_path):
    d = tmp_path / "pmc"
    # two launches of the G1 kernel, one of G2: averages per launch, bytes by request size
    _db(str(d / "rd" / "run_results.db"), [
        (G1, "TCC_EA0_RDREQ_sum", 100), (G1, "TCC_EA0_RDREQ_sum", 300),
        (G1, "TCC_EA0_RDREQ_32B_sum", 10), (G1, "TCC_EA0_RDREQ_32B_sum", 10),
        (G1, "TCC_EA0_RDREQ_64B_sum", 20), (G1, "TCC_EA0_RDREQ_64B_sum", 40),
        (G1, "TCC_EA0_RDREQ_128B_sum", 70), (G1, "TCC_EA0_RDREQ_128B_sum", 250),
        (G2, "TCC_EA0_RDREQ_sum", 5), (G2, "TCC_EA0_RDREQ_128B_sum", 5)])
    _db(str(d / "wr" / "run_results.db"), [
        (G1, "TCC_EA0_WRREQ_sum", 40), (G1, "TCC_EA0_WRREQ_64B_sum", 30), (G1, "TCC_EA0_RDREQ_DRAM_sum", 200)])
    _db(str(d / "hit" / "run_results.db"), [(G1, "TCC_HIT_sum", 3), (G1, "TCC_MISS_sum", 1)])
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_attrib.py"), str(d)],
                       capture_output=True, text=True, check=True)
    res = json.loads(p.stdout)
    g1 = res["g1"]
    assert g1["launches"] == 2
    assert g1["read_bytes"] == 32 * 10 + 64 * 30 + 128 * 160          # per-launch averages
    assert g1["write_bytes"] == 32 * (40 - 30) + 64 * 30
    assert g1["l2_hit_rate"] == 0.75
    assert res["g2"]["read_bytes"] == 128 * 5
    tr = json.load(open(d / "pmc_traffic.json"))
    assert tr["unit"] == "bytes per launch"
    assert tr["kernels"][G1]["traffic"] == g1["read_bytes"] + g1["write_bytes"]


def test_wtrace_proof_split_and_gantt():
    import wtrace
    dt = np.dtype([("kind", "<u4"), ("hwid", "<u4"), ("t0", "<u8"), ("t1", "<u8"), ("c0", "<u8"), ("c1", "<u8")])
    r = np.zeros(7, dt)
    # proof 1: two acc waves overlapping, a stitch, an acc after a gap; proof 2 after a 1 ms idle gap
    r["kind"] = [1, 1, 2, 1, 1, 3, 1]
    r["t0"] = [0, 50, 200, 400, 100000, 100300, 100500]
    r["t1"] = [150, 120, 300, 450, 100200, 100400, 100600]
    r["c1"] = (r["t1"] - r["t0"]) * 24  # 2.4 GHz against the 100-MHz wall clock
    ps = wtrace.proofs_of(r, gap_us=150.0)
    assert [len(p) for p in ps] == [4, 3]
    g = wtrace.gantt(ps[0])
    assert [(x["kind"], x["start_us"], x["end_us"], x["waves"]) for x in g] == [
        ("acc", 0.0, 1.5, 2), ("stitch", 2.0, 3.0, 1), ("acc", 4.0, 4.5, 1)]
    assert all(abs(x["clock_GHz"] - 2.4) < 1e-9 for x in g)
    assert wtrace.kind_name(1 | 32) == "acc_g2"
