#!/usr/bin/env python3
"""Summary of tools/pmc_attrib.sh: per launch of each MSM accumulation kernel, the L2's memory-side
read requests by size (32 / 64 / 128 B -> exact read bytes), how many went to DRAM (the rest were
served by the Infinity Cache), write requests (32 / 64 B) and the L2 hit rate; bytes per
accumulated entry with the metric circuit's entry counts (one-slot run: A, B1, C + H per proof).

    python3 tools/pmc_attrib.py gpurun_out/pmc_attrib
"""
import json
import os
import sqlite3
import sys


def counters(db):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, count(*), avg(value) from counters_collection "
                     "group by kernel_name, counter_name").fetchall()
    out = {}
    for k, n, cnt, v in rows:
        out.setdefault(k, {})[n] = (cnt, v)
    return out


def main():
    d = sys.argv[1]
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd"))
    merged = {}
    for p in ("rd", "wr", "hit"):
        dbs = [os.path.join(r, f) for r, _, fs in os.walk(os.path.join(d, p)) for f in fs if f.endswith(".db")]
        for db in dbs:
            for k, cs in counters(db).items():
                merged.setdefault(k, {}).update(cs)
    res = {}
    kernels = {}
    for k, cs in merged.items():
        g = lambda n: cs.get(n, (0, 0.0))[1]  # noqa: E731
        rdb = 32 * g("TCC_EA0_RDREQ_32B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + 128 * g("TCC_EA0_RDREQ_128B_sum")
        wr, wr64 = g("TCC_EA0_WRREQ_sum"), g("TCC_EA0_WRREQ_64B_sum")
        wrb = 32 * (wr - wr64) + 64 * wr64
        kernels[k] = {"launches": cs.get("TCC_EA0_RDREQ_sum", (0, 0))[0], "read": round(rdb), "write": round(wrb),
                      "traffic": round(rdb + wrb)}
        if "k_msm_accumulate" not in k:
            continue
        g = lambda n: cs.get(n, (0, 0.0))[1]  # noqa: E731
        n32, n64, n128 = g("TCC_EA0_RDREQ_32B_sum"), g("TCC_EA0_RDREQ_64B_sum"), g("TCC_EA0_RDREQ_128B_sum")
        rd = g("TCC_EA0_RDREQ_sum")
        wr, wr64 = g("TCC_EA0_WRREQ_sum"), g("TCC_EA0_WRREQ_64B_sum")
        hit, miss = g("TCC_HIT_sum"), g("TCC_MISS_sum")
        name = "g2" if "Fq2" in k else "g1"
        res[name] = {
            "launches": cs.get("TCC_EA0_RDREQ_sum", (0, 0))[0],
            "read_requests": round(rd), "read_32B": round(n32), "read_64B": round(n64), "read_128B": round(n128),
            "read_bytes": round(32 * n32 + 64 * n64 + 128 * n128),
            "read_dram_requests": round(g("TCC_EA0_RDREQ_DRAM_sum")),
            "write_requests": round(wr), "write_bytes": round(32 * (wr - wr64) + 64 * wr64),
            "l2_hit_rate": round(hit / (hit + miss), 4) if hit + miss else None,
        }
    print(json.dumps(res, indent=1))
    # bench.py's traffic file (profiles/pmc_traffic.json): exact HBM-side bytes per launch of every
    # kernel, tied to the library's build id
    try:
        from zkfl import native
        bid = native.build_id()
    except Exception as e:  # noqa: BLE001
        bid = f"unknown ({e})"
    with open(os.path.join(d, "pmc_traffic.json"), "w") as f:
        json.dump({"build_id": bid, "unit": "bytes per launch",
                   "method": "rocprofv3 --pmc, three separate passes (tools/pmc_attrib.sh): L2 -> memory read "
                             "requests by size, 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B (exact; "
                             "FETCH_SIZE counts a 128-B request as 64 B on gfx950), writes 32 x (WRREQ - "
                             "WRREQ_64B) + 64 x WRREQ_64B; one-slot run of circuit "
                             + (sys.argv[2] if len(sys.argv) > 2 else "M"),
                   "kernels": kernels}, f, indent=1)


if __name__ == "__main__":
    main()
