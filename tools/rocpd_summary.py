#!/usr/bin/env python3
"""Summaries of rocprofv3 (ROCm 7.2, rocpd SQLite output) runs for profiles/.

  rocpd_summary.py kernels RUN.db OUT.csv
      per-kernel calls / total / avg / min / max duration from --kernel-trace
  rocpd_summary.py roofline RUN.db BENCH.log OUT.json
      the dispatches of bench.py's serialized roofline pass (the last `launches` dispatches of
      each instrumented kernel in a traced bench.py run): median / mean duration, to compare with
      the bench line's roofline.avg_launch_ms (median) / mean_launch_ms
  rocpd_summary.py breakdown RUN.db OUT.csv [PROOFS]
      per-proof kernel time of bench.py's serialized roofline pass (the last PROOFS=6 proofs,
      one slot, every kernel alone on the GPU): where a proof's device time goes
  rocpd_summary.py timeline RUN.db OUT.txt
      concurrency over the timed (throughput) region of a traced bench.py run: fraction of wall time
      with k kernels of each category running, from 10-us samples
  rocpd_summary.py pmc FETCH.db WRITE.db CALIB.db OUT.json [BUILD_ID]
      per-kernel average FETCH_SIZE / WRITE_SIZE per launch (separate --pmc passes, as
      MI355X_MICROARCH.md §rocprofv3 PMC slots requires), plus the FETCH_SIZE calibration of the
      MSM gather pattern from tools/pmc_calib.hip (CALIB.db: --pmc FETCH_SIZE of pmc_calib):
      factor = known bytes / reported bytes for 64-B (G1) and 128-B (G2) records.
      bench.py reads OUT.json (profiles/pmc_traffic.json) for the roofline "traffic" field, and only
      when BUILD_ID (the profiled libzkfl.so's zkfl_build_id) equals the library it has loaded.
"""
import csv
import json
import sqlite3
import sys

CALIB_LANES = 4 << 20  # tools/pmc_calib.hip


def kernels(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     "from kernels group by name order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ms", "avg_us", "min_us", "max_us", "pct"])
        for r in rows:
            w.writerow([r[0], r[1], round(r[2] / 1e6, 3), round(r[3] / 1e3, 2), round(r[4] / 1e3, 2),
                        round(r[5] / 1e3, 2), round(100 * r[2] / tot, 2)])


def _pmc(db, counter):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, count(*), avg(value) from counters_collection where counter_name=? "
                     "group by kernel_name", (counter,)).fetchall()
    return {r[0]: (r[1], r[2]) for r in rows}  # KiB per launch


def pmc(fetch_db, write_db, calib_db, out, build_id=None):
    fetch, write = _pmc(fetch_db, "FETCH_SIZE"), _pmc(write_db, "WRITE_SIZE")
    calib = _pmc(calib_db, "FETCH_SIZE")
    factors = {}
    for rb in (64, 128):
        k = [v for n, v in calib.items() if f"k_gather<{rb}>" in n]
        factors[rb] = (CALIB_LANES * rb) / (k[0][1] * 1024) if k else None
    res = {"unit": "bytes per launch", "build_id": build_id, "fetch_calibration": {
        "g1_64B_records": factors[64], "g2_128B_records": factors[128],
        "method": "tools/pmc_calib.hip: 4 Mi lanes each gather one random record from a 4 GiB table; "
                  "factor = known bytes / FETCH_SIZE bytes"}, "kernels": {}}
    for name, (n, f_kib) in fetch.items():
        w_kib = write.get(name, (0, 0.0))[1]
        rb = 128 if "Fq2Ops" in name else 64
        fac = factors[rb] if "k_msm_accumulate" in name and factors[rb] else 1.0
        res["kernels"][name] = {"launches": n, "fetch_raw": round(f_kib * 1024), "write": round(w_kib * 1024),
                                "fetch_factor": round(fac, 4),
                                "traffic": round(f_kib * 1024 * fac + w_kib * 1024)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


ROOFLINE_KERNELS = {"msm_accumulate_g1": "k_msm_accumulate<zkfl::FqOps",
                    "msm_accumulate_g2": "k_msm_accumulate<zkfl::Fq2"}


def roofline(db, bench_log, out):
    line = [ln for ln in open(bench_log) if ln.startswith("{")][-1]
    rep = json.loads(line)
    n = rep["roofline"]["launches"]
    c = sqlite3.connect(db)
    res = {"bench_roofline": rep["roofline"], "trace": {}}
    for tag, sym in ROOFLINE_KERNELS.items():
        d = [r[0] for r in c.execute("select end-start from kernels where name like ? order by start",
                                     (f"%{sym}%",)).fetchall()]
        per = rep["roofline"].get("launches_per_proof", 4)            # G1 MSM launches per G2 MSM
        launches = n if tag == rep["roofline"]["kernel"] else n // per
        last = sorted(x / 1e6 for x in d[-launches:])
        if last:
            mid = len(last) // 2
            med = last[mid] if len(last) % 2 else 0.5 * (last[mid - 1] + last[mid])
            res["trace"][tag] = {"dispatches": len(last), "median_ms": round(med, 4),
                                 "mean_ms": round(sum(last) / len(last), 4),
                                 "min_ms": round(last[0], 4), "max_ms": round(last[-1], 4)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


def _short(name):
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void rocprim"):
        return "rocprim::" + name.split("detail::")[2].split("<")[0]
    return name.split("(")[0].replace("void ", "").replace("zkfl::", "")


def breakdown(db, out, proofs=6):
    """k_proof_start opens every proof (zkfl.hip enqueue_proof_body); the roofline pass is the last
    `proofs` proofs of the run, serialized on one stream."""
    c = sqlite3.connect(db)
    starts = [r[0] for r in c.execute("select start from kernels where name like '%k_proof_start%' or name like '%k_set_extra%' order by start")]
    t0 = starts[-proofs]
    # the pass ends with its last proof's k_assemble (bench.py verifies the proofs afterwards)
    t1 = c.execute("select max(end) from kernels where name like '%k_assemble(%'").fetchone()[0]
    rows = c.execute("select name, count(*), sum(end-start) from kernels where start >= ? and end <= ? "
                     "group by name", (t0, t1)).fetchall()
    span = t1 - t0
    agg = {}
    for name, cnt, tot in rows:
        k = _short(name)
        a = agg.setdefault(k, [0, 0])
        a[0] += cnt
        a[1] += tot
    busy = sum(v[1] for v in agg.values())
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "launches_per_proof", "ms_per_proof", "pct_of_busy"])
        for k, (cnt, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([k, round(cnt / proofs, 2), round(tot / 1e6 / proofs, 4), round(100 * tot / busy, 2)])
        w.writerow(["(busy total)", "", round(busy / 1e6 / proofs, 4), 100.0])
        w.writerow(["(wall span)", "", round(span / 1e6 / proofs, 4), ""])


def _category(name):
    for key, cat in (("k_msm_accumulate<zkfl::FqOps", "acc_g1"), ("k_msm_accumulate<zkfl::Fq2", "acc_g2"),
                     ("bin_", "sort"),
                     ("stitch", "stitch"), ("wsum", "reduce"), ("rocprim", "sort"),
                     ("k_ntt", "ntt"), ("k_abc", "abc"), ("assemble", "asm")):
        if key in name:
            return cat
    return "other"


def timeline(db, out, step_us=10.0):
    """Samples the window between the timed region and the start of the serialized roofline pass
    (its first k_proof_start is the 6th from last)."""
    c = sqlite3.connect(db)
    ks = c.execute("select name, start, end from kernels order by start").fetchall()
    sx = [k[1] for k in ks if "k_proof_start" in k[0]]
    t_end = sx[-6]
    t_begin = sx[len(sx) // 4]  # skip warmup-ish quarter
    cats = {}
    for name, s0, e0 in ks:
        if e0 < t_begin or s0 > t_end:
            continue
        cats.setdefault(_category(name), []).append((max(s0, t_begin), min(e0, t_end)))
    nsamp = int((t_end - t_begin) / (step_us * 1e3))
    lines = [f"window {(t_end - t_begin) / 1e6:.2f} ms, {nsamp} samples of {step_us} us"]
    import bisect
    tot_any = [0] * nsamp
    for cat, iv in sorted(cats.items()):
        cnt = [0] * nsamp
        for s0, e0 in iv:
            a = int((s0 - t_begin) / (step_us * 1e3))
            b = int((e0 - t_begin) / (step_us * 1e3))
            for k in range(max(a, 0), min(b + 1, nsamp)):
                cnt[k] += 1
                tot_any[k] += 1
        hist = {}
        for v in cnt:
            hist[v] = hist.get(v, 0) + 1
        busy = sum(1 for v in cnt if v) / max(1, nsamp)
        mean = sum(cnt) / max(1, nsamp)
        lines.append(f"{cat:8s} busy {busy:6.1%}  mean running {mean:5.2f}  dist " +
                     " ".join(f"{k}:{v / nsamp:.0%}" for k, v in sorted(hist.items()) if v / nsamp >= 0.01))
    lines.append(f"all      mean running {sum(tot_any) / max(1, nsamp):5.2f}")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    if sys.argv[1] == "timeline":
        timeline(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "breakdown":
        breakdown(sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 6)
    elif sys.argv[1] == "kernels":
        kernels(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "roofline":
        roofline(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        pmc(*sys.argv[2:7])
