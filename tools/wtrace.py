#!/usr/bin/env python3
"""Wave-level timeline of the prover under load (GPU box; library built with -DZK_WTRACE=1:
`bash tools/build_ab.sh wtrace "-DZK_WTRACE=1"`, then ZKFL_LIB=build_ab/wtrace/libzkfl.so).

Every instrumented kernel's waves record {kind, HW_ID, start, end} (csrc/wtrace.h) -- one atomic
and one store per wave, so unlike rocprofv3's kernel trace (which cost the 20-slot bench a third
of its throughput) the timeline is the unperturbed one.  This runs the bench's workload (M, 20
slots) and reports, over the timed window:
  * per kernel kind: waves per proof, wave-time per proof (sum of wave durations), mean wave
    duration, the mean number of its waves resident;
  * the share of the window with an accumulation kernel resident, and the mean SIMD share held by
    each kind (a wave's VGPR allocation / 512 per SIMD, from the code object: tools/isa_check.py);
  * the same for proofs run one at a time (--isolated), with the last one's kernel timeline (per
    kernel kind, the stretches in which its waves ran back to back: start, end, waves, clock).
Writes <out>/summary.json, <out>/waves.npz (kind, t0, t1 in 10-ns ticks) for the first --keep
proofs' window and <out>/waves_isolated.npz (every record of the isolated proofs).

    ZKFL_LIB=build_ab/wtrace/libzkfl.so python3 tools/wtrace.py --proofs 120 --out gpurun_out/wt
    --c5 ROUNDS: instead, config 5 (bench.py's c5 leg: ROUNDS federated rounds of 8 clients x
    {training, secure aggregation} through zkfl_groth16_full_prove_multi, witnesses included)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("ZKFL_HW_QUEUES", "28")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

KINDS = {1: "acc", 2: "stitch", 3: "wsum0", 4: "wsum1", 5: "sort_count", 6: "sort_scan", 7: "sort_scatter",
         8: "sort_bins", 9: "tail_reset", 10: "ntt_cols_inv", 11: "ntt_lds", 12: "ntt_cols_fwd", 13: "abc",
         14: "abc_rows", 15: "join", 16: "assemble", 17: "set_extra", 18: "witness"}
# kernel symbol fragment per kind (for the VGPR allocation); G2 kinds use the Fq2Pair29 instance
SYMBOL = {"acc": "k_msm_accumulate", "stitch": "k_msm_stitch", "wsum0": "k_msm_wsumI.*Lb1", "wsum1": "k_msm_wsumI.*Lb0",
          "sort_count": "k_msm_bin_count", "sort_scan": "k_msm_bin_scan", "sort_scatter": "k_msm_bin_scatter",
          "sort_bins": "k_msm_bin_sort", "tail_reset": "k_msm_tail_reset", "ntt_cols_inv": "k_ntt_colsILb1",
          "ntt_lds": "k_ntt_lds_pair", "ntt_cols_fwd": "k_ntt_colsILb0", "abc": "k_abc_chunks", "abc_rows": "k_abc_rows",
          "join": "k_join", "assemble": "k_assemble", "set_extra": "k_proof_start", "witness": "k_wit_lvl"}


def kind_name(k):
    base = KINDS.get(k & 31, f"k{k & 31}")
    return base + ("_g2" if k & 32 else "") + ("_joint" if k & 64 else "")


def vgpr_share(lib_path):
    """kind name -> SIMD share of one wave (VGPRs rounded to the allocation granule of 8, / 512)."""
    import isa_check
    res = isa_check.resources(lib_path, r"k_msm_|k_ntt_|k_abc_|k_join|k_assemble|k_proof_start")
    out = {}
    for name, pat in SYMBOL.items():
        import re
        for g2 in (False, True):
            cands = [(s, r) for s, r in res.items() if re.search(pat, s)]
            curve = name in ("acc", "stitch", "wsum0", "wsum1", "tail_reset")  # G1 / G2 instances
            if g2 and not curve:
                continue
            if curve:
                cands = [(s, r) for s, r in cands if ("Fq2" in s) == g2]
            if cands:
                v = max(r.get("vgpr_count", 0) for _, r in cands)
                out[name + ("_g2" if g2 else "")] = min(1.0, ((v + 7) // 8 * 8) / 512.0)
    return out


def analyse(rec, n_proofs, shares):
    kind = rec["kind"].astype(np.int64)
    t0 = rec["t0"].astype(np.int64)
    t1 = rec["t1"].astype(np.int64)
    lo, hi = int(t0.min()), int(t1.max())
    span = max(1, hi - lo)
    ticks_us = 0.01  # s_memrealtime: 100 MHz
    out = {"window_ms": span * ticks_us / 1e3, "proofs": n_proofs, "waves": int(len(kind)),
           "ms_per_proof": span * ticks_us / 1e3 / n_proofs, "kinds": {}}
    for k in sorted(set(kind.tolist())):
        m = kind == k
        d = (t1[m] - t0[m]) * ticks_us
        name = kind_name(k)
        sh = shares.get(name, shares.get(name.replace("_g2", ""), 0.0))
        out["kinds"][name] = {
            "waves_per_proof": round(int(m.sum()) / n_proofs, 1),
            "wave_ms_per_proof": round(float(d.sum()) / 1e3 / n_proofs, 3),
            "mean_wave_us": round(float(d.mean()), 1),
            "mean_resident_waves": round(float(d.sum()) / (span * ticks_us), 1),
            "simd_share_per_wave": round(sh, 3),
            "mean_simd_share": round(float(d.sum()) * sh / (span * ticks_us) / 1024.0, 4),  # of the 1024 SIMDs
        }
        if "c0" in rec.dtype.names:  # the shader clock the waves ran at: cycles / real time
            cyc = (rec["c1"][m].astype(np.int64) - rec["c0"][m].astype(np.int64)).astype(np.float64)
            real = (t1[m] - t0[m]).astype(np.float64) * 1e-8  # seconds
            ok = real > 2e-6
            if ok.any():
                out["kinds"][name]["clock_GHz"] = round(float(cyc[ok].sum() / real[ok].sum() / 1e9), 3)
    # share of the window with >= 1 accumulation wave resident (G1 or G2)
    acc = (kind & 31) == 1
    ev = np.concatenate([np.stack([t0[acc], np.ones(acc.sum(), np.int64)], 1),
                         np.stack([t1[acc], -np.ones(acc.sum(), np.int64)], 1)])
    ev = ev[np.lexsort((-ev[:, 1], ev[:, 0]))]
    cur, last, busy = 0, lo, 0
    for t, dlt in ev:
        if cur > 0:
            busy += t - last
        cur += dlt
        last = t
    out["acc_resident_share"] = round(busy / span, 4)
    # share of the window with ANY instrumented wave resident (the rest: the GPU idle, waiting for
    # the host or for uninstrumented work such as copies)
    ev = np.concatenate([np.stack([t0, np.ones(len(t0), np.int64)], 1), np.stack([t1, -np.ones(len(t1), np.int64)], 1)])
    ev = ev[np.lexsort((-ev[:, 1], ev[:, 0]))]
    cur, last, busy = 0, lo, 0
    for t, dlt in ev:
        if cur > 0:
            busy += t - last
        cur += dlt
        last = t
    out["any_resident_share"] = round(busy / span, 4)
    out["simd_share_total"] = round(sum(v["mean_simd_share"] for v in out["kinds"].values()), 4)
    return out


def proofs_of(rec, gap_us=150.0):
    """Split a one-proof-at-a-time trace into proofs: a proof ends where no wave is resident for
    more than gap_us (the host's turn between prove calls)."""
    o = np.argsort(rec["t0"], kind="stable")
    r = rec[o]
    t0, t1 = r["t0"].astype(np.int64), r["t1"].astype(np.int64)
    run_end = np.maximum.accumulate(t1)
    cut = np.nonzero(t0[1:] > run_end[:-1] + int(gap_us * 100))[0] + 1
    return np.split(r, cut)


def gantt(rec):
    """One proof's kernel timeline: per kind, the stretches in which its waves follow each other
    without a gap (one launch, or launches of that kind back to back), times from the proof's start."""
    lo = int(rec["t0"].min())
    segs = []
    for k in sorted(set(rec["kind"].tolist())):
        r = rec[rec["kind"] == k]
        r = r[np.argsort(r["t0"], kind="stable")]
        t0, t1 = r["t0"].astype(np.int64), r["t1"].astype(np.int64)
        run_end = np.maximum.accumulate(t1)
        cut = np.nonzero(t0[1:] > run_end[:-1])[0] + 1
        for part in np.split(np.arange(len(r)), cut):
            a, b = int(t0[part].min()), int(t1[part].max())
            cyc = float((r["c1"][part].astype(np.int64) - r["c0"][part].astype(np.int64)).sum())
            real = float((t1[part] - t0[part]).sum()) * 1e-8
            segs.append({"kind": kind_name(k), "start_us": round((a - lo) / 100, 1), "end_us": round((b - lo) / 100, 1),
                         "waves": int(len(part)), "mean_wave_us": round(float((t1[part] - t0[part]).mean()) / 100, 1),
                         "clock_GHz": round(cyc / real / 1e9, 3) if real > 0 else None})
    segs.sort(key=lambda s: s["start_us"])
    return segs


def c5_trace(args, shares, dt):
    """Config 5 under the tracer: the c5 leg's keys and jobs (bench.py), one full_prove_multi call."""
    import json as _json
    sys.path.insert(0, ROOT)
    import bench
    from zkfl import circuits, clients, native, wprog, zkey
    ctx = native.Context(0)
    circ = {"train": circuits.build("sgd_verified", 8, 4, 3, 1000), "secagg": circuits.build("secure_masked_update", 4, 7)}
    keys, progs, images = {}, {}, {}
    for i, (nm, b) in enumerate(circ.items()):
        zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=0xC5 + i, alpha=3, beta=5, gamma=7, delta=11 + i))
        keys[nm] = native.ProvingKey(ctx, zk)
        keys[nm].set_slots(args.c5_slots)
        images[nm] = wprog.compile_program(b)
        progs[nm] = native.WitnessProgram(ctx, images[nm])

    def jobs(nrounds, first):
        out = []
        for r in range(nrounds):
            for tr, sa, _ in clients.federated_round(8, rnd=r + 1, first_id=first):
                out += [("train", _json.dumps(tr)), ("secagg", _json.dumps(sa))]
        return [(keys[nm], progs[nm], native.parse_inputs(images[nm], txt)) for nm, txt in out]
    ctx.full_prove_multi(jobs(1, 1))
    ctx.synchronize()
    js = jobs(args.c5, 1)
    cap = 200000 * (len(js) + 4)
    ctx.wtrace_start(cap)
    t = time.perf_counter()
    ctx.full_prove_multi(js)
    ctx.synchronize()
    wall = time.perf_counter() - t
    raw, n = ctx.wtrace_stop(cap)
    rec = np.frombuffer(raw, dtype=dt)
    out = analyse(rec, len(js), shares)
    out["host_wall_ms_per_proof"] = wall * 1e3 / len(js)
    out["proofs_per_s"] = len(js) / wall
    out["records"], out["overflow"] = int(n), bool(n > cap)
    np.savez_compressed(os.path.join(args.out, "waves_c5.npz"), rec=rec)
    # the batch chain of one small proof with nothing beside it: the training key on one slot, two
    # proofs through the same pipe (witness group, then the proofs one after the other); the
    # timeline of the second
    keys["train"].set_slots(1)
    one = [j for j in jobs(1, 1) if j[0] is keys["train"]][:2]
    ctx.full_prove_multi(one)
    ctx.synchronize()
    ctx.wtrace_start(200000)
    ctx.full_prove_multi(one)
    ctx.synchronize()
    raw, n = ctx.wtrace_stop(200000)
    rec1 = np.frombuffer(raw, dtype=dt)
    out["isolated_gantt"] = gantt(rec1)
    ctx.wtrace_free()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proofs", type=int, default=120)
    ap.add_argument("--slots", type=int, default=20)
    ap.add_argument("--isolated", type=int, default=4, help="proofs run one at a time afterwards")
    ap.add_argument("--keep", type=int, default=30, help="proofs whose raw waves go to waves.npz")
    ap.add_argument("--out", default="gpurun_out/wtrace")
    ap.add_argument("--c5", type=int, default=0, help="config-5 rounds to trace instead of M")
    ap.add_argument("--c5-slots", type=int, default=8)
    args = ap.parse_args()
    if args.c5:
        from zkfl import native
        os.makedirs(args.out, exist_ok=True)
        dt = np.dtype([("kind", "<u4"), ("hwid", "<u4"), ("t0", "<u8"), ("t1", "<u8"), ("c0", "<u8"), ("c1", "<u8")])
        shares = vgpr_share(native.LIB_PATH)
        s = c5_trace(args, shares, dt)
        with open(os.path.join(args.out, "summary_c5.json"), "w") as f:
            json.dump(s, f, indent=1)
        print(f"== c5: {s['proofs_per_s']:.1f} proofs/s under the tracer, {s['ms_per_proof']:.3f} ms per proof (trace "
              f"window), any wave resident {100 * s['any_resident_share']:.1f}%, accumulation resident "
              f"{100 * s['acc_resident_share']:.1f}%, SIMD share {s['simd_share_total']:.3f}")
        for k, v in sorted(s["kinds"].items(), key=lambda kv: -kv[1]["wave_ms_per_proof"]):
            print(f"   {k:14s} waves/proof {v['waves_per_proof']:9.1f}  wave-ms/proof {v['wave_ms_per_proof']:9.3f}  "
                  f"mean wave {v['mean_wave_us']:8.1f} us  resident {v['mean_resident_waves']:7.1f}  "
                  f"SIMD share {v['mean_simd_share']:.4f}")
        print("== c5 training proofs alone (witness group, then two proofs on one slot):")
        for g in s["isolated_gantt"]:
            print(f"   {g['kind']:14s} {g['start_us']:8.1f} .. {g['end_us']:8.1f} us  waves {g['waves']:6d}  "
                  f"mean wave {g['mean_wave_us']:7.1f} us  clock {g['clock_GHz']} GHz")
        return
    from zkfl import circuits, clients, native, wprog, zkey
    os.makedirs(args.out, exist_ok=True)
    b = circuits.build("sgd_verified", 128, 4, 7, 1000)
    objs = [clients.Client(c + 1, 128, 4, 7, clients.JsLcg(12345 + c)).training_input(128, 1000, 100000000)[0]
            for c in range(4)]
    ctx = native.Context(0)
    zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=0x5EED, alpha=0xA1, beta=0xB2, gamma=0xC3, delta=0xD4))
    key = native.ProvingKey(ctx, zk)
    key.set_slots(args.slots)
    wp = native.WitnessProgram(ctx, wprog.compile_program(b))
    res = wp.compute_resident(key, [wprog.input_bytes(b, o) for o in objs])
    key.prove_batch([res[i % 4] for i in range(2 * args.slots)])
    ctx.synchronize()
    shares = vgpr_share(native.LIB_PATH)
    dt = np.dtype([("kind", "<u4"), ("hwid", "<u4"), ("t0", "<u8"), ("t1", "<u8"), ("c0", "<u8"), ("c1", "<u8")])
    summary = {"library": native.LIB_PATH, "slots": args.slots, "simd_share_per_wave": shares}
    cap = 80000 * (args.proofs + 4)
    # under load
    ctx.wtrace_start(cap)
    t = time.perf_counter()
    key.prove_batch([res[i % 4] for i in range(args.proofs)])
    ctx.synchronize()
    wall = time.perf_counter() - t
    raw, n = ctx.wtrace_stop(cap)
    rec = np.frombuffer(raw, dtype=dt)
    summary["loaded"] = analyse(rec, args.proofs, shares)
    summary["loaded"]["host_wall_ms_per_proof"] = wall * 1e3 / args.proofs
    summary["loaded"]["records"], summary["loaded"]["overflow"] = int(n), bool(n > cap)
    lo = int(rec["t0"].min())
    sel = rec[rec["t0"] < lo + (rec["t1"].max() - lo) * args.keep // max(1, args.proofs)]
    np.savez_compressed(os.path.join(args.out, "waves.npz"), kind=sel["kind"].astype(np.uint8),
                        t0=(sel["t0"] - lo).astype(np.uint32), t1=(sel["t1"] - lo).astype(np.uint32),
                        cu=((sel["hwid"] >> 8) & 0xFF).astype(np.uint8))
    # one proof at a time
    if args.isolated:
        key.set_slots(1)
        ctx.wtrace_start(80000 * (args.isolated + 1))
        for i in range(args.isolated):
            key.prove_batch([res[i % 4]])
        ctx.synchronize()
        raw, n = ctx.wtrace_stop(80000 * (args.isolated + 1))
        rec = np.frombuffer(raw, dtype=dt)
        summary["isolated"] = analyse(rec, args.isolated, shares)
        np.savez_compressed(os.path.join(args.out, "waves_isolated.npz"), rec=rec)
        ps = proofs_of(rec)
        summary["isolated"]["proof_spans_us"] = [round((int(p["t1"].max()) - int(p["t0"].min())) / 100, 1) for p in ps]
        summary["isolated"]["gantt_last"] = gantt(ps[-1])
    ctx.wtrace_free()
    with open(os.path.join(args.out, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    for mode in ("loaded", "isolated"):
        if mode not in summary:
            continue
        s = summary[mode]
        print(f"== {mode}: {s['ms_per_proof']:.3f} ms per proof (trace window), accumulation resident "
              f"{100 * s['acc_resident_share']:.1f}% of it, SIMD share held {s['simd_share_total']:.3f}")
        for k, v in sorted(s["kinds"].items(), key=lambda kv: -kv[1]["mean_simd_share"]):
            print(f"   {k:14s} waves/proof {v['waves_per_proof']:9.1f}  wave-ms/proof {v['wave_ms_per_proof']:9.3f}  "
                  f"mean wave {v['mean_wave_us']:8.1f} us  resident {v['mean_resident_waves']:7.1f}  "
                  f"SIMD share {v['mean_simd_share']:.4f}  clock {v.get('clock_GHz', 0):.2f} GHz")
    if "gantt_last" in summary.get("isolated", {}):
        print("== isolated proof spans (us):", summary["isolated"]["proof_spans_us"])
        for g in summary["isolated"]["gantt_last"]:
            print(f"   {g['kind']:14s} {g['start_us']:8.1f} .. {g['end_us']:8.1f} us  waves {g['waves']:6d}  "
                  f"mean wave {g['mean_wave_us']:7.1f} us  clock {g['clock_GHz']} GHz")


if __name__ == "__main__":
    main()
