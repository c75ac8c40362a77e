#!/usr/bin/env python3
"""Groth16 proofs/sec on the ZK-FL training-step circuit (~2^18 constraints), 1..N MI355X.

Workload (BASELINE.json metric): TrainingStepVerified(BATCH=128,
DIM=4, DEPTH=7, PRECISION=1000) — the reference's sgd_verified.circom at the Report's N=128
scale — with synthetic client inputs from the reference harness's seeded generator
(tests/full_system_simulation.mjs:273-303, weights = 0, tau^2 = 1e8, round 1).

A step = one batch of `--slots` Groth16 proofs (ABC, 3x coset NTT, 4 G1 + 1 G2 MSM, assembly),
one per in-flight proof slot, from device-resident witnesses with the proving key resident in HBM;
K steps = K x slots proofs pushed through the batch prover in one call (the slots stay full across
step boundaries).  r, s come from the OS CSPRNG on the host and are passed in, so every timed
proof is checked after the timed region: all of them by the GPU batch verifier, and the first one
bit-for-bit against the C oracle inside the cpu_baseline leg.  Multi-GPU: one process per GPU,
independent proofs per rank (weak scaling, no collective on the data path); the barrier /
max-over-ranks timing uses torch.distributed.

Prints ONE JSON line on rank 0 (see DESIGN.md §6 for the roofline definitions).
"""

from __future__ import annotations

import argparse
import json
import os
import resource
import sys
import time

# Each in-flight proof slot drives one HIP stream; HIP maps a process's streams onto
# GPU_MAX_HW_QUEUES hardware queues (HIP default 4, which the GPU boxes also export), and streams
# sharing a queue serialize.  Set it before anything initializes HIP.  Measured on MI355X
# (tools/concurrency_probe.hip): kernels on distinct streams run concurrently up to ~20 at 24
# queues, while 32 queues oversubscribe the hardware queue slots; 20 slots x 1 stream at 28 queues
# is the best measured configuration (322.2 / 320.0 against 317.4 for 16 x 24,
# profiles/r01_experiments.md).  ZKFL_HW_QUEUES overrides the value used here.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("ZKFL_HW_QUEUES", "28")

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd")
sys.path.insert(0, PKG_DIR)

METRIC = "Groth16 proofs/sec (training-step circuit, ~2^18 constraints) at 1/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# Roofline of record: algorithmic bytes of one G1 MSM = every base of its query
# read once (64 B affine) + its scalar (32 B); a launch of k_msm_accumulate<G1> is one MSM (A, B1,
# C or H, query lengths nVars, nVars, nVars - nPublic - 1, domainSize).
ALGO_BYTES_PER_BASE = {"msm_accumulate_g1": 64 + 32, "msm_accumulate_g2": 128 + 32}
# What this implementation moves instead: bases are window-expanded 16x at key load
# so every accumulated (base, window) entry reads its own 64 B / 128 B point + 2 B key + 4 B index.
IMPL_BYTES_PER_ENTRY = {"msm_accumulate_g1": 2 + 4 + 64, "msm_accumulate_g2": 2 + 4 + 128}
# Fq multiplications per entry: XYZZ mixed addition madd-2008-s = 8M + 2S over Fq (G1), over Fq2
# (G2: 3 Fq products per Fq2 product)
FQMUL_PER_ENTRY = {"msm_accumulate_g1": 10, "msm_accumulate_g2": 30}
# Integer-VALU ceiling from ISA issue rates, not from this library's own timing: the G1 kernels
# multiply in nine 29-bit limbs (csrc/field29.h), a Montgomery product is 81 + 81 v_mad_u64_u32
# (a*b and m*p limb products, 64-bit column accumulators, no carry adds); issue cost relative to a
# 2-cycle wave64 v_add_u32 is 2.2x (tools/isa_rate.hip, MI355X).  1024 SIMDs x 32 lanes/cycle x
# 2.4 GHz / (162 x 2.2) = 220.7 G Fq-mul/s.  (32-bit limbs: 128 mad + 128 carry adds, 2.2x / 1.8x:
# 153.6 G/s -- the G2 kernels' ceiling.)
FQMUL_PEAK_GPS = 1024 * 32 * 2.4 / (162 * 2.2)
FQMUL_PEAK_GPS_32 = 1024 * 32 * 2.4 / (128 * 2.2 + 128 * 1.8)
# rocprofv3 kernel names of the instrumented kernels (profiles/pmc_traffic.json keys)
KERNEL_SYMBOL = {"msm_accumulate_g1": "k_msm_accumulate<zkfl::FqOps",   # FqOps29 (G1 compute type)
                 "msm_accumulate_g2": "k_msm_accumulate<zkfl::Fq2"}     # Fq2PairOps
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")
# SQ / GRBM counters of the shipped kernels (tools/sq_r03.sh): the effective clock of the G1
# accumulation under load (GRBM_GUI_ACTIVE / 8 / duration) prices the VALU ceiling at the clock the
# chip actually holds (DVFS), beside the 2.4 GHz figure
SQ_COUNTERS = os.path.join(ROOT, "profiles", "sq_counters.json")
# the same two summaries for the 2^19-domain leg's key (tools/profile_round.sh: pmc_attrib.sh .. M19,
# SQ_CIRCUIT=M19 sq_r03.sh), so that leg's roofline carries its own traffic and clock
PMC_TRAFFIC_M19 = os.path.join(ROOT, "profiles", "pmc_traffic_m19.json")
SQ_COUNTERS_M19 = os.path.join(ROOT, "profiles", "sq_counters_m19.json")
PROFILED = ("msm_accumulate_g1", "msm_accumulate_g2", "ntt", "abc", "assemble", "prove")

CIRCUITS = {
    "M": ("sgd_verified", (128, 4, 7, 1000)),
    "C2": ("sgd_verified", (8, 4, 3, 1000)),
    # circom's compile of the Report's N=128 training circuit has ~283 K constraints (Report.pdf p.6
    # Table 5) -> domain 2^19; this build's tighter R1CS reaches that count (283,407) at BATCH = 124
    # with a depth-8 dataset tree (a depth-7 tree holds at most 128 samples)
    "M19": ("sgd_verified", (124, 4, 8, 1000)),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline_leg(zk: bytes, wt: bytes, rs: bytes, seconds_budget=20.0):
    """Oracle ("port") on the host cores: the C restatement (oracle/c/groth16_ref.c) proving
    the same zkey/wtns with the same (r, s) as the first timed GPU proof, bounded to
    ~seconds_budget, reported as proofs/s.  -> (report dict, the oracle's proof bytes)."""
    sys.path.insert(0, ROOT)
    from oracle import cbaseline
    return cbaseline.time_prove(zk, wt, seconds_budget, rs)


def draw_rs(n):
    """n x (r || s), 32 B little-endian each, uniform below the BN254 scalar order (OS CSPRNG)."""
    import secrets
    from zkfl.field import R
    return b"".join(secrets.randbelow(R).to_bytes(32, "little") + secrets.randbelow(R).to_bytes(32, "little")
                    for _ in range(n))


def timed_run(key, warm_w, steps_w, rs, ctx, dist):
    """W untimed steps, then exactly K timed steps (K x slots proofs in one batch call) bracketed
    by barrier + synchronize on both sides; returns (max-over-ranks elapsed seconds, proofs, host
    CPU seconds of this process over the timed region -- the warm-up's graph captures excluded)."""
    if warm_w:
        key.prove_batch(warm_w)
    _barrier(ctx, dist)
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t_start = time.perf_counter()
    proofs = key.prove_batch(steps_w, rs)      # K steps x `slots` proofs, `slots` in flight
    _barrier(ctx, dist)
    dt = time.perf_counter() - t_start
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    busy = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    return _max_over_ranks(dt, dist), proofs, busy


def verify_all(ctx, zk, proofs, pubs_of):
    """Every timed proof through the GPU batch verifier (zkfl_groth16_verify_batch)."""
    from zkfl import groth16
    vk = groth16.vk_bytes(groth16.export_verification_key(zk, alphabeta=False))
    pubs = b"".join(pubs_of(i) for i in range(len(proofs)))
    npub = len(pubs_of(0)) // 32
    ok = ctx.verify_batch(vk, pubs, b"".join(proofs), npub)
    return sum(ok)


def cli_leg(ctx, runs, names=("C2", "M")):
    """Like-for-like with how the reference proves (Report Table 3's 6.8 s is one
    `snarkjs groth16 prove` CLI invocation): the harness's exact command
    `npx snarkjs groth16 prove <c>_final.zkey <w>.wtns <proof>.json <public>.json`
    (tests/full_system_simulation.mjs:773-776, one child process per proof, cwd = the circuit dir),
    resolved offline by npm to this package's shim (node/snarkjs_shim.js -> N-API -> C ABI), run
    `runs` times per circuit; the witness comes from the harness's generate_witness.cjs string
    (:758-763).  Per circuit: median wall clock of the command and the median of each stage
    (npx and node start, libzkfl + HIP runtime load, HIP context, zkey map + parse, wait for the
    context, key load -- parse,
    QAP upload, base upload + 16x window expansion per query, first proof slot --, wtns read, GPU
    prove, JSON write) from the shim's and the library's timing marks (ZKFL_CLI_TIMING,
    ZKFL_LOAD_TIMING).  Every CLI proof is checked by the GPU batch verifier."""
    import shutil
    import statistics
    import subprocess
    import tempfile
    from zkfl import clients, groth16
    if not shutil.which("node") or not shutil.which("npm"):
        return {"skipped": "node / npm not found"}
    med = statistics.median
    tmp = tempfile.mkdtemp(prefix="zkfl_cli_")
    env = dict(os.environ, PYTHONPATH=PKG_DIR + os.pathsep + os.environ.get("PYTHONPATH", ""))

    def run(cmd, cwd, extra=None):
        p = subprocess.run(cmd, cwd=cwd, shell=True, capture_output=True, text=True, timeout=300,
                           env=dict(env, **(extra or {})))
        if p.returncode != 0:
            raise RuntimeError(f"{cmd}: {p.stderr[-400:]}")
        return p
    try:
        with open(os.path.join(tmp, "package.json"), "w") as f:
            json.dump({"name": "harness", "version": "1.0.0", "private": True,
                       "dependencies": {"zkfl-snarkjs": "file:" + PKG_DIR}}, f)
        run("npm install --offline --no-audit --no-fund", tmp)
        out = {"command": "npx snarkjs groth16 prove <c>_final.zkey <w>.wtns <proof>.json <public>.json",
               "reference": "tests/full_system_simulation.mjs:773-776", "runs": runs}
        for cname in names:
            name, params = CIRCUITS[cname]
            circ = os.path.join(tmp, cname)
            os.makedirs(circ)
            ps = " ".join(str(x) for x in params)
            py = sys.executable
            run(f"{py} -m zkfl compile {name} {ps} --name {name} --circom-layout -o .", circ)
            run(f"{py} -m zkfl setup {name} {ps} --name {name} -o .", circ)
            batch, dim, depth, precision = params
            inp = clients.Client(1, batch, dim, depth, clients.JsLcg(12345)).training_input(batch, precision,
                                                                                             100000000)[0]
            with open(os.path.join(circ, "input.json"), "w") as f:
                json.dump(inp, f)
            t = time.perf_counter()
            run(f'node "{name}_js/generate_witness.cjs" "{name}_js/{name}.wasm" "input.json" "w.wtns"', circ)
            wit_ms = (time.perf_counter() - t) * 1e3
            cli_t, load_t = os.path.join(circ, "cli.jsonl"), os.path.join(circ, "load.jsonl")
            walls = []
            for i in range(runs):
                t = time.perf_counter()
                run(f"npx snarkjs groth16 prove {name}_final.zkey w.wtns proof{i}.json public{i}.json", circ,
                    {"ZKFL_CLI_TIMING": cli_t, "ZKFL_LOAD_TIMING": load_t})
                walls.append((time.perf_counter() - t) * 1e3)
            zk = open(os.path.join(circ, name + "_final.zkey"), "rb").read()
            proofs = [groth16.proof_from_json(json.load(open(os.path.join(circ, f"proof{i}.json"))))
                      for i in range(runs)]
            pubs = [b"".join(int(x).to_bytes(32, "little") for x in json.load(open(os.path.join(circ, f"public{i}.json"))))
                    for i in range(runs)]
            verified = verify_all(ctx, zk, proofs, lambda i: pubs[i])
            marks = [dict(json.loads(ln)["marks"]) for ln in open(cli_t)]
            loads = [json.loads(ln) for ln in open(load_t)]
            # the shim creates the HIP context on a thread of its own while it maps + parses the key
            # file (zkey_read); context_wait = what was left of the context's creation after that
            seq = ["entry", "addon", "context", "zkey_read", "context_wait", "key_load", "wtns_read", "prove",
                   "json_write", "exit"]
            seq = [x for x in seq if all(x in m for m in marks)]
            stages = {"npx_and_node_start": med(w - m["exit"] + m["entry"] for w, m in zip(walls, marks))}
            for a, b_ in zip(seq, seq[1:]):
                stages[{"addon": "libzkfl_and_hip_runtime_load", "context": "hip_context_call"}.get(b_, b_)] = \
                    med(m[b_] - m[a] for m in marks)
            key_load = {k[:-3]: round(med(ld[k] for ld in loads), 2) for k in loads[0] if k.endswith("_ms")}
            out[cname] = {"circuit": f"{name}{params}", "zkey_MB": round(len(zk) / 1e6, 1),
                          "median_ms": round(med(walls), 1), "min_ms": round(min(walls), 1),
                          "verified": verified, "witness_cli_ms": round(wit_ms, 1),
                          "stages_ms": {k: round(v, 1) for k, v in stages.items()},
                          "key_load_stages_ms": key_load}
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def end_to_end_leg(key, wp, image, json_inputs, slots, steps, ctx, dist, zk, expect_pubs):
    """input.json text -> proofs through zkfl_groth16_full_prove_json_batch: host worker threads
    parse the texts (the C parser) while earlier proofs run, the witness engine computes a
    slot-group of witnesses at a time straight into HBM, one group ahead of the slots that prove
    them; `steps` x `slots` proofs per rank, max-over-ranks time.  The parse of every text is
    inside the timed region.  Afterwards every proof goes through the GPU batch verifier against
    the public signals it returned, and those must equal the ones its input commits to
    (expect_pubs[i % clients], from the host witness images): `steps` slot-groups reuse the
    pipeline's three device witness sets, so a reuse race would show here."""
    n = steps * slots
    texts = [json_inputs[i % len(json_inputs)] for i in range(n)]
    key.full_prove_json_batch(wp, texts[:slots])   # warm slot buffers
    _barrier(ctx, dist)
    t0 = time.perf_counter()
    out = key.full_prove_json_batch(wp, texts)
    _barrier(ctx, dist)
    dt = _max_over_ranks(time.perf_counter() - t0, dist)
    assert len(out) == n
    for i, (_, pub) in enumerate(out):
        got = b"".join(x.to_bytes(32, "little") for x in pub)
        if got != expect_pubs[i % len(expect_pubs)]:
            raise SystemExit(f"end-to-end proof {i}: public signals differ from its input's witness")
    ok = _sum_over_ranks(verify_all(ctx, zk, [p for p, _ in out], lambda i: expect_pubs[i % len(expect_pubs)]), dist)
    world = dist.get_world_size() if dist is not None else 1
    if ok != world * n:
        raise SystemExit(f"end-to-end: {world * n - ok} proofs do not verify")
    return {"value": round(world * n / dt, 3), "unit": "proofs/s", "proofs": world * n, "verified": ok,
            "path": "input.json texts -> C parse (host worker threads, overlapped) -> GPU witnesses a slot-group "
                    "at a time, one group ahead -> GPU proofs (zkfl_groth16_full_prove_json_batch)"}


def latency_leg(key, ws, n=24):
    """One proof alone, as the CLI's `groth16 prove` and the API's prove run it: a batch of one takes
    the low-latency schedule (csrc/zkfl.hip enqueue_proof_lowlat: B2 and the A/B1 tails + the
    s pi_A + r B1 multiplications on side streams beside ABC / NTT / C + H).  Host wall clock of
    prove_batch([w]) -- witness resident, from the call to the proof bytes in host memory --, n
    times after a warm-up call: median, spread and the verdict's <= 4.5 ms target."""
    import statistics
    # one slot, as a CLI process holds (idle slots measured no effect: 4.12 vs 4.13 ms with 20 / 1,
    # profiles/r04_ab_latency_slots.log)
    slots = getattr(key, "slots", None)
    key.set_slots(1)
    key.prove_batch(ws[:1])
    ts = []
    for i in range(n):
        t = time.perf_counter()
        key.prove_batch([ws[i % len(ws)]])
        ts.append((time.perf_counter() - t) * 1e3)
    med = statistics.median(ts)
    if slots:
        key.set_slots(slots)
    return {"median_ms": round(med, 3), "min_ms": round(min(ts), 3), "max_ms": round(max(ts), 3),
            "p90_ms": round(sorted(ts)[int(0.9 * (n - 1))], 3), "proofs": n,
            "path": "prove_batch of one resident witness on a one-slot key -> low-latency schedule (3 streams), "
                    "host wall clock"}


def roofline_pass(key, ctx, ws, slots, n=6, reps=3):
    """Per-kernel HIP-event timings with every kernel running alone (one slot, a proof's
    streams serialized onto one), after the timed region: the roofline's average launch time.
    `reps` passes of n proofs; the pass with the shortest summed proof time is kept -- the boxes
    show occasional ~10 ms stalls of a whole process (the latency leg's max), and one such stall
    inside a pass moved the mean G1 launch time 2x while its median stayed put."""
    key.set_slots(1)
    key.prove_batch(ws[:1])
    best = None
    for _ in range(reps):
        ctx.profile_reset()
        ctx.set_profiling(True, serialize=True)
        key.prove_batch([ws[i % len(ws)] for i in range(n)])
        ctx.set_profiling(False)
        prof = {k: ctx.profile(k) for k in PROFILED}
        if best is None or prof["prove"][0] < best["prove"][0]:
            best = prof
    ctx.profile_reset()
    key.set_slots(slots)
    return best, n


def _pmc_traffic(kernel, path=PMC_TRAFFIC):
    """HBM bytes per launch of `kernel` from a committed PMC summary (tools/pmc_attrib.py), used
    only when that summary was collected on a library built from the same sources as the one loaded
    now (its build_id == zkfl_build_id()).  -> (bytes or None, provenance note)"""
    from zkfl import native
    rel = os.path.relpath(path, ROOT)
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, f"no PMC summary ({rel})"
    if d.get("build_id") != native.build_id():
        return None, f"PMC summary is of build {d.get('build_id')}, not the loaded {native.build_id()}"
    for name, v in d.get("kernels", {}).items():
        if KERNEL_SYMBOL[kernel] in name:
            return v["traffic"], f"{rel}, build {d['build_id']}"
    return None, "kernel absent from the PMC summary"


def _measured_clock(kernel, path=SQ_COUNTERS):
    """(GHz, provenance) of `kernel`'s effective clock from a committed SQ/GRBM counter summary."""
    from zkfl import native
    rel = os.path.relpath(path, ROOT)
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, f"no counter summary ({rel})"
    for name, v in d.get("kernels", {}).items():
        if KERNEL_SYMBOL[kernel].replace("zkfl::", "") in name.replace("zkfl::", "") and v.get("clock_GHz"):
            same = d.get("build_id") == native.build_id()
            return v["clock_GHz"], (f"{rel} ({'this build' if same else 'build ' + str(d.get('build_id'))}"
                                    f", single-slot PMC run: GRBM_GUI_ACTIVE / 8 / kernel duration)")
    return None, "kernel absent from the counter summary"


def stage_times(prof, nprof):
    """Per-proof stage times of the serialized pass.  A stage with one timed region per proof
    (ntt, abc, assemble, prove) reports the MEDIAN over the proofs -- robust to the one proof whose
    region a clock change or a late launch stretched; the accumulations (several launches of
    different sizes per proof) report their summed time per proof."""
    out = {}
    for k, (tot, launches, _, med) in prof.items():
        if launches == nprof and med:
            out[k] = round(med, 3)
        else:
            out[k] = round(tot / max(1, nprof), 3)
    return out


def roofline(prof, key, traffic=True, nprof=1, pmc_path=PMC_TRAFFIC, sq_path=SQ_COUNTERS):
    """The dominant kernel's roofline; pmc_path / sq_path: the counter summaries of
    this key's one-slot runs (the metric key's by default)."""
    cand = {k: v for k, v in prof.items() if k in IMPL_BYTES_PER_ENTRY and v[1] > 0}
    if not cand:
        return None
    dom = max(cand, key=lambda k: cand[k][0])
    ms_tot, launches, units, med_ms = prof[dom]
    # mean launch time: the launches of a proof differ in size (A, B1 and the merged C + H), so the
    # average query length below goes with the mean duration, not the median
    avg_s = ms_tot / launches / 1e3
    if dom == "msm_accumulate_g1":
        # a proof's G1 launches: A, B1, then C + H as one merged MSM (3 per proof; 4 -- A, B1, C,
        # H -- in a build without MSM_MERGE_CH): the average query length per launch
        per_proof = max(1, round(launches / max(1, nprof)))
        q = (2 * key.n_vars + (key.n_vars - key.n_public - 1) + key.domain_size) / per_proof
    else:
        per_proof = 1
        q = key.n_vars
    algo = q * ALGO_BYTES_PER_BASE[dom]
    entries = units / launches
    impl = entries * IMPL_BYTES_PER_ENTRY[dom]
    collect = traffic
    traffic, traffic_src = _pmc_traffic(dom, pmc_path) if collect else (None, "not collected for this leg")
    achieved = algo / avg_s / 1e9 if avg_s > 0 else 0.0
    fq = entries * FQMUL_PER_ENTRY[dom] / avg_s / 1e9 if avg_s > 0 else 0.0
    clk, clk_src = _measured_clock(dom, sq_path) if collect else (None, "not collected for this leg")
    peak_clk = FQMUL_PEAK_GPS * clk / 2.4 if clk else None
    # "bound" stays the roofline of record (north_star: HBM bandwidth fraction); "binding" names the
    # one that limits this kernel: the integer VALU issue rate (the "valu" object below)
    return {"bound": "hbm", "binding": "valu", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "algorithmic_bytes": round(algo), "query_length": round(q),
            "impl_bytes": round(impl), "impl_GBps": round(impl / avg_s / 1e9, 1) if avg_s > 0 else 0.0,
            "traffic_over_algorithmic": round(traffic / algo, 2) if traffic else None, "traffic_source": traffic_src,
            "avg_launch_ms": round(avg_s * 1e3, 4), "median_launch_ms": round(med_ms, 4),
            "launches": launches, "launches_per_proof": per_proof, "entries_per_launch": round(entries),
            "valu": {"achieved": round(fq, 2), "peak": round(FQMUL_PEAK_GPS, 1), "unit": "G Fq-mul/s",
                     "frac": round(fq / FQMUL_PEAK_GPS, 4),
                     "peak_basis": "ISA issue rates: 1024 SIMD x 32 lanes x 2.4 GHz / (162 mad x 2.2), 29-bit limbs",
                     "peak_32bit_limbs": round(FQMUL_PEAK_GPS_32, 1),
                     "measured_clock_GHz": clk, "peak_at_measured_clock": round(peak_clk, 1) if peak_clk else None,
                     "frac_at_measured_clock": round(fq / peak_clk, 4) if peak_clk else None,
                     "clock_source": clk_src}}


def c5_leg(ctx, rank, world, rounds, slots, dist, weak_rounds=0, check=True):
    """BASELINE config 5: federated rounds of 8 clients x {training sgd_verified(8,4,3), secure
    aggregation SecureMaskedUpdate(4,7)} (tests/full_system_simulation.mjs:1278-1343), both keys
    resident, input.json text -> C parse -> GPU witness -> proof through zkfl_groth16_full_prove_multi
    (the two circuits' proofs interleaved on the device).  Two measurements over the same keys:
      strong: `rounds` rounds in total, global proof k -> GPU k mod G;
      weak:   `weak_rounds` rounds of 8 clients per GPU (each rank its own clients, ids offset by
              8 x rank), so per-GPU work is fixed as G grows -- "batch-sharded across 8 MI355X".
    Every proof is GPU-verified afterwards (check=False: counted, not enforced -- knock-out probes
    only, tools/c5_probe.py --no-check).  -> (strong report, weak report or None) (rank 0)."""
    from zkfl import circuits, clients, groth16, native, wprog, zkey
    t0 = time.perf_counter()
    circ = {"train": circuits.build("sgd_verified", 8, 4, 3, 1000), "secagg": circuits.build("secure_masked_update", 4, 7)}
    keys, progs, images, vks = {}, {}, {}, {}
    for i, (nm, b) in enumerate(circ.items()):
        zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=0xC5 + i, alpha=3, beta=5, gamma=7, delta=11 + i))
        keys[nm] = native.ProvingKey(ctx, zk)
        keys[nm].set_slots(slots)
        images[nm] = wprog.compile_program(b)
        progs[nm] = native.WitnessProgram(ctx, images[nm])
        vks[nm] = groth16.vk_bytes(groth16.export_verification_key(zk, alphabeta=False))

    def jobs_of(nrounds, first_id):
        jobs = []          # (round, circuit, input.json text) in the reference's order: per client training, secagg
        for r in range(nrounds):
            for tr, sa, _ in clients.federated_round(8, rnd=r + 1, first_id=first_id):
                jobs += [(r, "train", json.dumps(tr)), (r, "secagg", json.dumps(sa))]
        return jobs

    def run(js):
        return ctx.full_prove_multi([(keys[nm], progs[nm], native.parse_inputs(images[nm], txt)) for _, nm, txt in js])

    def verified(js, out):
        ok = 0
        for nm in keys:
            sel = [o for (_, n2, _), o in zip(js, out) if n2 == nm]
            if sel:
                pubs = b"".join(x.to_bytes(32, "little") for _, pub in sel for x in pub)
                ok += sum(ctx.verify_batch(vks[nm], pubs, b"".join(p for p, _ in sel), keys[nm].n_public))
        return _sum_over_ranks(ok, dist)

    cpu = {}

    def timed(js, tag):
        # host CPU time of this process (every thread: the C parse workers, the launching thread,
        # the HIP runtime's) over the timed region, per proof proved here
        _barrier(ctx, dist)
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        t_start = time.perf_counter()
        out = run(js)
        _barrier(ctx, dist)
        dt = time.perf_counter() - t_start
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        busy = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
        cpu[tag] = {"host_cpu_ms_per_proof": round(busy * 1e3 / max(1, len(js)), 3),
                    "host_cpu_cores_busy": round(busy / dt, 2)}
        return _max_over_ranks(dt, dist), out

    all_jobs = jobs_of(rounds + 1, 1)                  # round 0 = warm-up
    mine = [j for k, j in enumerate([j for j in all_jobs if j[0] > 0]) if k % world == rank]
    warm = [j for k, j in enumerate([j for j in all_jobs if j[0] == 0]) if k % world == rank]
    log(f"[bench r{rank}] c5: keys for {[(nm, b.n_constraints) for nm, b in circ.items()]}, "
        f"{len(mine)} of {rounds * 16} proofs on this rank ({time.perf_counter() - t0:.1f} s)")
    run(warm)
    elapsed, out = timed(mine, "strong")
    ok = verified(mine, out)
    if check and ok != rounds * 16:
        raise SystemExit(f"[bench r{rank}] c5: {rounds * 16 - ok} proofs do not verify")
    workload = ("8 clients x {sgd_verified(8,4,3,1000) training, SecureMaskedUpdate(4,7) secagg} per round, "
                "input.json -> C parse -> GPU witness groups per key -> proof (zkfl_groth16_full_prove_multi, "
                "both keys resident)")
    strong = {"value": round(rounds * 16 / elapsed, 3), "unit": "proofs/s", "proofs": rounds * 16, "verified": ok,
              "rounds": rounds, "ms_per_round": round(elapsed / rounds * 1e3, 3), "scaling": "strong",
              "workload": workload + "; proof k -> GPU k mod G",
              "constraints": {nm: b.n_constraints for nm, b in circ.items()}, **cpu["strong"]}
    weak = None
    if weak_rounds:
        mine_w = jobs_of(weak_rounds, 1 + 8 * rank)     # this GPU's own 8 clients, every round
        elapsed_w, out_w = timed(mine_w, "weak")
        ok_w = verified(mine_w, out_w)
        total = world * weak_rounds * 16
        if check and ok_w != total:
            raise SystemExit(f"[bench r{rank}] c5 weak: {total - ok_w} proofs do not verify")
        weak = {"value": round(total / elapsed_w, 3), "unit": "proofs/s", "proofs": total, "verified": ok_w,
                "rounds_per_gpu": weak_rounds, "clients_per_gpu": 8, "scaling": "weak",
                "ms_per_round": round(elapsed_w / weak_rounds * 1e3, 3), **cpu["weak"],
                "workload": workload + "; 8 clients per GPU (ids 8 x rank + 1..8), every GPU proves its own rounds"}
    for x in list(progs.values()) + list(keys.values()):
        x.close()
    return strong, weak


def extra_circuit_leg(ctx, rank, world, circuit, steps, slots, dist):
    """Throughput on another training-circuit size (default: M19, the 2^19 domain the Report's
    ~283 K-constraint N=128 circuit has under circom): same prover, same slots, every proof
    GPU-verified; stage times and the G1 roofline from a serialized pass.  -> report dict."""
    from zkfl import circuits, clients, native, wprog, zkey
    name, params = CIRCUITS[circuit]
    t0 = time.perf_counter()
    b = circuits.build(name, *params)
    batch, dim, depth, precision = params
    objs = [clients.Client(rank * 2 + c + 1, batch, dim, depth, clients.JsLcg(777 + c)).training_input(
        batch, precision, 100000000)[0] for c in range(2)]
    inputs = [wprog.input_bytes(b, x) for x in objs]
    zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=0x19, alpha=0xA1, beta=0xB2, gamma=0xC3, delta=0xD4))
    key = native.ProvingKey(ctx, zk)
    key.set_slots(slots)
    wp = native.WitnessProgram(ctx, wprog.compile_program(b))
    res = wp.compute_resident(key, inputs)
    wts = wp.compute(inputs)
    log(f"[bench r{rank}] {circuit}: {b.n_constraints} constraints, domain {key.domain_size} "
        f"(setup {time.perf_counter() - t0:.1f} s)")
    n = steps * slots
    elapsed, proofs, _ = timed_run(key, [res[i % 2] for i in range(slots)], [res[i % 2] for i in range(n)],
                                   draw_rs(n), ctx, dist)
    pubs = [w[76 + 32:76 + 32 * (1 + key.n_public)] for w in wts]
    ok = _sum_over_ranks(verify_all(ctx, zk, proofs, lambda i: pubs[i % 2]), dist)
    if ok != world * n:
        raise SystemExit(f"[bench r{rank}] {circuit}: {world * n - ok} proofs do not verify")
    prof, nprof = roofline_pass(key, ctx, res, slots)
    for r_ in res:
        r_.close()
    wp.close()
    rep = {"value": round(world * n / elapsed, 3), "unit": "proofs/s", "proofs": world * n, "verified": ok,
           "workload": f"groth16 prove, {name}{params} (BATCH,DIM,DEPTH,PRECISION)",
           "constraints": b.n_constraints, "domain": key.domain_size, "ms_per_step": round(elapsed / steps * 1e3, 3),
           "stage_ms_isolated_per_proof": stage_times(prof, nprof),
           "roofline_g1": roofline({k: v for k, v in prof.items() if k == "msm_accumulate_g1"}, key,
                                   traffic=circuit == "M19", nprof=nprof, pmc_path=PMC_TRAFFIC_M19,
                                   sq_path=SQ_COUNTERS_M19)}
    key.close()
    return rep


POS_RP = (56, 57, 56, 60, 60, 63, 64, 63, 60, 66, 60, 65, 70, 60, 64, 68)     # circomlib R_P, t = 2..17
MAC_PEAK_PER_S = 1024 * 32 * 2.4e9 / (2.2 + 1.8)   # v_mad_u64_u32 + v_addc pairs/s (ISA issue rates)


def split_leg(ctx, rank, world, zk, wts, full_key, dist, n=8, warm=2):
    """One proof split over ALL ranks (optional row; zkfl/split.py): every rank loads
    shard `rank` of the key and the same witnesses `wts`, proves its share of each proof's MSMs, the
    parts are all-gathered and rank 0 assembles.  Proofs are issued one at a time, so this is LATENCY: ms per proof from
    rank 0's (r, s) broadcast to its assembled proof, against rank 0's unsplit proof on one GPU
    (same key, one proof in flight).  Every split proof is GPU-verified and equals the unsplit proof
    of the same (r, s)."""
    from zkfl import native, split
    key = native.ProvingKey(ctx, zk, shard=rank, n_shards=world)
    ws = [key.upload(w) for w in wts[:2]]
    grp = dist.group.WORLD if dist is not None else None
    lat, proofs = [], []
    rs_all = draw_rs(warm + n)  # read on rank 0 only (split_prove broadcasts the root's)
    for i in range(warm + n):
        _barrier(ctx, dist)
        t0 = time.perf_counter()
        out = split.split_prove(lambda r: key.prove_part_batch([ws[i % len(ws)]], r),
                                lambda parts, k, r: ctx.assemble(parts, k, r), 1, rs_all[64 * i:64 * i + 64], grp)
        t1 = time.perf_counter()
        if i >= warm and rank == 0:
            lat.append((t1 - t0) * 1e3)
            proofs.append(out[0])
    for w in ws:
        w.close()
    key.close()
    res = None
    if rank == 0:
        # the unsplit baseline: same witnesses, one proof in flight on the full key
        fws = [full_key.upload(w) for w in wts[:2]]
        one, same = [], 0
        for i in range(warm + n):
            t0 = time.perf_counter()
            p = full_key.prove_batch([fws[i % 2]], rs_all[64 * i:64 * i + 64])
            if i >= warm:
                one.append((time.perf_counter() - t0) * 1e3)
                same += p[0] == proofs[i - warm]
        for w in fws:
            w.close()
        pubs = [w[76 + 32:76 + 32 * (1 + full_key.n_public)] for w in wts[:2]]
        verified = verify_all(ctx, zk, proofs, lambda i: pubs[(i + warm) % 2])
        lat.sort()
        one.sort()
        res = {"gpus": world, "proofs": n, "verified": verified, "equal_to_unsplit": same,
               "ms_per_proof_median": round(lat[n // 2], 3),
               "ms_per_proof_min": round(lat[0], 3), "single_gpu_ms_median": round(one[n // 2], 3),
               "speedup": round(one[n // 2] / lat[n // 2], 3),
               "path": "shard k of G: base i of each query with i % G == k (zkfl_zkey_load_shard) -> ABC + NTT "
                       "(whole) + this shard's MSMs -> 768 B part (XYZZ, no inversion) -> all_gather (gloo) -> rank 0: parts summed "
                       "+ assembly on the GPU (zkfl_groth16_assemble)",
               "exchange_bytes_per_rank": 768}
        if verified != n or same != n:
            raise SystemExit(f"[bench] split proofs: {verified}/{n} verify, {same}/{n} equal the unsplit proof")
    return res


def pos_macs(t):
    """Multiply-add pairs of one csrc/poseidon.h permutation of width t: S-boxes are 3 Montgomery
    products (128 pairs each); an MDS row is groups of <= 5 products with one reduction (64 per
    product + 64); every round applies t rows except the last (row 0 only)."""
    rp = POS_RP[t - 2]
    sbox = 3 * 128 * (8 * t + rp)
    row = sum(64 * g + 64 for g in [5] * (t // 5) + ([t % 5] if t % 5 else []))
    return sbox + row * ((8 + rp - 1) * t + 1)


def merkle_leg(ctx, rank, log2n=20, ln=5):
    """computeDatasetCommitment (tests/full_system_simulation.mjs:309-335) on the GPU
    for 2^log2n samples of `ln` values (DIM 4 features + label): vectorHash leaves (Poseidon t = ln+1)
    then the depth-log2n Poseidon(2) tree, zkfl_dataset_commit.  Reports hashes/s of the kernels
    (HIP events) and of the whole call (PCIe in and out included), the VALU roofline of the tree
    kernel, and checks sampled nodes against the host-side Python Poseidon.  -> dict"""
    import numpy as np
    n, depth = 1 << log2n, log2n
    raw = np.random.default_rng(rank).integers(0, 2**63, size=(n * ln, 4), dtype=np.uint64)
    raw[:, 3] &= np.uint64((1 << 60) - 1)        # < 2^252 < r
    values = raw.tobytes()
    ctx.dataset_commit_raw(values[:32 * ln * 1024], 1024, ln, 10)        # tables + warm-up
    ctx.profile_reset()
    ctx.set_profiling(True)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        tree = ctx.dataset_commit_raw(values, n, ln, depth)
    dt = (time.perf_counter() - t0) / reps
    ctx.set_profiling(False)
    vh_ms, _, vh_units, vh_med = ctx.profile("vector_hash")
    mk_ms, _, mk_units, mk_med = ctx.profile("merkle")
    ctx.profile_reset()
    from zkfl.clients import vector_hash       # the host-side Python Poseidon (zkfl/field.py)
    from zkfl.field import poseidon_hash
    node = lambda lvl, j: int.from_bytes(tree[32 * ((2 << depth) - (2 << (depth - lvl)) + j):][:32], "little")  # noqa: E731
    val = lambda i, k: int.from_bytes(values[32 * (i * ln + k):][:32], "little")  # noqa: E731
    rnd = np.random.default_rng(7)
    for i in [0, n - 1] + [int(x) for x in rnd.integers(0, n, 3)]:
        assert node(0, i) == vector_hash([val(i, k) for k in range(ln)]), "leaf"
    for lvl in range(1, depth + 1):
        j = int(rnd.integers(0, 1 << (depth - lvl)))
        assert node(lvl, j) == poseidon_hash([node(lvl - 1, 2 * j), node(lvl - 1, 2 * j + 1)]), "node"
    hashes = n + (n - 1)
    mk_s = mk_med / 1e3
    achieved_macs = (n - 1) * pos_macs(3) / mk_s
    return {"samples": n, "values_per_sample": ln, "depth": depth, "hashes": hashes,
            "kernel_hashes_per_s": round(hashes / ((vh_med + mk_med) / 1e3)),
            "call_hashes_per_s": round(hashes / dt), "call_ms": round(dt * 1e3, 3),
            "vector_hash_ms": round(vh_med, 3), "tree_ms": round(mk_med, 3),
            "tree_roofline": {"bound": "valu", "achieved": round(achieved_macs / 1e12, 3),
                              "peak": round(MAC_PEAK_PER_S / 1e12, 3), "unit": "T mad+addc pairs/s",
                              "frac": round(achieved_macs / MAC_PEAK_PER_S, 4),
                              "per_hash_pairs": pos_macs(3),
                              "hbm_bytes_per_hash": 96, "hbm_GBps": round((n - 1) * 96 / mk_s / 1e9, 2)},
            "path": "zkfl_dataset_commit: values (host) -> vectorHash leaves -> Poseidon(2) levels -> padded tree (host)",
            "checked": "sampled leaves and one node per level == host Poseidon (zkfl/field.py)"}


def _barrier(ctx, dist):
    ctx.synchronize()
    if dist is not None:
        dist.barrier()


def _max_over_ranks(x, dist):
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sum_over_ranks(x, dist):
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


class KeyInfo:
    """The proving-key sizes the roofline needs (kept after the key itself is freed)."""

    def __init__(self, n_vars, n_public, domain_size):
        self.n_vars, self.n_public, self.domain_size = n_vars, n_public, domain_size


def _distinct_over_ranks(device, dist):
    """Number of distinct GPUs the ranks run on (ranks may share a device in tests)."""
    if dist is None:
        return 1
    import torch
    t = torch.zeros(64, dtype=torch.int64)
    t[device % 64] = 1
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.sum().item())


def _cpulist(text):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def _gpu_topology():
    """Host CPUs local to every GPU of the node, in KFD order (= HIP's device order when nothing is
    hidden), from sysfs alone (no HIP call: this runs before the rank initializes the runtime).  KFD
    topology nodes with SIMDs are the GPUs; a node's PCI location gives
    /sys/bus/pci/devices/<bdf>/local_cpulist.  [] if unknown."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    gpus = []
    try:
        for node in sorted(os.listdir(base), key=int):
            props = {}
            for ln in open(os.path.join(base, node, "properties")):
                k, _, v = ln.partition(" ")
                props[k] = v.strip()
            if int(props.get("simd_count", "0")) <= 0:
                continue
            loc, dom = int(props.get("location_id", "0")), int(props.get("domain", "0"))
            bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1F:02x}.{loc & 7}"
            try:
                cpus = _cpulist(open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read())
            except OSError:
                cpus = []
            gpus.append(cpus)
    except (OSError, ValueError):
        return []
    return gpus


def _visible_gpus(n_all):
    """Indices (into the node's GPUs) this process sees, from ROCR_VISIBLE_DEVICES then
    HIP_VISIBLE_DEVICES (numeric lists; HIP's list indexes what ROCr left visible); None if neither
    is set, [] if a list does not parse."""
    idx = None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        sel = os.environ.get(var)
        if sel:
            base = idx if idx is not None else list(range(n_all))
            try:
                idx = [base[int(x)] for x in sel.split(",") if x.strip()]
            except (ValueError, IndexError):
                return []
    return idx


def pin_host_cores(local_rank, local_world, topo=None, allowed=None, apply=True):
    """With several ranks on one node, pins this rank (before its first HIP call) to the host cores
    local to its GPU, shared evenly with the other ranks whose GPUs hang off the same cores; when
    the topology is unknown or leaves too few allowed cores, to an even 1/local_world share of the
    allowed cores.  The config-5 legs parse input.json and launch ~50 kernels per proof on host
    threads (0.6-0.9 ms of host CPU per proof, ~1.2-1.8 cores per rank), so 8 unpinned ranks
    compete for the same cores and cross NUMA nodes.  One rank alone is left unpinned.
    ZKFL_PIN=0 disables it.  Which GPU is this rank's: local rank r drives device r of what it sees
    (bench.py: `local_rank % n_dev`); when a launcher gives each rank ONE visible GPU
    (ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES = its index), that GPU, and the peers are counted
    on the node's whole topology with rank r on node GPU r.  topo / allowed / apply: the node's GPU
    topology, the allowed cores and whether to set the affinity (tests fake an 8-GPU node).
    Returns what was done (reported per rank in the bench line)."""
    allowed = sorted(allowed if allowed is not None else os.sched_getaffinity(0))
    info = {"allowed_cpus": len(allowed), "pinned": False, "cpus": len(allowed), "source": "none"}
    if local_world <= 1 or os.environ.get("ZKFL_PIN", "1") == "0":
        return info
    node = topo if topo is not None else _gpu_topology()
    sel = _visible_gpus(len(node)) if node else None
    if node and sel is not None and len(sel) == 1:
        gpu_of = [node[r % len(node)] for r in range(local_world)]   # rank r on node GPU r
        mine = node[sel[0]]
    else:
        seen = [node[i] for i in sel] if (node and sel) else ([] if sel == [] else node)
        gpu_of = [seen[r % len(seen)] for r in range(local_world)] if seen else []
        mine = gpu_of[local_rank] if seen else None
    share, source = None, "even split of the allowed cores"
    if mine is not None:
        pool = [c for c in allowed if c in set(mine)]
        peers = [r for r in range(local_world) if gpu_of[r] == mine]
        if local_rank not in peers:
            peers = sorted(peers + [local_rank])
        n, k = len(peers), peers.index(local_rank)
        if len(pool) >= max(2, len(allowed) // (2 * local_world)) * n:
            share = pool[k * len(pool) // n:(k + 1) * len(pool) // n]
            source = f"GPU-local cores ({len(pool)} allowed, {n} ranks on them)"
    if not share:
        n = len(allowed)
        share = allowed[local_rank * n // local_world:(local_rank + 1) * n // local_world] or allowed
    if apply:
        os.sched_setaffinity(0, share)
    info.update(pinned=True, cpus=len(share), source=source, share=share if not apply else None,
                cpulist=f"{share[0]}-{share[-1]}" if share == list(range(share[0], share[-1] + 1))
                else ",".join(map(str, share)))
    if apply:
        del info["share"]
    return info


def host_report(rank, device, dist, pin, cpu):
    """Per-rank host facts for the line: the node's CPUs, each rank's pinning and host CPU per
    proof of the timed legs (`cpu`: leg -> ms per proof), gathered to rank 0 (gloo)."""
    mine = {"rank": rank, "device": device, "pin": pin, "host_cpu_ms_per_proof": cpu}
    ranks = [mine]
    if dist is not None:
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, mine)
    return {"node_cpus": os.cpu_count(), "ranks": ranks}


def launch_ranks(n):
    """bench.py --gpus N without a launcher: N child processes of this script, one per GPU, with
    the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT).
    Called before any HIP call in this process; rank 0's JSON line is the children's stdout.
    Returns the first non-zero exit status (the others are then terminated)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code and not rc:
                rc = code
                for q in pending:
                    q.terminate()
        time.sleep(0.2)
    return rc


def report(args, world, elapsed, n_timed_all, verified_all, prof, nprof, key, config, extra):
    """The bench JSON line (rank 0).  `extra`: roofline / end_to_end / c5 / cpu_baseline fields."""
    stage_ms = stage_times(prof, nprof)
    line = {
        "metric": METRIC, "value": round(n_timed_all / elapsed, 4), "unit": "proofs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (reference harness seeded client generator)",
        "config": config, "proofs_timed": n_timed_all, "verified": verified_all,
        "roofline": roofline(prof, key, nprof=nprof) if key is not None else None,
        "stage_ms_isolated_per_proof": stage_ms,
    }
    line.update(extra)
    # whole-proof VALU efficiency: every accumulated MSM entry of a proof (G1: 10 Fq products, G2:
    # 30) at the timed throughput, against the same ISA ceiling -- the accumulations' share of the
    # chip's multiply issue, with every other stage (sort, stitching, reduction, NTT, ABC, assembly)
    # counted as overhead
    if line.get("roofline") and nprof:
        fq = sum(prof[k][2] / nprof * FQMUL_PER_ENTRY[k] for k in FQMUL_PER_ENTRY if k in prof)
        achieved = fq * line["value"] / 1e9
        clk = line["roofline"]["valu"].get("measured_clock_GHz")
        line["roofline"]["whole_proof_valu"] = {
            "fq_mul_equivalents_per_proof": round(fq), "achieved": round(achieved, 2), "unit": "G Fq-mul/s",
            "frac": round(achieved / FQMUL_PEAK_GPS, 4),
            "frac_at_measured_clock": round(achieved / (FQMUL_PEAK_GPS * clk / 2.4), 4) if clk else None}
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16, help="timed steps (one step = --slots proofs)")
    ap.add_argument("--warmup", type=int, default=2, help="untimed steps")
    ap.add_argument("--circuit", default="M", choices=sorted(CIRCUITS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--slots", type=int, default=20, help="proofs in flight per GPU (one HIP stream each)")
    ap.add_argument("--clients", type=int, default=4, help="distinct synthetic client witnesses, cycled")
    ap.add_argument("--e2e-steps", type=int, default=16, help="steps of the input.json -> proof leg (0: skip)")
    # 16 rounds: at 8 (~75 ms timed) the first round's ramp (slots filling, the first witness group)
    # weighed 1/8 -- bench 1751-1828 against 1900-1915 from tools/c5_probe.py's 16 rounds, same box
    ap.add_argument("--c5-rounds", type=int, default=16, help="federated rounds of the config-5 leg (0: skip)")
    ap.add_argument("--c5-weak-rounds", type=int, default=16,
                    help="config-5 weak-scaling leg: federated rounds of 8 own clients per GPU (0: skip)")
    ap.add_argument("--merkle-log2n", type=int, default=20, help="dataset-commitment leg: 2^k samples (0: skip)")
    ap.add_argument("--extra-circuit", default="M19", help="second training-circuit size leg ('' or none: skip)")
    ap.add_argument("--extra-steps", type=int, default=16,
                    help="timed steps of the extra-circuit leg (16 x 20 proofs: over 1 s, VERDICT r3)")
    ap.add_argument("--c5-slots", type=int, default=8, help="proof slots per key in the config-5 legs")
    # off by default: the split proof is dominated by one GPU's latency schedule (the
    # Amdahl bound at G = 8 is above one proof alone), and the leg loads a second (shard) key
    ap.add_argument("--split-proofs", type=int, default=0,
                    help="split-proof leg: proofs, one at a time, each split over all ranks (0: skip)")
    ap.add_argument("--cli-runs", type=int, default=5,
                    help="cli_prove leg: `npx snarkjs groth16 prove` invocations per circuit (0: skip; 1 GPU only)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no outside launcher: start one process per GPU here, before anything touches HIP
        return launch_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU "
                         "(or drop the launcher and let bench.py start them)")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    pin = pin_host_cores(local_rank, int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))  # before any HIP call
    from zkfl import circuits, clients, native, wprog, zkey
    # libzkfl (and with it /opt/rocm's HIP runtime) is loaded before torch, whose wheel carries its
    # own libamdhip64 under the same soname: one HIP runtime per process.  torch.distributed is the
    # control plane only (barrier, max-over-ranks time, counts) over gloo; the proofs of different
    # ranks are independent, there is no collective on the data path.
    native.lib()
    n_dev = native.device_count()
    dist = None
    if world > 1:
        import torch.distributed as dist_mod
        dist = dist_mod
        dist.init_process_group(backend="gloo")
    device = local_rank % max(1, n_dev)     # ranks beyond the device count share devices (tests)
    devices_used = _distinct_over_ranks(device, dist)
    build_id, source_id = native.build_id(), native.source_id()
    if build_id != source_id:
        log(f"[bench r{rank}] WARNING: libzkfl.so build {build_id} is not this tree's sources ({source_id})")

    name, params = CIRCUITS[args.circuit]
    t0 = time.perf_counter()
    b = circuits.build(name, *params)
    batch, dim, depth, precision = params
    input_objs = []
    for c in range(args.clients):
        client = clients.Client(rank * args.clients + c + 1, batch, dim, depth, clients.JsLcg(12345 + c))
        input_objs.append(client.training_input(batch, precision, 100000000)[0])
    inputs = [wprog.input_bytes(b, x) for x in input_objs]
    log(f"[bench r{rank}] circuit {name}{params}: {b.n_constraints} constraints, {b.n_wires} wires "
        f"({time.perf_counter() - t0:.1f} s); device {device} of {n_dev}")

    ctx = native.Context(device)
    t0 = time.perf_counter()
    zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=0x5EED, alpha=0xA1, beta=0xB2, gamma=0xC3, delta=0xD4))
    log(f"[bench r{rank}] dev setup {len(zk) / 1e6:.0f} MB zkey ({time.perf_counter() - t0:.1f} s)")
    # config 5 first, with only its own two keys on the device: the main key's slots (20 streams and
    # their scratch) stay out of its way (the same c5 code read 1894 proofs/s alone and 1440 after
    # the main legs on one box, round 4)
    c5 = c5w = None
    if args.c5_rounds:
        c5, c5w = c5_leg(ctx, rank, world, args.c5_rounds, args.c5_slots, dist, args.c5_weak_rounds)
        log(f"[bench r{rank}] config 5: {c5}; weak: {c5w}")
    t0 = time.perf_counter()
    key = native.ProvingKey(ctx, zk)
    key.set_slots(args.slots)
    wp = native.WitnessProgram(ctx, wprog.compile_program(b))
    log(f"[bench r{rank}] key + witness program load ({time.perf_counter() - t0:.1f} s), domain {key.domain_size}, "
        f"slots {args.slots}")
    t0 = time.perf_counter()
    res = wp.compute_resident(key, inputs)      # GPU witness generation straight into HBM
    log(f"[bench r{rank}] {len(res)} client witnesses on the GPU ({(time.perf_counter() - t0) * 1e3:.1f} ms)")
    wts = wp.compute(inputs)                    # host .wtns images: public signals + the oracle check
    n_timed = args.steps * args.slots
    steps_w = [res[i % len(res)] for i in range(n_timed)]
    warm_w = [res[i % len(res)] for i in range(args.warmup * args.slots)]
    rs = draw_rs(n_timed)

    # one proof alone first, on the idle chip a CLI invocation meets (measured after the 20-slot
    # run it read 4.49 / 4.64 ms on two boxes, against 4.06-4.22 ms for tools/ko_probe.py --latency
    # on a fresh process on others)
    lat = latency_leg(key, res)
    log(f"[bench r{rank}] one proof alone: {lat}")
    elapsed, proofs, busy = timed_run(key, warm_w, steps_w, rs, ctx, dist)
    host_cpu = {"main": round(busy * 1e3 / n_timed, 3)}
    assert len(proofs) == n_timed and all(len(p) == 256 for p in proofs)
    pubs = [w[76 + 32:76 + 32 * (1 + key.n_public)] for w in wts]   # wtns v2: header 76 B, wire 0 = 1
    verified = verify_all(ctx, zk, proofs, lambda i: pubs[i % len(pubs)])
    log(f"[bench r{rank}] {n_timed} proofs in {elapsed:.3f} s; GPU batch verifier: {verified}/{n_timed} valid")
    verified_all = _sum_over_ranks(verified, dist)
    if verified_all != n_timed * world:
        raise SystemExit(f"[bench r{rank}] {n_timed * world - verified_all} timed proofs do not verify")
    prof, nprof = roofline_pass(key, ctx, res, args.slots)
    kinfo = KeyInfo(key.n_vars, key.n_public, key.domain_size)
    e2e = None
    if args.e2e_steps:
        e2e = end_to_end_leg(key, wp, wprog.compile_program(b), [json.dumps(x) for x in input_objs], args.slots,
                             args.e2e_steps, ctx, dist, zk, pubs)
        log(f"[bench r{rank}] end to end: {e2e}")
    split_wts = None
    if args.split_proofs:
        # every shard of a split proof needs the SAME witness: rank 0's first two clients on all ranks
        common = [wprog.input_bytes(b, clients.Client(c + 1, batch, dim, depth, clients.JsLcg(12345 + c))
                                    .training_input(batch, precision, 100000000)[0]) for c in range(2)]
        split_wts = wp.compute(common) if world > 1 else wts[:2]
    for r_ in res:
        r_.close()
    wp.close()
    key.set_slots(1)
    extra = None
    if args.extra_circuit and args.extra_circuit != "none" and args.extra_circuit != args.circuit:
        extra = extra_circuit_leg(ctx, rank, world, args.extra_circuit, args.extra_steps, args.slots, dist)
        log(f"[bench r{rank}] {args.extra_circuit}: {extra}")
    merkle = None
    if args.merkle_log2n:
        merkle = merkle_leg(ctx, rank, args.merkle_log2n)
        log(f"[bench r{rank}] dataset commitment: {merkle}")
    split_res = {"skipped": "off by default (--split-proofs N runs it): one proof split over the ranks is bounded "
                            "by one GPU's latency schedule (DESIGN.md §7)"}
    if args.split_proofs:  # last: the other legs never run beside a second (shard) key
        split_res = split_leg(ctx, rank, world, zk, split_wts, key, dist, args.split_proofs)
        log(f"[bench r{rank}] split proof: {split_res}")
    for tag, leg in (("c5", c5), ("c5_weak", c5w)):
        if leg:
            host_cpu[tag] = leg["host_cpu_ms_per_proof"]
    host = host_report(rank, device, dist, pin, host_cpu)   # collective: every rank
    cli = None
    if args.cli_runs and world == 1:
        try:
            cli = cli_leg(ctx, args.cli_runs)
        except Exception as e:  # noqa: BLE001
            cli = {"error": str(e)[-300:]}
        log(f"[bench r{rank}] cli prove: {cli}")
    if rank == 0:
        cpu, oracle_match = None, None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu, ref = cpu_baseline_leg(zk, wts[0], rs[:64])
                oracle_match = ref == proofs[0]
                cpu["oracle_check"] = "timed proof 0 == C oracle proof (same zkey, wtns, r, s)" if oracle_match \
                    else "MISMATCH: timed proof 0 differs from the C oracle"
            except Exception as e:  # noqa: BLE001
                log(f"[bench] cpu baseline failed: {e}")
        config = {"workload": f"groth16 prove, {name}{params} (BATCH,DIM,DEPTH,PRECISION)",
                  "constraints": b.n_constraints, "wires": b.n_wires, "domain": kinfo.domain_size,
                  "global_batch": args.slots * world, "step": f"{args.slots} proofs per GPU (one per slot)",
                  "parallelism": f"replicas{world}", "slots_in_flight": args.slots,
                  "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))}
        line = report(args, world, elapsed, n_timed * world, verified_all, prof, nprof, kinfo, config,
                      {"n_gpus": devices_used, "ranks": world, "build_id": build_id,
                       "build_matches_sources": build_id == source_id, "oracle_match": oracle_match,
                       "end_to_end": e2e, "c5": c5, "c5_weak": c5w, "extra_circuit": extra,
                       "latency_single_proof": lat, "dataset_commit": merkle, "split_proof": split_res,
                       "cli_prove": cli, "cpu_baseline": cpu, "host": host})
        print(json.dumps(line), flush=True)
        if oracle_match is False:
            raise SystemExit("[bench] timed proof 0 differs from the C oracle")
    if key is not None:
        key.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
