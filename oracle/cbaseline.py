"""ctypes wrapper of the C oracle (oracle/c/groth16_ref.c) — TEST INFRASTRUCTURE ONLY.

Used by tests/ as the M-scale checker and by bench.py's cpu_baseline leg (kind "port")."""
from __future__ import annotations

import ctypes as C
import os
import time

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libgroth16_ref.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            raise RuntimeError(f"{_LIB} not built (make -C oracle)")
        L = C.CDLL(_LIB)
        L.ref_prove.restype = C.c_int
        L.ref_prove.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p,
                                C.POINTER(C.c_uint8), C.c_int]
        L.ref_prove_ex.restype = C.c_int
        L.ref_prove_ex.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p,
                                   C.POINTER(C.c_uint8), C.c_int, C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)]
        L.ref_msm_g1.restype = C.c_int
        L.ref_msm_g1.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_uint8), C.c_int]
        for nm in ("ref_g1_gen_mul", "ref_g2_gen_mul"):
            f = getattr(L, nm)
            f.restype = C.c_int
            f.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_uint8), C.c_int]
        _lib = L
    return _lib


def prove(zkey: bytes, wtns: bytes, rs: bytes, threads: int = 0) -> bytes:
    out = (C.c_uint8 * 256)()
    rc = lib().ref_prove(zkey, len(zkey), wtns, len(wtns), rs, out, threads)
    if rc:
        raise RuntimeError(f"ref_prove failed: {rc}")
    return bytes(out)


def prove_parts(zkey: bytes, wtns: bytes, rs: bytes, domain_size: int, threads: int = 0):
    """-> (proof 256 B, h list of ints, dict A/B1/B2/C/H of std affine bytes): the layout of
    zkfl_debug_prove_parts (include/zkfl.h), for the GPU parity tests at the metric size."""
    out = (C.c_uint8 * 256)()
    h = (C.c_uint8 * (32 * domain_size))()
    m = (C.c_uint8 * 384)()
    rc = lib().ref_prove_ex(zkey, len(zkey), wtns, len(wtns), rs, out, threads, h, m)
    if rc:
        raise RuntimeError(f"ref_prove_ex failed: {rc}")
    hb, mb = bytes(h), bytes(m)
    hs = [int.from_bytes(hb[32 * i:32 * i + 32], "little") for i in range(domain_size)]
    return bytes(out), hs, dict(A=mb[0:64], B1=mb[64:128], B2=mb[128:256], C=mb[256:320], H=mb[320:384])


def msm_g1(bases: bytes, scalars: bytes, threads: int = 0) -> bytes:
    out = (C.c_uint8 * 64)()
    lib().ref_msm_g1(bases, scalars, len(scalars) // 32, out, threads)
    return bytes(out)


def _cgroup_quota_cores():
    """The CPU time this process may use, in cores, from cgroup v2's cpu.max ("quota period"):
    None when unlimited or unknown.  The GPU boxes expose all 256 node CPUs in the affinity mask
    but cap a one-GPU job at 16 cores of CPU time this way."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q == "max":
            return None
        return max(1, int(q) // int(p))
    except (OSError, ValueError):
        return None


def host_cores() -> dict:
    """The host's cores as this process sees them: the affinity mask, the cgroup CPU quota, the node."""
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count() or 1
    return {"allowed_cpus": allowed, "cgroup_quota_cores": _cgroup_quota_cores(), "node_cpus": os.cpu_count()}


def default_threads() -> int:
    """Every core the job may use: the allowed CPUs, capped by the cgroup CPU quota when there is
    one (more OpenMP threads than the quota only get throttled).  No fixed cap."""
    h = host_cores()
    q = h["cgroup_quota_cores"]
    return max(1, min(h["allowed_cpus"], q) if q else h["allowed_cpus"])


def time_prove(zkey: bytes, wtns: bytes, seconds_budget: float = 20.0, rs: bytes | None = None):
    """cpu_baseline leg: full proofs of the same zkey/wtns on the job's host cores (default_threads)
    until ~2/3 of the budget, then at half the threads for the rest (the scaling between the two
    gives the node-share extrapolation, labelled as such).  -> (report dict, the proof bytes) --
    bench.py compares the proof with the GPU's for the same rs."""
    threads = default_threads()
    host = host_cores()
    rs = rs or (12345).to_bytes(32, "little") + (67890).to_bytes(32, "little")

    def run(th, budget, kmax):
        t0 = time.perf_counter()
        k = 0
        while True:
            proof = prove(zkey, wtns, rs, th)
            k += 1
            dt = time.perf_counter() - t0
            if dt * (k + 1) / k > budget or k >= kmax:
                return k / dt, k, dt, proof
    rate, k, dt, proof = run(threads, seconds_budget * 2 / 3, 8)
    rep = {"value": round(rate, 5), "unit": "proofs/s", "cores": threads, "kind": "port",
           "sample": f"{k} full proof(s) of the same zkey/wtns by the C oracle "
                     f"(oracle/c/groth16_ref.c, OpenMP {threads} threads) in {dt:.1f} s",
           "host": host}
    if threads >= 2:
        half = threads // 2
        rate_h, kh, dth, _ = run(half, seconds_budget / 3, 4)
        eff = rate / (2 * rate_h)      # parallel efficiency of the step half -> all threads
        share = host["allowed_cpus"] // 8 if host["allowed_cpus"] >= 16 else None
        rep["scaling"] = {"threads": [half, threads], "proofs_per_s": [round(rate_h, 5), round(rate, 5)],
                          "efficiency_doubling": round(eff, 3)}
        if share and share > threads:
            # NOT measured: the job's quota stops at `threads`; linear in cores at the measured
            # doubling efficiency, per doubling
            import math
            est = rate * eff ** math.log2(share / threads) * share / threads
            rep["node_gpu_share_extrapolation"] = {
                "cores": share, "value": round(est, 5),
                "basis": f"allowed node CPUs / 8 GPUs; extrapolated from {threads} threads at the measured "
                         f"doubling efficiency {eff:.3f} (not measured: the job's cgroup quota is {threads} cores)"}
    return rep, proof


def g1_gen_mul(scalars: bytes, threads: int = 0) -> bytes:
    n = len(scalars) // 32
    out = (C.c_uint8 * max(1, 64 * n))()
    lib().ref_g1_gen_mul(scalars, n, out, threads)
    return bytes(out)[:64 * n]


def g2_gen_mul(scalars: bytes, threads: int = 0) -> bytes:
    n = len(scalars) // 32
    out = (C.c_uint8 * max(1, 128 * n))()
    lib().ref_g2_gen_mul(scalars, n, out, threads)
    return bytes(out)[:128 * n]
