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


def default_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", n))))


def time_prove(zkey: bytes, wtns: bytes, seconds_budget: float = 20.0, rs: bytes | None = None):
    """cpu_baseline leg: full proofs of the same zkey/wtns on the host until ~budget.
    -> (report dict, the proof bytes) — bench.py compares the proof with the GPU's for the same rs."""
    threads = default_threads()
    rs = rs or (12345).to_bytes(32, "little") + (67890).to_bytes(32, "little")
    t0 = time.perf_counter()
    k = 0
    while True:
        proof = prove(zkey, wtns, rs, threads)
        k += 1
        dt = time.perf_counter() - t0
        if dt * (k + 1) / k > seconds_budget or k >= 5:
            break
    return ({"value": round(k / dt, 5), "unit": "proofs/s", "cores": threads, "kind": "port",
             "sample": f"{k} full proof(s) of the same zkey/wtns by the C oracle "
                       f"(oracle/c/groth16_ref.c, OpenMP {threads} threads) in {dt:.1f} s"}, proof)


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
