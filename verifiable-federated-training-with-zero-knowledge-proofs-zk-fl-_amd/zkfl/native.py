"""ctypes binding of libzkfl.so (the C ABI declared in include/zkfl.h).

This is the Python twin of the N-API binding shown in INTEGRATION.md.  The library is built
in-tree (``make`` in the package directory, or ``__graft_entry__.build()``); if it is missing
every call raises ``ZkflError`` — there is no CPU fallback on the proving path.
"""

from __future__ import annotations

import ctypes as C
import os

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ZKFL_LIB: an alternative build of the library (A/B experiments); default the in-tree one
LIB_PATH = os.path.abspath(os.environ["ZKFL_LIB"]) if os.environ.get("ZKFL_LIB") else os.path.join(_PKG_DIR, "libzkfl.so")

ZKFL_OK = 0
# one shard's part of a split proof: A' | B1' | B2' | C' | H as XYZZ points (X, Y, ZZ, ZZZ), every
# coordinate std-form 32 B LE (G2: c0, c1); ZZ = 0 is infinity (include/zkfl.h)
PART_BYTES = 768
PART_LAYOUT = {"A": (0, 128), "B1": (128, 256), "B2": (256, 512), "C": (512, 640), "H": (640, 768)}
ERRORS = {
    -1: "ZKFL_E_ARG", -2: "ZKFL_E_FORMAT", -3: "ZKFL_E_PRIME", -4: "ZKFL_E_MISMATCH",
    -5: "ZKFL_E_DEVICE", -6: "ZKFL_E_OOM", -7: "ZKFL_E_CONSTRAINT",
}

# every exported symbol of include/zkfl.h with (restype, argtypes)
_P = C.c_void_p
_U8P = C.POINTER(C.c_uint8)
SIGNATURES = {
    "zkfl_version": (C.c_int, []),
    "zkfl_build_id": (C.c_char_p, []),
    "zkfl_last_error": (C.c_char_p, []),
    "zkfl_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "zkfl_ctx_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "zkfl_ctx_destroy": (C.c_int, [_P]),
    "zkfl_ctx_set_profiling": (C.c_int, [_P, C.c_int]),
    "zkfl_ctx_profile": (C.c_int, [_P, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "zkfl_ctx_profile_reset": (C.c_int, [_P]),
    "zkfl_ctx_synchronize": (C.c_int, [_P]),
    "zkfl_zkey_load": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    "zkfl_zkey_load_shard": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_uint32, C.c_uint32, C.POINTER(_P)]),
    "zkfl_zkey_file_open": (C.c_int, [C.c_char_p, C.POINTER(_P)]),
    "zkfl_zkey_load_file": (C.c_int, [_P, _P, C.POINTER(_P)]),
    "zkfl_zkey_file_close": (C.c_int, [_P]),
    "zkfl_key_shard": (C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "zkfl_groth16_prove_part_batch": (C.c_int, [_P, _P, C.c_size_t, C.POINTER(_P), C.c_char_p, _U8P]),
    "zkfl_groth16_assemble": (C.c_int, [_P, C.c_size_t, C.c_size_t, C.c_char_p, C.c_char_p, _U8P]),
    "zkfl_key_free": (C.c_int, [_P]),
    "zkfl_key_info": (C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "zkfl_key_set_slots": (C.c_int, [_P, C.c_int]),
    "zkfl_groth16_prove": (C.c_int, [_P, _P, C.c_char_p, C.c_size_t, C.c_char_p, _U8P, _U8P,
                                     C.POINTER(C.c_size_t)]),
    "zkfl_witness_upload": (C.c_int, [_P, _P, C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    "zkfl_witness_free": (C.c_int, [_P]),
    "zkfl_groth16_prove_resident": (C.c_int, [_P, _P, _P, C.c_char_p, _U8P]),
    "zkfl_groth16_prove_batch": (C.c_int, [_P, _P, C.c_size_t, C.POINTER(_P), C.c_char_p, _U8P]),
    "zkfl_debug_prove_parts": (C.c_int, [_P, _P, C.c_char_p, C.c_size_t, _U8P, _U8P]),
    "zkfl_debug_glv_split": (C.c_int, [C.c_char_p, _U8P]),
    "zkfl_debug_g1_glv_mul": (C.c_int, [_P, C.c_size_t, C.c_char_p, C.c_char_p, _U8P]),
    "zkfl_debug_wtrace": (C.c_int, [_P, C.c_int, C.c_uint32, _P, C.POINTER(C.c_uint32)]),
    "zkfl_msm_g1": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_size_t, _U8P]),
    "zkfl_msm_g2": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_size_t, _U8P]),
    "zkfl_ntt_coset": (C.c_int, [_P, _U8P, C.c_uint32]),
    "zkfl_setup_g1_gen_mul": (C.c_int, [_P, C.c_char_p, C.c_size_t, _U8P]),
    "zkfl_setup_g2_gen_mul": (C.c_int, [_P, C.c_char_p, C.c_size_t, _U8P]),
    "zkfl_setup_g1_scale": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_size_t, _U8P]),
    "zkfl_setup_g2_scale": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_size_t, _U8P]),
    "zkfl_setup_g1_lagrange": (C.c_int, [_P, C.c_char_p, C.c_uint32, _U8P]),
    "zkfl_setup_g2_lagrange": (C.c_int, [_P, C.c_char_p, C.c_uint32, _U8P]),
    "zkfl_setup_g1_lincomb": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_size_t, C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint32), C.c_char_p, _U8P]),
    "zkfl_setup_g2_lincomb": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_size_t, C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint32), C.c_char_p, _U8P]),
    "zkfl_groth16_verify": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p]),
    "zkfl_groth16_verify_batch": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_size_t, C.c_char_p, C.c_size_t,
                                            C.c_char_p, C.POINTER(C.c_int32)]),
    "zkfl_pairing": (C.c_int, [_P, C.c_size_t, C.c_char_p, C.c_char_p, _U8P]),
    "zkfl_debug_miller_loop": (C.c_int, [_P, C.c_size_t, C.c_char_p, C.c_char_p, _U8P]),
    "zkfl_wprog_load": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    "zkfl_wprog_free": (C.c_int, [_P]),
    "zkfl_wprog_info": (C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "zkfl_wtns_size": (C.c_size_t, [_P]),
    "zkfl_witness_compute": (C.c_int, [_P, _P, C.c_size_t, C.c_char_p, _U8P]),
    "zkfl_witness_compute_resident": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_char_p, C.POINTER(_P)]),
    "zkfl_wprog_parse_inputs": (C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, _U8P, C.c_size_t,
                                          C.POINTER(C.c_size_t)]),
    "zkfl_witness_compute_json": (C.c_int, [_P, _P, C.c_char_p, _U8P]),
    "zkfl_groth16_full_prove_batch": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_char_p, C.c_char_p, _U8P, _U8P]),
    "zkfl_poseidon_params": (C.c_int, [C.c_uint32, _U8P, _U8P, C.POINTER(C.c_uint32)]),
    "zkfl_poseidon_batch": (C.c_int, [_P, C.c_uint32, C.c_size_t, C.c_char_p, _U8P]),
    "zkfl_vector_hash_batch": (C.c_int, [_P, C.c_uint32, C.c_size_t, C.c_char_p, _U8P]),
    "zkfl_merkle_build": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_uint32, _U8P]),
    "zkfl_dataset_commit": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_uint32, C.c_uint32, _U8P]),
    "zkfl_groth16_full_prove_json": (C.c_int, [_P, _P, _P, C.c_char_p, C.c_char_p, _U8P, _U8P]),
    "zkfl_groth16_prove_multi": (C.c_int, [_P, C.c_size_t, C.POINTER(_P), C.POINTER(_P), C.c_char_p, _U8P]),
    "zkfl_groth16_full_prove_json_batch": (C.c_int, [_P, _P, _P, C.c_size_t, C.POINTER(C.c_char_p), C.c_char_p, _U8P,
                                                     _U8P]),
    "zkfl_groth16_full_prove_multi": (C.c_int, [_P, C.c_size_t, C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_char_p),
                                                C.c_char_p, _U8P, C.POINTER(_U8P)]),
}


class ZkflError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ZkflError(-5, f"{LIB_PATH} not built (run make in the package dir / __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        # an A/B build named by ZKFL_LIB (tools/ab.sh) may predate an entry point: bind what it has
        ab = bool(os.environ.get("ZKFL_LIB"))
        for name, (res, args) in SIGNATURES.items():
            if ab and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != ZKFL_OK:
        raise ZkflError(rc, lib().zkfl_last_error().decode(errors="replace"))


def _frs(values) -> bytes:
    return b"".join(int(v).to_bytes(32, "little") for v in values)


def _ints(b: bytes) -> list:
    return [int.from_bytes(b[i:i + 32], "little") for i in range(0, len(b), 32)]


def _levels(flat, depth):
    out, pos = [], 0
    for lvl in range(depth + 1):
        w = 1 << (depth - lvl)
        out.append(flat[pos:pos + w])
        pos += w
    return out


def poseidon_params(t: int):
    """Host only (no device): circomlib's raw constants for width t from the library's own Grain
    LFSR -> (round constants, x points, y points, R_P)."""
    c = _buf(32 * (8 + 70) * t)     # R_P <= 70 for t <= 17
    xy = _buf(64 * t)
    rp = C.c_uint32()
    check(lib().zkfl_poseidon_params(t, c, xy, C.byref(rp)))
    consts = _ints(bytes(c))[:(8 + rp.value) * t]
    pts = _ints(bytes(xy))
    return consts, pts[:t], pts[t:], rp.value


def build_id() -> str:
    """The loaded library's source hash (zkfl_build_id, set by the package Makefile)."""
    return lib().zkfl_build_id().decode()


def source_id(pkg_dir: str = _PKG_DIR) -> str:
    """The same hash recomputed from the sources in this tree: csrc/*.h, *.hip, *.cc sorted by
    name, then include/zkfl.h (the Makefile's ID_SRCS), SHA-256, first 16 hex digits."""
    import glob
    import hashlib
    names = sorted(os.path.relpath(p, pkg_dir) for ext in ("h", "hip", "cc")
                   for p in glob.glob(os.path.join(pkg_dir, "csrc", "*." + ext)))
    h = hashlib.sha256()
    for n in names + [os.path.join("..", "include", "zkfl.h")]:
        with open(os.path.join(pkg_dir, n), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def device_count() -> int:
    """HIP devices visible to this process (0 when there is no GPU or no driver)."""
    n = C.c_int(0)
    if lib().zkfl_device_count(C.byref(n)) != ZKFL_OK:
        return 0
    return n.value


def _buf(n):
    return (C.c_uint8 * n)()


class Context:
    """One device, one HIP stream (one process per GPU for multi-GPU)."""

    def __init__(self, device: int = 0):
        import weakref
        h = _P()
        check(lib().zkfl_ctx_create(device, C.byref(h)))
        self.h = h
        self.device = device
        # keys, programs and resident witnesses made on this context: closed before it, so none
        # outlives the context it points into (a key freed after its context reads freed memory)
        self._deps = weakref.WeakSet()

    def _own(self, obj):
        self._deps.add(obj)
        return obj

    def close(self):
        if self.h:
            for d in list(self._deps):
                d.close()
            lib().zkfl_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # profiling (bench.py roofline)
    def set_profiling(self, on, serialize: bool = False):
        check(lib().zkfl_ctx_set_profiling(self.h, (2 if serialize else 1) if on else 0))

    def profile(self, name: str):
        """-> (total ms, launches, units, median launch ms)"""
        ms, n, u, med = C.c_double(), C.c_uint64(), C.c_double(), C.c_double()
        check(lib().zkfl_ctx_profile(self.h, name.encode(), C.byref(ms), C.byref(n), C.byref(u), C.byref(med)))
        return ms.value, n.value, u.value, med.value

    def profile_reset(self):
        check(lib().zkfl_ctx_profile_reset(self.h))

    def synchronize(self):
        check(lib().zkfl_ctx_synchronize(self.h))

    # wave timeline (libraries built with -DZK_WTRACE=1; tools/wtrace.py)
    def wtrace_start(self, cap: int):
        check(lib().zkfl_debug_wtrace(self.h, 1, cap, None, None))

    def wtrace_stop(self, cap: int) -> tuple[bytes, int]:
        """-> (min(count, cap) records of 40 B, count recorded)"""
        buf = C.create_string_buffer(40 * cap)
        n = C.c_uint32(0)
        check(lib().zkfl_debug_wtrace(self.h, 2, cap, buf, C.byref(n)))
        return buf.raw[:40 * min(n.value, cap)], n.value

    def wtrace_free(self):
        check(lib().zkfl_debug_wtrace(self.h, 0, 0, None, None))

    # primitives
    def msm_g1(self, bases: bytes, scalars: bytes) -> bytes:
        n = len(scalars) // 32
        assert len(bases) == 64 * n
        out = _buf(64)
        check(lib().zkfl_msm_g1(self.h, bases, scalars, n, out))
        return bytes(out)

    def g1_glv_mul(self, points: bytes, scalars: bytes) -> bytes:
        """The assembly's scalar multiplications (parity hook): k_i P_i, affine std in and out."""
        n = len(scalars) // 32
        assert len(points) == 64 * n
        out = _buf(64 * n)
        check(lib().zkfl_debug_g1_glv_mul(self.h, n, points, scalars, out))
        return bytes(out)

    def msm_g2(self, bases: bytes, scalars: bytes) -> bytes:
        n = len(scalars) // 32
        assert len(bases) == 128 * n
        out = _buf(128)
        check(lib().zkfl_msm_g2(self.h, bases, scalars, n, out))
        return bytes(out)

    def ntt_coset(self, data: bytes) -> bytes:
        n = len(data) // 32
        logn = n.bit_length() - 1
        assert 1 << logn == n
        buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
        check(lib().zkfl_ntt_coset(self.h, buf, logn))
        return bytes(buf)

    def g1_gen_mul(self, scalars: bytes) -> bytes:
        n = len(scalars) // 32
        out = _buf(64 * n if n else 1)
        check(lib().zkfl_setup_g1_gen_mul(self.h, scalars, n, out))
        return bytes(out)[:64 * n]

    def g2_gen_mul(self, scalars: bytes) -> bytes:
        n = len(scalars) // 32
        out = _buf(128 * n if n else 1)
        check(lib().zkfl_setup_g2_gen_mul(self.h, scalars, n, out))
        return bytes(out)[:128 * n]

    # ceremony primitives (zkfl/ptau.py, zkfl/zkey.py::setup_from_ptau / zkey_contribute)
    def _scale(self, fn, size, points: bytes, scalars: bytes) -> bytes:
        n = len(scalars) // 32
        if len(points) != size * n or len(scalars) != 32 * n:
            raise ZkflError(-1, f"scale: {len(points)} B of points for {n} scalars")
        out = _buf(size * n if n else 1)
        check(fn(self.h, points, scalars, n, out))
        return bytes(out)[:size * n]

    def g1_scale(self, points: bytes, scalars: bytes) -> bytes:
        """out[i] = k_i * P_i (mont affine points, std scalars)."""
        return self._scale(lib().zkfl_setup_g1_scale, 64, points, scalars)

    def g2_scale(self, points: bytes, scalars: bytes) -> bytes:
        return self._scale(lib().zkfl_setup_g2_scale, 128, points, scalars)

    def _lagrange(self, fn, size, points: bytes, logn: int) -> bytes:
        if len(points) != size << logn:
            raise ZkflError(-1, f"lagrange: expected {1 << logn} points")
        out = _buf(size << logn)
        check(fn(self.h, points, logn, out))
        return bytes(out)

    def g1_lagrange(self, points: bytes, logn: int) -> bytes:
        """Inverse FFT over G1: [tau^i G] (2^logn points) -> [L_j(tau) G]."""
        return self._lagrange(lib().zkfl_setup_g1_lagrange, 64, points, logn)

    def g2_lagrange(self, points: bytes, logn: int) -> bytes:
        return self._lagrange(lib().zkfl_setup_g2_lagrange, 128, points, logn)

    def _lincomb(self, fn, size, bases: bytes, rowptr, idx, coefs: bytes) -> bytes:
        import numpy as np
        rp = np.ascontiguousarray(rowptr, dtype=np.uint64)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        n_out = len(rp) - 1
        if len(coefs) != 32 * len(ix) or int(rp[-1]) != len(ix) or len(bases) % size:
            raise ZkflError(-1, "lincomb: inconsistent term arrays")
        out = _buf(size * n_out if n_out else 1)
        check(fn(self.h, bases, len(bases) // size, n_out, rp.ctypes.data_as(C.POINTER(C.c_uint64)),
                 ix.ctypes.data_as(C.POINTER(C.c_uint32)), coefs, out))
        return bytes(out)[:size * n_out]

    def g1_lincomb(self, bases: bytes, rowptr, idx, coefs: bytes) -> bytes:
        """out[r] = sum_{t in row r} coefs[t] * bases[idx[t]] (rowptr: n_out + 1 offsets)."""
        return self._lincomb(lib().zkfl_setup_g1_lincomb, 64, bases, rowptr, idx, coefs)

    def g2_lincomb(self, bases: bytes, rowptr, idx, coefs: bytes) -> bytes:
        return self._lincomb(lib().zkfl_setup_g2_lincomb, 128, bases, rowptr, idx, coefs)

    # verification (snarkjs groth16 verify)
    def verify(self, vk: bytes, public: bytes, proof: bytes) -> bool:
        """vk image (zkfl.groth16.vk_bytes), public signals npub x 32 B std LE, proof 256 B."""
        assert len(proof) == 256 and len(public) % 32 == 0
        rc = lib().zkfl_groth16_verify(self.h, vk, len(vk), public, len(public) // 32, proof)
        if rc < 0:
            check(rc)
        return rc == 1

    def verify_batch(self, vk: bytes, publics: bytes, proofs: bytes, npub: int) -> list:
        n = len(proofs) // 256
        assert len(proofs) == 256 * n and len(publics) == 32 * npub * n
        res = (C.c_int32 * max(1, n))()
        check(lib().zkfl_groth16_verify_batch(self.h, vk, len(vk), n, publics, npub, proofs, res))
        return [bool(res[i]) for i in range(n)]

    # Poseidon / vectorHash / Merkle trees (the reference's data and server side)
    def poseidon_batch(self, rows) -> list:
        """[[ints] * arity] -> [Poseidon(row)] (circomlibjs poseidon, on the GPU)."""
        if not rows:
            return []
        arity = len(rows[0])
        assert all(len(r) == arity for r in rows)
        out = _buf(32 * len(rows))
        check(lib().zkfl_poseidon_batch(self.h, arity, len(rows), _frs(v for r in rows for v in r), out))
        return _ints(bytes(out))

    def vector_hash_batch(self, vectors) -> list:
        """[[ints] * len] -> [vectorHash(v)] (tests/full_system_simulation.mjs:139-156)."""
        if not vectors:
            return []
        ln = len(vectors[0])
        assert all(len(v) == ln for v in vectors)
        out = _buf(32 * len(vectors))
        check(lib().zkfl_vector_hash_batch(self.h, ln, len(vectors), _frs(x for v in vectors for x in v), out))
        return _ints(bytes(out))

    def merkle_build(self, leaves, depth: int) -> list:
        """buildMerkleTree(leaves, depth) -> the reference's `tree` (list of padded levels of ints)."""
        out = _buf(32 * ((2 << depth) - 1))
        check(lib().zkfl_merkle_build(self.h, _frs(leaves), len(leaves), depth, out))
        return _levels(_ints(bytes(out)), depth)

    def dataset_commit(self, samples, depth: int) -> list:
        """computeDatasetCommitment: leaves = vectorHash(sample) on the device, then the tree."""
        ln = len(samples[0]) if samples else 1
        assert all(len(v) == ln for v in samples)
        flat = self.dataset_commit_raw(_frs(x for v in samples for x in v), len(samples), ln, depth)
        return _levels(_ints(flat), depth)

    def dataset_commit_raw(self, values: bytes, n: int, ln: int, depth: int) -> bytes:
        """Byte form: values n x ln x 32 B std -> the flattened padded tree ((2^(depth+1) - 1) x 32 B)."""
        assert len(values) == 32 * n * ln
        out = _buf(32 * ((2 << depth) - 1))
        check(lib().zkfl_dataset_commit(self.h, values, n, ln, depth, out))
        return bytes(out)

    # multi-key batches (one federated round: several circuits' proofs interleaved on one device)
    def prove_multi(self, jobs, rs: bytes | None = None) -> list:
        """jobs: [(ProvingKey, ResidentWitness)] -> [proof 256 B] (zkfl_groth16_prove_multi)."""
        n = len(jobs)
        keys = (_P * max(1, n))(*[k.h for k, _ in jobs])
        ws = (_P * max(1, n))(*[w.h for _, w in jobs])
        out = _buf(256 * max(1, n))
        check(lib().zkfl_groth16_prove_multi(self.h, n, keys, ws, rs, out))
        ob = bytes(out)
        return [ob[256 * i:256 * i + 256] for i in range(n)]

    def full_prove_multi(self, jobs, rs: bytes | None = None) -> list:
        """jobs: [(ProvingKey, WitnessProgram, input vector bytes)] -> [(proof, [public ints])]
        (zkfl_groth16_full_prove_multi: witness + proof per slot, keys interleaved)."""
        n = len(jobs)
        for k, wp, inp in jobs:
            if len(inp) != 32 * wp.n_inputs:
                raise ZkflError(-1, f"expected {wp.n_inputs} input values (32 B each)")
        keys = (_P * max(1, n))(*[k.h for k, _, _ in jobs])
        progs = (_P * max(1, n))(*[wp.h for _, wp, _ in jobs])
        ins = (C.c_char_p * max(1, n))(*[inp for _, _, inp in jobs])
        pub_bufs = [_buf(32 * max(1, k.n_public)) for k, _, _ in jobs]
        pubs = (_U8P * max(1, n))(*[C.cast(b, _U8P) for b in pub_bufs])
        out = _buf(256 * max(1, n))
        check(lib().zkfl_groth16_full_prove_multi(self.h, n, keys, progs, ins, rs, out, pubs))
        ob = bytes(out)
        res = []
        for i, (k, _, _) in enumerate(jobs):
            pb = bytes(pub_bufs[i])
            res.append((ob[256 * i:256 * i + 256],
                        [int.from_bytes(pb[32 * j:32 * j + 32], "little") for j in range(k.n_public)]))
        return res

    def assemble(self, parts: bytes, n_parts: int, rs: bytes) -> list:
        """Split proofs: parts = n x n_parts x 768 B (proof-major, zkfl_groth16_prove_part_batch's
        layout), rs = n x 64 B -> n proofs of 256 B (zkfl_groth16_assemble)."""
        n = len(rs) // 64
        if len(rs) != 64 * n or len(parts) != PART_BYTES * n * n_parts:
            raise ZkflError(-1, "assemble: parts / rs sizes disagree")
        out = _buf(256 * max(1, n))
        check(lib().zkfl_groth16_assemble(self.h, n, n_parts, parts, rs, out))
        ob = bytes(out)
        return [ob[256 * i:256 * i + 256] for i in range(n)]

    def pairing(self, g1: bytes, g2: bytes, final_exp: bool = True) -> bytes:
        """e(P_i, Q_i) for n pairs (std affine); 384 B std Fq12 each (toObject order)."""
        n = len(g1) // 64
        assert len(g1) == 64 * n and len(g2) == 128 * n
        out = _buf(384 * n if n else 1)
        fn = lib().zkfl_pairing if final_exp else lib().zkfl_debug_miller_loop
        check(fn(self.h, n, g1, g2, out))
        return bytes(out)[:384 * n]


class ProvingKey:
    """A .zkey made device-resident (bases expanded per MSM window)."""

    def __init__(self, ctx: Context, zkey, shard: int = 0, n_shards: int = 1):
        """zkey: the key bytes, or its path (mapped and parsed on host threads: zkfl_zkey_file_open
        + zkfl_zkey_load_file).  shard / n_shards: keep only this shard's share of every query
        (split proofs, zkfl_zkey_load_shard); the default is the whole key."""
        h = _P()
        if isinstance(zkey, (str, os.PathLike)):
            if (shard, n_shards) != (0, 1):
                with open(zkey, "rb") as f:
                    zkey = f.read()
            else:
                fh = _P()
                check(lib().zkfl_zkey_file_open(os.fsencode(zkey), C.byref(fh)))
                try:
                    check(lib().zkfl_zkey_load_file(ctx.h, fh, C.byref(h)))
                finally:
                    lib().zkfl_zkey_file_close(fh)
        if h:
            pass
        elif n_shards == 1 and shard == 0:
            check(lib().zkfl_zkey_load(ctx.h, zkey, len(zkey), C.byref(h)))
        else:
            check(lib().zkfl_zkey_load_shard(ctx.h, zkey, len(zkey), shard, n_shards, C.byref(h)))
        self.h = h
        self.shard, self.n_shards = shard, n_shards
        self.ctx = ctx
        ctx._own(self)
        nv, npub, dom = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(lib().zkfl_key_info(h, C.byref(nv), C.byref(npub), C.byref(dom)))
        self.n_vars, self.n_public, self.domain_size = nv.value, npub.value, dom.value

    def close(self):
        if self.h:
            lib().zkfl_key_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_slots(self, slots: int):
        """Proofs kept in flight by prove_batch (each slot = 3 HIP streams + scratch)."""
        check(lib().zkfl_key_set_slots(self.h, slots))
        self.slots = slots

    def prove(self, wtns: bytes, rs: bytes | None = None):
        """-> (proof 256 B, [public signal ints])"""
        proof = _buf(256)
        pub = _buf(32 * max(1, self.n_public))
        npub = C.c_size_t()
        check(lib().zkfl_groth16_prove(self.ctx.h, self.h, wtns, len(wtns), rs, proof, pub, C.byref(npub)))
        pb = bytes(pub)
        return bytes(proof), [int.from_bytes(pb[32 * i:32 * i + 32], "little") for i in range(npub.value)]

    def upload(self, wtns: bytes) -> "ResidentWitness":
        return ResidentWitness(self, wtns)

    def prove_resident(self, w: "ResidentWitness", rs: bytes | None = None) -> bytes:
        proof = _buf(256)
        check(lib().zkfl_groth16_prove_resident(self.ctx.h, self.h, w.h, rs, proof))
        return bytes(proof)

    def prove_batch(self, ws, rs: bytes | None = None) -> list:
        n = len(ws)
        arr = (_P * n)(*[w.h for w in ws])
        out = _buf(256 * n)
        check(lib().zkfl_groth16_prove_batch(self.ctx.h, self.h, n, arr, rs, out))
        ob = bytes(out)
        return [ob[256 * i:256 * i + 256] for i in range(n)]

    def prove_part_batch(self, ws, rs: bytes) -> list:
        """This shard's parts of n proofs (rs REQUIRED, n x 64 B, the same on every shard)
        -> [768 B] (zkfl_groth16_prove_part_batch)."""
        n = len(ws)
        if rs is None or len(rs) != 64 * n:
            raise ZkflError(-1, "prove_part_batch: rs must be n x 64 bytes")
        arr = (_P * max(1, n))(*[w.h for w in ws])
        out = _buf(PART_BYTES * max(1, n))
        check(lib().zkfl_groth16_prove_part_batch(self.ctx.h, self.h, n, arr, rs, out))
        ob = bytes(out)
        return [ob[PART_BYTES * i:PART_BYTES * (i + 1)] for i in range(n)]

    def full_prove_batch(self, prog: "WitnessProgram", inputs, rs: bytes | None = None):
        """input vectors (wprog.input_bytes / parse_inputs) -> [(proof 256 B, [public ints])]:
        witness and proof pipelined per slot on the GPU (zkfl_groth16_full_prove_batch)."""
        n = len(inputs)
        buf = prog._inputs(inputs)
        out = _buf(256 * max(1, n))
        pubs = _buf(32 * max(1, self.n_public) * max(1, n))
        check(lib().zkfl_groth16_full_prove_batch(self.ctx.h, self.h, prog.h, n, buf, rs, out, pubs))
        ob, pb = bytes(out), bytes(pubs)
        k = self.n_public
        return [(ob[256 * i:256 * i + 256],
                 [int.from_bytes(pb[32 * (i * k + j):32 * (i * k + j) + 32], "little") for j in range(k)])
                for i in range(n)]

    def full_prove_json_batch(self, prog: "WitnessProgram", texts, rs: bytes | None = None):
        """input.json texts -> [(proof 256 B, [public ints])]: parsed by host threads while earlier
        proofs run (zkfl_groth16_full_prove_json_batch)."""
        n = len(texts)
        arr = (C.c_char_p * max(1, n))(*[t.encode() if isinstance(t, str) else t for t in texts])
        out = _buf(256 * max(1, n))
        pubs = _buf(32 * max(1, self.n_public) * max(1, n))
        check(lib().zkfl_groth16_full_prove_json_batch(self.ctx.h, self.h, prog.h, n, arr, rs, out, pubs))
        ob, pb = bytes(out), bytes(pubs)
        k = self.n_public
        return [(ob[256 * i:256 * i + 256],
                 [int.from_bytes(pb[32 * (i * k + j):32 * (i * k + j) + 32], "little") for j in range(k)])
                for i in range(n)]

    def full_prove_json(self, prog: "WitnessProgram", input_json: str, rs: bytes | None = None):
        """snarkjs groth16.fullProve for one input.json text -> (proof 256 B, [public ints])."""
        out = _buf(256)
        pub = _buf(32 * max(1, self.n_public))
        check(lib().zkfl_groth16_full_prove_json(self.ctx.h, self.h, prog.h, input_json.encode(), rs, out, pub))
        return bytes(out), _ints(bytes(pub))[:self.n_public]

    def debug_parts(self, wtns: bytes):
        """-> (h list of ints, dict of MSM results as std affine bytes)"""
        h = _buf(32 * self.domain_size)
        m = _buf(384)
        check(lib().zkfl_debug_prove_parts(self.ctx.h, self.h, wtns, len(wtns), h, m))
        hb, mb = bytes(h), bytes(m)
        hs = [int.from_bytes(hb[32 * i:32 * i + 32], "little") for i in range(self.domain_size)]
        parts = dict(A=mb[0:64], B1=mb[64:128], B2=mb[128:256], C=mb[256:320], H=mb[320:384])
        return hs, parts


class ResidentWitness:
    def __init__(self, key: ProvingKey, wtns: bytes | None = None, handle=None):
        if handle is not None:
            self.h = handle
            key.ctx._own(self)
            return
        h = _P()
        check(lib().zkfl_witness_upload(key.ctx.h, key.h, wtns, len(wtns), C.byref(h)))
        self.h = h
        key.ctx._own(self)

    def close(self):
        if self.h:
            lib().zkfl_witness_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def parse_inputs(image: bytes, input_json: str, cap: int | None = None) -> bytes:
    """circom input.json -> flattened input vector via the program's signal table (host only).
    cap: room for this many values (default: the image's input count, header word 4 + 5)."""
    if cap is None:
        cap = max(1, int.from_bytes(image[16:20], "little") + int.from_bytes(image[20:24], "little"))
    out = _buf(32 * cap)
    n = C.c_size_t()
    check(lib().zkfl_wprog_parse_inputs(image, len(image), input_json.encode(), out, cap, C.byref(n)))
    return bytes(out)[:32 * n.value]


class WitnessProgram:
    """A compiled circuit witness program (zkfl.wprog image) loaded on the device: the
    replacement of circom's <circuit>.wasm + generate_witness.cjs."""

    def __init__(self, ctx: Context, image: bytes):
        h = _P()
        check(lib().zkfl_wprog_load(ctx.h, image, len(image), C.byref(h)))
        self.h, self.ctx = h, ctx
        ctx._own(self)
        nw, ni, npub = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(lib().zkfl_wprog_info(h, C.byref(nw), C.byref(ni), C.byref(npub)))
        self.n_wires, self.n_inputs, self.n_public = nw.value, ni.value, npub.value
        self.wtns_size = lib().zkfl_wtns_size(h)

    def close(self):
        if self.h:
            lib().zkfl_wprog_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _inputs(self, inputs) -> bytes:
        buf = b"".join(inputs)
        if len(buf) != 32 * self.n_inputs * len(inputs):
            raise ZkflError(-1, f"expected {self.n_inputs} input values (32 B each) per witness")
        return buf

    def compute(self, inputs) -> list:
        """inputs: list of per-witness input byte strings (zkfl.wprog.input_bytes) -> .wtns images."""
        n = len(inputs)
        out = _buf(self.wtns_size * max(1, n))
        check(lib().zkfl_witness_compute(self.ctx.h, self.h, n, self._inputs(inputs), out))
        ob = bytes(out)
        return [ob[i * self.wtns_size:(i + 1) * self.wtns_size] for i in range(n)]

    def compute_json(self, input_json: str) -> bytes:
        """One witness from circom's input.json text -> .wtns image."""
        out = _buf(self.wtns_size)
        check(lib().zkfl_witness_compute_json(self.ctx.h, self.h, input_json.encode(), out))
        return bytes(out)

    def compute_resident(self, key: ProvingKey, inputs) -> list:
        """-> ResidentWitness per input, computed in HBM for `key` (no host round trip)."""
        n = len(inputs)
        arr = (_P * max(1, n))()
        check(lib().zkfl_witness_compute_resident(self.ctx.h, self.h, key.h, n, self._inputs(inputs), arr))
        return [ResidentWitness(key, handle=_P(arr[i])) for i in range(n)]
