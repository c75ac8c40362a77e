"""The C-ABI library loads and exports every symbol include/zkfl.h declares (no GPU calls)."""
import ctypes
import os
import re

from zkfl import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "zkfl.h")).read()
    return sorted(set(re.findall(r"\b(zkfl_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_surface():
    names = _declared()
    for must in ("zkfl_zkey_load", "zkfl_groth16_prove", "zkfl_groth16_prove_batch", "zkfl_msm_g1",
                 "zkfl_msm_g2", "zkfl_ntt_coset", "zkfl_setup_g1_gen_mul", "zkfl_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(native.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name
    assert set(_declared()) == set(native.SIGNATURES)


def test_version_and_error_paths_without_device():
    L = native.lib()
    assert L.zkfl_version() == 1
    # null-argument paths return ZKFL_E_ARG without touching a device
    assert L.zkfl_key_info(None, None, None, None) == -1
    assert L.zkfl_ctx_set_profiling(None, 1) == -1


def test_glv_split_host():
    """The assembly's GLV split (csrc/glv.h, host code): k = k1 + k2*lambda (mod r), |k_i| < 2^128,
    on edge scalars and seeded random ones; r >= r is rejected."""
    import random
    from oracle import bn254 as bn
    lam = 0xb3c4d79d41a917585bfc41088d8daaa78b17ea66b99c90dd
    assert (lam * lam + lam + 1) % bn.R == 0
    L = native.lib()
    rnd = random.Random(5)
    ks = [0, 1, 2, lam, bn.R - 1, bn.R // 2, (1 << 253)] + [rnd.randrange(bn.R) for _ in range(500)]
    out = (ctypes.c_uint8 * 40)()
    for k in ks:
        assert L.zkfl_debug_glv_split(k.to_bytes(32, "little"), out) == 0
        b = bytes(out)
        k1 = int.from_bytes(b[0:16], "little") * (-1 if b[16] else 1)
        k2 = int.from_bytes(b[20:36], "little") * (-1 if b[36] else 1)
        assert (k1 + k2 * lam - k) % bn.R == 0, k
        assert abs(k1) < 1 << 128 and abs(k2) < 1 << 128
    assert L.zkfl_debug_glv_split(bn.R.to_bytes(32, "little"), out) == -1


def test_node_addon_loads():
    """N-API addon (node/zkfl.node) loads in Node and exposes the binding (no GPU calls)."""
    import shutil
    import subprocess
    node = shutil.which("node")
    addon = os.path.join(os.path.dirname(native.LIB_PATH), "node", "zkfl.node")
    if not node or not os.path.exists(addon):
        import pytest
        pytest.skip("node or addon not available")
    js = ("const a=require(process.argv[1]);"
          "const k=['version','deviceCount','createContext','loadKey','keyInfo','prove'];"
          "for (const f of k) if (typeof a[f] !== 'function') throw new Error(f);"
          "console.log(a.version());")
    out = subprocess.run([node, "-e", js, addon], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "1"


def test_poseidon_params_host_generator_matches_oracle():
    """The library's native Grain-LFSR generator (csrc/merkle.hip, host code, no device) yields
    circomlib's constants for every width t = 2..17: the round constants and the MDS matrix
    M[i][j] = 1/(x_i + y_j) equal oracle/poseidon.py's (pinned by the reference fixture)."""
    from oracle import poseidon as op
    for t in range(2, 18):
        consts, xs, ys, rp = native.poseidon_params(t)
        C, M = op.constants(t)
        assert rp == op.N_ROUNDS_P[t - 2]
        assert consts == list(C)
        assert [[pow(x + y, op.R - 2, op.R) for y in ys] for x in xs] == [list(r) for r in M]
    assert native.lib().zkfl_poseidon_params(18, None, None, None) == -1
