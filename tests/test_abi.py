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
