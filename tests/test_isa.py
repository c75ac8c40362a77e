"""gfx950 ISA of the built libzkfl.so, checked on the CPU (tools/isa_check.py; no GPU needed).

Guards the LDS-DMA ordering of the MSM accumulation kernels (csrc/msm.h k_msm_accumulate): every
ds_read_b128 of the prefetch buffer must be preceded, on every control-flow path, by an
`s_waitcnt vmcnt(0)` after the global_load_lds_dwordx4 that fills it.  In round 3 the compiler
dropped that wait on the loop's first iteration once the buffer became a native vector type
(commit 5a57083): 25 GPU proof tests failed while the MSM primitive tests passed by timing, so
the ordering is now checked statically on the shipped code object instead of by luck on the GPU.
"""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_check  # noqa: E402

SO = os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd", "libzkfl.so")


@pytest.fixture(scope="module")
def acc():
    if not os.path.exists(SO):
        pytest.skip("libzkfl.so not built (__graft_entry__.build())")
    if not shutil.which(os.path.join(isa_check.LLVM, "llvm-objdump")):
        pytest.skip("llvm-objdump not available")
    ks = isa_check.disassemble(SO, r"k_msm_accumulate")
    return ks


def test_both_accumulation_kernels_present(acc):
    names = list(acc)
    assert any("FqOps29" in n for n in names) and any("Fq2Pair29" in n for n in names), names


def test_lds_dma_waited_before_every_read(acc):
    for name, lines in acc.items():
        assert sum("global_load_lds_dwordx4" in ln for ln in lines) >= 4, name   # the prefetch exists
        assert sum("ds_read_b128" in ln for ln in lines) >= 4, name
        bad = isa_check.lds_dma_hazards(lines)
        assert not bad, f"{name}: LDS reads with a DMA possibly in flight: {bad}"


def test_checker_finds_a_dropped_wait(acc):
    """The checker itself: the same kernels with their vmcnt(0) waits deleted must be flagged
    (the round-3 failure mode)."""
    for name, lines in acc.items():
        stripped = [ln for ln in lines if not ln.startswith("s_waitcnt") or "vmcnt(0)" not in ln]
        assert isa_check.lds_dma_hazards(stripped), name


def test_accumulation_kernels_do_not_spill(acc):
    """G1 and G2, each as the one-MSM kernel and the multi-MSM one (small keys' A, B1, C + H in one
    launch, k_msm_accumulate_multi: the same body, msm_acc_chunk)."""
    res = isa_check.resources(SO, r"k_msm_accumulate")
    assert len(res) == 4 and sum("_multi" in n for n in res) == 2, list(res)
    for name, r in res.items():
        assert r.get("vgpr_spill_count", 0) == 0 and r.get("private_segment_fixed_size", 0) == 0, (name, r)
        assert r["group_segment_fixed_size"] == 8192, (name, r)  # two 4 KB LDS-DMA buffers per wave


def test_assembly_row_chains(acc):
    """The assembly's GLV chains in row form (csrc/row29.h): the kernels that run them hold no
    scratch, and their products use the DPP row broadcasts and row shifts and the gfx950 row swaps
    they were written for (a compiler fallback to LDS or scalar paths would show as their absence)."""
    res = isa_check.resources(SO, r"k_assemble|k_debug_glv_mul")
    assert len(res) == 4, list(res)  # k_assemble, k_assemble_t, k_assemble_c, k_debug_glv_mul
    for name, r in res.items():
        assert r.get("vgpr_spill_count", 0) == 0 and r.get("private_segment_fixed_size", 0) == 0, (name, r)
    for name, lines in isa_check.disassemble(SO, r"k_assemble_t|k_debug_glv_mul").items():
        text = "\n".join(lines)
        for op in ("row_newbcast:0", "row_newbcast:8", "row_shl:1", "row_shr:1", "v_permlane16_swap",
                   "v_permlane32_swap"):
            assert op in text, (name, op)


def test_accumulation_census(acc):
    """The main loops hold the point formula's products exactly (G1 madd: 6 products x 162 + 2
    squares x 126 + the Y3 sum 243 = 1467 v_mad_u64_u32; G2 per lane 2187), and the G1 formula's
    other instructions stay within the budget the paired products brought (round 5: 2,345 -> 2,211
    VALU instructions, the 17 column joins of each paired product gone)."""
    for name, lines in acc.items():
        g2 = "Fq2Pair29" in name
        cz = isa_check.census(lines, 2187 if g2 else 1467)
        assert cz["formula"]["mad64"] == (2187 if g2 else 1467), name
        assert cz["formula"]["mul_lo"] == 81, name  # 9 Montgomery m per reduction, 9 reductions per lane
        if not g2:
            assert cz["formula"]["valu"] <= 2250, (name, cz["formula"])
            assert cz["formula"]["add64"] <= 180, (name, cz["formula"])  # joins of unpaired products only


def test_no_function_clobbers_its_return_address():
    """Round-3 G2 ceremony hang (commit 68f6c67), root cause found on the CPU from the pre-fix code
    object: the outlined smul_xyzz<Fq2Ops> / smul_aff<Fq2Ops> (333 / 276 KB, past the +-128 KB
    reach of s_branch) got long branches `s_getpc_b64 s[30:31]; s_add_u32 s30 ..; s_setpc_b64
    s[30:31]` that used the return-address pair as scratch, so the final `s_setpc_b64 s[30:31]`
    jumped back into the loop and the waves never finished.  No non-kernel function of the shipped
    library may write s[30:31]."""
    if not os.path.exists(SO):
        pytest.skip("libzkfl.so not built")
    fns = isa_check.functions(SO)
    assert fns, "the pairing helpers are outlined (csrc/pairing.h ZK_NOINLINE): expected functions"
    bad = {n: isa_check.return_address_clobbers(ls) for n, ls in fns.items()}
    assert not {n: b for n, b in bad.items() if b}, bad


def test_return_address_checker_flags_the_r03_code():
    """The checker on an excerpt of the round-3 smul_xyzz<Fq2Ops> disassembly (its entry up to the
    first long branch, and its end): the long branch writes s[30:31], then the 'return' uses it."""
    path = os.path.join(ROOT, "tests", "golden", "isa_r03_smul_xyzz_g2_excerpt.s")
    lines = [ln.strip() for ln in open(path) if ln.strip() and ln.strip() != "..."]
    got = isa_check.return_address_clobbers(lines)
    assert any(g.startswith("s_getpc_b64 s[30:31]") for g in got)
    assert lines[-1].startswith("s_setpc_b64 s[30:31]")
