#!/usr/bin/env python3
"""gfx950 ISA checks on the built library (CPU only: no GPU needed).

  * code_objects(so): the gfx950 code objects of a HIP shared library -- every clang offload
    bundle in its .hip_fatbin section, the `hipv4-amdgcn-amd-amdhsa--gfx950` entry of each.
  * disassemble(so, pattern): {symbol: [instruction lines]} of the kernels whose mangled name
    matches `pattern` (llvm-objdump --mcpu=gfx950).
  * resources(so, pattern): {symbol: {vgpr_count, sgpr_count, vgpr_spill_count, private_segment_fixed_size,
    group_segment_fixed_size}} from the code objects' metadata notes.
  * lds_dma_hazards(lines): every ds_read_b128 that can execute while a global_load_lds_dwordx4
    (LDS DMA, counted by vmcnt) may still be in flight on some control-flow path, i.e. with no
    `s_waitcnt vmcnt(0)` between them.  A forward dataflow over the kernel's basic blocks (branch
    targets from the disassembly's <sym+0xOFF> annotations): "DMA pending" is set by the load,
    cleared by the wait, OR-ed over predecessors.

The hazard is the one found by the GPU proof tests in round 3 (commit 5a57083): with the
prefetch buffer as a native vector type the compiler stopped tying the LDS reads to the LDS-DMA
writes and dropped the vmcnt wait of the accumulation loop's first iteration (csrc/msm.h,
k_msm_accumulate); the MSM primitive tests passed by timing.  tests/test_isa.py runs this on
both accumulation kernels.

  * functions(so) / return_address_clobbers(lines): non-kernel functions that write s[30:31], the
    return address (the round-3 G2 ceremony hang, commit 68f6c67; see return_address_clobbers).

    python3 tools/isa_check.py [path/to/libzkfl.so]
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TRIPLE = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(so: str) -> list[bytes]:
    data = open(so, "rb").read()
    out = []
    for m in re.finditer(re.escape(MAGIC), data):
        off = m.start()
        p = off + len(MAGIC)
        (n,) = struct.unpack_from("<Q", data, p)
        p += 8
        for _ in range(n):
            o, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if triple == TRIPLE:
                out.append(data[off + o:off + o + size])
    return out


def _objdump(co: bytes, *args: str) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        return subprocess.run([os.path.join(LLVM, "llvm-objdump"), *args, f.name], check=True,
                              capture_output=True, text=True).stdout


def disassemble(so: str, pattern: str) -> dict[str, list[str]]:
    rx = re.compile(pattern)
    kernels: dict[str, list[str]] = {}
    for co in code_objects(so):
        cur = None
        for ln in _objdump(co, "-d", "--mcpu=gfx950").splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:$", ln)
            if m:
                cur = m.group(1) if rx.search(m.group(1)) else None
                if cur:
                    kernels[cur] = []
                continue
            if cur and ln.strip():
                kernels[cur].append(ln.strip())
    return kernels


def resources(so: str, pattern: str) -> dict[str, dict[str, int]]:
    rx = re.compile(pattern)
    keys = ("vgpr_count", "sgpr_count", "vgpr_spill_count", "private_segment_fixed_size",
            "group_segment_fixed_size")
    out: dict[str, dict[str, int]] = {}
    for co in code_objects(so):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], check=True,
                                   capture_output=True, text=True).stdout
        for block in notes.split("  - .agpr_count")[1:]:  # one amdhsa.kernels entry each
            name = re.search(r"\.name:\s+(\S+)", block)
            if not name or not rx.search(name.group(1)):
                continue
            out[name.group(1)] = {k: int(re.search(rf"\.{k}:\s+(\d+)", block).group(1)) for k in keys
                                  if re.search(rf"\.{k}:\s+(\d+)", block)}
    return out


_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_TARGET = re.compile(r"<[^>+]+\+0x([0-9a-f]+)>")


def _cfg(lines: list[str]):
    """(ins, blocks, succs): the kernel's instructions as (offset from its start, text), its basic
    blocks as [start, end) instruction index ranges, and each block's successor blocks (branch
    targets from the disassembly's <sym+0xOFF> annotations)."""
    ins = []  # (offset from the kernel start, text)
    base = None
    for ln in lines:
        m = _ADDR.search(ln)
        if not m:
            continue
        a = int(m.group(1), 16)
        base = a if base is None else base
        ins.append((a - base, ln.split("//")[0].strip()))
    index = {off: i for i, (off, _) in enumerate(ins)}
    src = [ln for ln in lines if _ADDR.search(ln)]  # ins[i] is src[i] (its branch-target annotation)
    # basic-block leaders: the entry, branch targets, instructions after a branch
    succ_of: dict[int, list[int]] = {}
    leaders = {0}
    for i, (off, text) in enumerate(ins):
        op = text.split()[0] if text else ""
        if op.startswith("s_cbranch") or op == "s_branch":
            t = _TARGET.search(src[i])
            tgt = index.get(int(t.group(1), 16)) if t else None
            succ_of[i] = ([tgt] if tgt is not None else []) + ([i + 1] if op != "s_branch" else [])
            if tgt is not None:
                leaders.add(tgt)
            leaders.add(i + 1)
        elif op in ("s_endpgm", "s_setpc_b64"):
            succ_of[i] = []
            leaders.add(i + 1)
    starts = sorted(x for x in leaders if x < len(ins))
    blocks = [(s, (starts[k + 1] if k + 1 < len(starts) else len(ins))) for k, s in enumerate(starts)]
    block_of = {s: k for k, (s, _) in enumerate(blocks)}
    succs: list[list[int]] = []
    for s, e in blocks:
        last = e - 1
        nxt = succ_of.get(last, [e] if e < len(ins) else [])
        succs.append([block_of[x] for x in nxt if x in block_of])
    return ins, blocks, succs


def lds_dma_hazards(lines: list[str]) -> list[str]:
    """ds_read_b128 instructions reachable with an LDS DMA possibly in flight (see module doc)."""
    ins, blocks, succs = _cfg(lines)
    wait0 = re.compile(r"^s_waitcnt\b.*\bvmcnt\(0\)")

    def transfer(k: int, pending: bool, report: list[str] | None) -> bool:
        s, e = blocks[k]
        for i in range(s, e):
            text = ins[i][1]
            if text.startswith("global_load_lds_dwordx4"):
                pending = True
            elif wait0.match(text):
                pending = False
            elif text.startswith("ds_read_b128") and pending and report is not None:
                report.append(f"+0x{ins[i][0]:x}: {text}")
        return pending

    entry = [False] * len(blocks)
    work = list(range(len(blocks)))
    while work:
        k = work.pop()
        out = transfer(k, entry[k], None)
        for t in succs[k]:
            if out and not entry[t]:
                entry[t] = True
                work.append(t)
    bad: list[str] = []
    for k in range(len(blocks)):
        transfer(k, entry[k], bad)
    return bad


# VALU instruction classes of the census (first match wins); everything else starting with v_ is
# "valu other", ds_ LDS, global_/buffer_ VMEM, s_ scalar
_CLASSES = (
    ("mad64", ("v_mad_u64_u32",)),                                  # the limb products
    ("mul_lo", ("v_mul_lo_u32",)),                                  # Montgomery m = c * n' mod 2^29
    ("add64", ("v_lshl_add_u64", "v_add_co_u32", "v_addc_co_u32", "v_add_u64")),  # column joins / sums
    ("shift64", ("v_lshrrev_b64", "v_lshlrev_b64", "v_alignbit_b32")),  # column carries, limb repacking
    ("mask", ("v_and_b32", "v_bfe_u32", "v_and_or_b32", "v_bfi_b32")),  # 29-bit limb masks
    ("add32", ("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_add3_u32", "v_sub_co", "v_subb", "v_add_lshl")),
    ("logic", ("v_or", "v_xor", "v_lshl", "v_lshr", "v_ashr", "v_not", "v_bitop3", "v_perm")),
    ("cmp_sel", ("v_cmp", "v_cndmask")),
    ("mov", ("v_mov",)),
    ("lane", ("v_readlane", "v_writelane", "v_readfirstlane", "v_permlane")),
)


def _cls(text: str) -> str:
    op = text.split()[0] if text else ""
    for name, prefixes in _CLASSES:
        if op.startswith(prefixes):
            return name
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_")):
        return "vmem"
    return "salu"


_VALU = tuple(n for n, _ in _CLASSES) + ("valu_other",)


def census(lines: list[str], formula_mads: int) -> dict:
    """Instruction census of an accumulation kernel's main loop (the innermost loop that holds the
    point formula).  formula_mads: the mads of one point addition as written (G1 madd:
    6 products x 162 + 2 squares x 126 + the Y3 product sum 243 = 1467); the loop's blocks with mads
    whose counts sum to exactly that are the formula's ("formula"), other blocks with mads are the
    special cases (P == 0: the doubling, "cold"), blocks with a global store are the run ends
    ("emit": executed when any lane of the wave closes a bucket run), mad-free blocks on every path
    from the loop header to the formula are the loop head ("head": key / index loads, the LDS read
    of the prefetched base and its 8 x 32 -> 9 x 29 repacking, the zero tests), the rest "other"
    (the run ends' bookkeeping, the latch).  The
    per-entry path is head + formula."""
    import itertools
    ins, blocks, succs = _cfg(lines)
    cnt = []
    for s, e in blocks:
        c: dict[str, int] = {}
        for i in range(s, e):
            k = _cls(ins[i][1])
            c[k] = c.get(k, 0) + 1
        c["stores"] = sum(1 for i in range(s, e) if ins[i][1].startswith(("global_store", "buffer_store")))
        cnt.append(c)
    # the main loop: the innermost back edge whose blocks contain the formula (a subset of its
    # blocks with mads summing to formula_mads exactly)
    def formula_in(blks):
        withmad = [j for j in blks if cnt[j].get("mad64", 0)]
        for r in range(1, len(withmad) + 1):
            for comb in itertools.combinations(withmad, r):
                if sum(cnt[j]["mad64"] for j in comb) == formula_mads:
                    return list(comb)
        return None
    preds: list[list[int]] = [[] for _ in blocks]
    for k, ss in enumerate(succs):
        for t in ss:
            preds[t].append(k)

    def natural_loop(t, k):  # the header t and every block that reaches the latch k without passing t
        body, work = {t, k}, [k]
        while work:
            x = work.pop()
            for p in preds[x]:
                if p not in body:
                    body.add(p)
                    work.append(p)
        return sorted(body)
    # dominators (iterative): an edge k -> t is a back edge when t dominates k (the compiler may
    # place a loop's latch before its header, so address order does not tell)
    nb = len(blocks)
    dom = [set(range(nb)) for _ in range(nb)]
    dom[0] = {0}
    changed = True
    while changed:
        changed = False
        for x in range(1, nb):
            ps = [dom[p] for p in preds[x]]
            d = (set.intersection(*ps) if ps else set()) | {x}
            if d != dom[x]:
                dom[x], changed = d, True
    best = None
    for k, ss in enumerate(succs):
        for t in ss:
            if t in dom[k]:
                body = natural_loop(t, k)
                if best is None or len(body) < len(best[0]):
                    f = formula_in(body)
                    if f:
                        best = (body, f)
    assert best, f"no loop holds {formula_mads} mads in a subset of its blocks"
    loop, formula = best
    header = next(t for t in loop if all(t in dom[j] for j in loop))
    first = min(formula)
    rows = []
    for j in loop:
        c = cnt[j]
        if j in formula:
            kind = "formula"
        elif c.get("mad64"):
            kind = "cold"
        elif c["stores"]:
            kind = "emit"
        elif j in dom[first]:  # on every path from the loop header to the formula
            kind = "head"
        else:
            kind = "other"
        rows.append((ins[blocks[j][0]][0], kind, c))

    def total(kinds):
        t: dict[str, int] = {}
        for _, kind, c in rows:
            if kind in kinds:
                for k, v in c.items():
                    t[k] = t.get(k, 0) + v
        t["valu"] = sum(t.get(k, 0) for k in _VALU)
        return t
    return {"blocks": rows, "path": total(("head", "formula")), "formula": total(("formula",)),
            "head": total(("head",)), "emit": total(("emit",)), "cold": total(("cold",))}


def print_census(name: str, cz: dict) -> None:
    print(f"{name}: main-loop census (per lane, per accumulated entry on the path head + formula)")
    keys = _VALU + ("lds", "vmem")
    print("   block      kind     valu " + " ".join(f"{k:>9s}" for k in keys))
    for off, kind, c in cz["blocks"]:
        v = sum(c.get(k, 0) for k in _VALU)
        print(f"   +0x{off:<7x} {kind:8s} {v:5d} " + " ".join(f"{c.get(k, 0):9d}" for k in keys))
    for part in ("head", "formula", "path", "emit"):
        t = cz[part]
        print(f"   {part:8s} valu {t['valu']:5d}: " + ", ".join(f"{k} {t[k]}" for k in keys if t.get(k)))


def functions(so: str) -> dict[str, list[str]]:
    """Non-kernel functions (called by s_swappc) of every gfx950 code object: {symbol: lines}."""
    out: dict[str, list[str]] = {}
    for co in code_objects(so):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], check=True,
                                   capture_output=True, text=True).stdout
        kernels = set(re.findall(r"\.name:\s+(\S+)", notes))
        cur = None
        for ln in _objdump(co, "-d", "--mcpu=gfx950").splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:$", ln)
            if m:
                cur = None if m.group(1) in kernels else m.group(1)
                if cur:
                    out[cur] = []
                continue
            if cur and ln.strip():
                out[cur].append(ln.strip())
    return out


_RA_WRITE = re.compile(r"^(s_getpc_b64|s_mov_b64|s_add_u32|s_addc_u32|s_mov_b32|s_load_dwordx2)\s+s(\[30:31\]|30\b|31\b)")


def return_address_clobbers(lines: list[str]) -> list[str]:
    """Writes of s[30:31] -- the return address of the AMDGPU calling convention -- inside a
    non-kernel function.  The round-3 G2 ceremony hang (commit 68f6c67): the outlined 215 KB
    smul_xyzz<Fq2Ops> / smul_aff<Fq2Ops> were past the +-128 KB reach of s_branch, and the long
    branches the compiler expanded them into (s_getpc_b64 s[30:31]; s_add_u32 s30 ...;
    s_setpc_b64 s[30:31]) took s[30:31] as their scratch pair without saving it, so the function's
    final `s_setpc_b64 s[30:31]` "returned" to the last long-branch target inside the loop: the
    waves never left.  A function here may restore s[30:31] from a save before it returns; this
    flags every write so such a case is looked at, and there is none in the current library."""
    return [ln.split("//")[0].strip() for ln in lines if _RA_WRITE.match(ln)]


def main() -> int:
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        root, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd", "libzkfl.so")
    ks = disassemble(so, r"k_msm_accumulate")
    rc = 0
    for name, lines in ks.items():
        n_dma = sum(1 for ln in lines if "global_load_lds_dwordx4" in ln)
        n_rd = sum(1 for ln in lines if "ds_read_b128" in ln)
        bad = lds_dma_hazards(lines)
        print(f"{name}: {len(lines)} instructions, {n_dma} LDS-DMA loads, {n_rd} ds_read_b128, "
              f"{len(bad)} reads with a DMA possibly in flight")
        for b in bad:
            print("   ", b)
        rc |= bool(bad)
    for name, lines in ks.items():  # the formula's mads: G1 madd 1467; G2 per lane (lane pairs) 2187
        print_census(name[:60], census(lines, 2187 if "Fq2Pair29" in name else 1467))
    for name, r in resources(so, r"k_msm_(accumulate|stitch|wsum)|k_assemble").items():
        print(name[:60], r)
    for name, lines in functions(so).items():
        bad = return_address_clobbers(lines)
        addrs = [int(m.group(1), 16) for m in map(_ADDR.search, lines) if m]
        size = (addrs[-1] - addrs[0] + 8) if addrs else 0
        print(f"function {name[:70]}: {len(lines)} instructions, {size // 1024} KB "
              f"(s_branch reaches +-128 KB), {len(bad)} writes of the return address s[30:31]")
        rc |= bool(bad)
    return rc


if __name__ == "__main__":
    sys.exit(main())
