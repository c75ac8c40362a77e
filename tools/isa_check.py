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


def lds_dma_hazards(lines: list[str]) -> list[str]:
    """ds_read_b128 instructions reachable with an LDS DMA possibly in flight (see module doc)."""
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
