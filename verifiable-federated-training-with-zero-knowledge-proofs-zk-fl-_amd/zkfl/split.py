"""One Groth16 proof split over the ranks of a torch.distributed group (optional).

The reference proves every client's update with one `npx snarkjs groth16 prove` on one machine
(tests/full_system_simulation.mjs:773-776); its throughput path here is one proof per GPU slot,
replicas across GPUs.  This module is the other axis: ONE proof's latency divided
over G GPUs, one process per GPU.

    rank k: zkey shard k of G (zkfl_zkey_load_shard: base i of every query when i % G == k,
            the alpha/beta/delta augmentation on shard 0), the FULL witness, the same (r, s)
      -> ABC + coset NTT (whole, redundant on every rank) + this shard's share of the 5 MSMs
      -> a 768-byte part: A' | B1' | B2' | C'+H | H as XYZZ points, std-form coordinates
         (zkfl_groth16_prove_part_batch; no inversion on the shard)
    all_gather of the parts (768 B per proof per rank: a latency-bound exchange, not a bandwidth
    one -- EC addition is not a collective reduction op, so gather + add on the root)
    rank 0: sum the parts and assemble pi_c = C' + H + s pi_a + r B1' on its GPU
            (zkfl_groth16_assemble) -> 256-byte proofs, byte-identical to an unsplit proof with
            the same r, s.

`split_prove` is the collective protocol with the two device calls passed in, so the same code
runs on the CPU in tests (tests/test_split_cpu.py drives it over gloo with the CPU oracle as the
device) and with libzkfl on MI355X (tests/test_gpu_split.py, bench.py's split leg).  The exchange
uses the group's backend: gloo moves the parts as host tensors (they come back from the device
anyway, 768 B each); an nccl (RCCL) group moves them as device tensors over xGMI.  The tests and
the bench use gloo: RCCL refuses two ranks on one device, which is all a 1-GPU lease has.
"""

from __future__ import annotations

import secrets

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
PART_BYTES = 768  # native.PART_BYTES (kept here so the protocol imports without the library)


def draw_rs(n: int) -> bytes:
    """n pairs (r, s), each uniform below r, 32 B little-endian (snarkjs: Fr.random())."""
    out = bytearray()
    for _ in range(2 * n):
        while True:
            v = int.from_bytes(secrets.token_bytes(32), "little") & ((1 << 254) - 1)
            if v < R:
                break
        out += v.to_bytes(32, "little")
    return bytes(out)


def split_prove(part_fn, assemble_fn, n: int, rs: bytes | None = None, group=None, device=None,
                root: int = 0):
    """Prove n proofs split over the group's ranks.

    part_fn(rs) -> list of n PART_BYTES-byte parts (this rank's shard);
    assemble_fn(parts, n_parts, rs) -> list of n 256-byte proofs, parts = n x n_parts x PART_BYTES;
    rs: n x 64 B (read on the root only) or None (the root draws them);
    device: where the collective's tensors live (cuda:k for nccl, cpu for gloo).
    Returns the proofs on the root, None elsewhere."""
    import sys

    dist = sys.modules.get("torch.distributed")
    if dist is None or not (dist.is_available() and dist.is_initialized()):
        # one process, no collective -- and no torch import: loading torch's runtime libraries into
        # a prover process that never uses them measurably slowed its later host-bound work
        rs = draw_rs(n) if rs is None else rs
        return assemble_fn(b"".join(part_fn(rs)), 1, rs)
    import torch

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device("cpu") if device is None else torch.device(device)
    # the root's (r, s) to every rank: each shard folds them into its augmentation terms
    if rank == root:
        rs = draw_rs(n) if rs is None else rs
        if len(rs) != 64 * n:
            raise ValueError(f"rs must be {64 * n} bytes, got {len(rs)}")
        rs_t = torch.frombuffer(bytearray(rs), dtype=torch.uint8).to(dev)
    else:
        rs_t = torch.empty(64 * n, dtype=torch.uint8, device=dev)
    dist.broadcast(rs_t, src=dist.get_global_rank(group, root) if group is not None else root, group=group)
    rs = bytes(rs_t.cpu().numpy().tobytes())
    parts = part_fn(rs)
    if len(parts) != n or any(len(p) != PART_BYTES for p in parts):
        raise ValueError(f"part_fn must return n parts of {PART_BYTES} bytes")
    mine = torch.frombuffer(bytearray(b"".join(parts)), dtype=torch.uint8).to(dev)
    gathered = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine, group=group)
    if rank != root:
        return None
    # rank-major [world][n][part] -> proof-major [n][world][part]
    stack = torch.stack(gathered).view(world, n, PART_BYTES).transpose(0, 1).contiguous()
    return assemble_fn(bytes(stack.cpu().numpy().tobytes()), world, rs)


class SplitProver:
    """A proving key sharded over the group's ranks (one process per GPU).

    prover = SplitProver(ctx, zkey_bytes)           # every rank, same zkey
    w = prover.upload(wtns)                          # every rank, the full witness
    proofs = prover.prove([w])                       # root: [256 B]; other ranks: None
    """

    def __init__(self, ctx, zkey: bytes, group=None, root: int = 0):
        import torch
        import torch.distributed as dist

        from .native import ProvingKey

        self.ctx, self.group, self.root = ctx, group, root
        if dist.is_available() and dist.is_initialized():
            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
            backend = dist.get_backend(group)
        else:
            self.rank, self.world, backend = 0, 1, "none"
        self.key = ProvingKey(ctx, zkey, shard=self.rank, n_shards=self.world)
        self.device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")

    def upload(self, wtns: bytes):
        return self.key.upload(wtns)

    def prove(self, ws, rs: bytes | None = None):
        return split_prove(lambda r: self.key.prove_part_batch(ws, r),
                           lambda parts, n_parts, r: self.ctx.assemble(parts, n_parts, r),
                           len(ws), rs, self.group, self.device, self.root)

    def close(self):
        self.key.close()
