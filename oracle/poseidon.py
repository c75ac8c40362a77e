"""circomlib Poseidon restated on the CPU — TEST INFRASTRUCTURE ONLY (parity oracle).

Reference semantics:
  * ``src/circuits/lib/poseidon.circom:35-96`` (PoseidonHash2/1/N wrap circomlib ``Poseidon(n)``),
    included from circomlib ^2.0.5 [ext, not vendored; package.json:38].
  * Off-circuit twin used by the harness: circomlibjs ``buildPoseidon`` (^0.1.7 [ext]),
    ``tests/full_system_simulation.mjs:134-155``.
Parameters (circomlib): t = nInputs + 1, x^5 S-box, R_F = 8, R_P per t from
``[56,57,56,60,60,63,64,63,60,66,60,65,70,60,64,68]`` (t = 2..17), state = [0, inputs...],
output = state[0].  Round constants and the Cauchy MDS matrix are regenerated with the
Grain LFSR of the Poseidon reference parameter script (field=1, sbox=0, n=254 bits),
which is how circomlib's ``poseidon_constants`` were produced.  The regeneration is
pinned by the reference fixture ``data/test_input_v5.json`` (root_G, leaves, root_D;
SURVEY.md Appendix B) and the public circomlibjs vectors.
"""

from __future__ import annotations

from functools import lru_cache

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
N_ROUNDS_F = 8
N_ROUNDS_P = [56, 57, 56, 60, 60, 63, 64, 63, 60, 66, 60, 65, 70, 60, 64, 68]


class _Grain:
    def __init__(self, t: int, rf: int, rp: int, n: int = 254):
        bits = []
        for val, width in ((1, 2), (0, 4), (n, 12), (t, 12), (rf, 10), (rp, 10)):
            bits += [int(c) for c in bin(val)[2:].zfill(width)]
        bits += [1] * 30
        self.s = bits
        for _ in range(160):
            self._clock()

    def _clock(self):
        s = self.s
        nb = s[62] ^ s[51] ^ s[38] ^ s[23] ^ s[13] ^ s[0]
        s.pop(0)
        s.append(nb)
        return nb

    def bit(self):
        # self-shrinking: draw pairs (a, b); output b when a == 1
        while True:
            a = self._clock()
            b = self._clock()
            if a == 1:
                return b

    def bits_int(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | self.bit()
        return v

    def field_elem(self, n: int = 254) -> int:
        while True:
            v = self.bits_int(n)
            if v < R:
                return v


@lru_cache(maxsize=None)
def constants(t: int):
    """Return (C list of (R_F+R_P)*t round constants, M t x t) for width t."""
    rp = N_ROUNDS_P[t - 2]
    g = _Grain(t, N_ROUNDS_F, rp)
    C = [g.field_elem() for _ in range((N_ROUNDS_F + rp) * t)]
    while True:
        vals = [g.bits_int(254) % R for _ in range(2 * t)]
        if len(set(vals)) != 2 * t:
            continue
        xs, ys = vals[:t], vals[t:]
        if any((x + y) % R == 0 for x in xs for y in ys):
            continue
        M = [[pow((xs[i] + ys[j]) % R, -1, R) for j in range(t)] for i in range(t)]
        return C, M


def permute(state):
    t = len(state)
    C, M = constants(t)
    rp = N_ROUNDS_P[t - 2]
    half = N_ROUNDS_F // 2
    st = [x % R for x in state]
    for r in range(N_ROUNDS_F + rp):
        st = [(st[i] + C[r * t + i]) % R for i in range(t)]
        if r < half or r >= half + rp:
            st = [pow(x, 5, R) for x in st]
        else:
            st[0] = pow(st[0], 5, R)
        st = [sum(M[i][j] * st[j] for j in range(t)) % R for i in range(t)]
    return st


def poseidon(inputs):
    """circomlib Poseidon(n): hash of 1..16 field elements."""
    ins = [int(x) % R for x in inputs]
    assert 1 <= len(ins) <= 16
    return permute([0] + ins)[0]


# ---- reference helpers (tests/full_system_simulation.mjs:139-238) ----------
CHUNK_SIZE = 16


def vector_hash(values):
    """``vectorHash`` (tests/full_system_simulation.mjs:139-155) == VectorHash(DIM)
    (src/circuits/training/vector_hash.circom:46-89)."""
    vals = [int(v) % R for v in values]
    if len(vals) <= CHUNK_SIZE:
        return poseidon(vals)
    chunks = [poseidon(vals[i:i + CHUNK_SIZE]) for i in range(0, len(vals), CHUNK_SIZE)]
    return poseidon(chunks)


def gradient_commitment(grad_field, client_id, rnd):
    """``gradientCommitment`` (:159-164) == GradientCommitment (vector_hash.circom:195-218)."""
    return poseidon([vector_hash(grad_field), poseidon([client_id, rnd])])


def weight_commitment(weights):
    """``weightCommitment`` (:168-170) == WeightCommitmentSimple (sgd_verified.circom:150-160)."""
    return vector_hash(weights)


def build_merkle_tree(leaf_hashes, depth):
    """``buildMerkleTree`` (:198-223): pad with Poseidon([0]), hash pairs bottom-up."""
    zero = poseidon([0])
    leaves = list(leaf_hashes) + [zero] * ((1 << depth) - len(leaf_hashes))
    tree = [leaves]
    cur = leaves
    while len(cur) > 1:
        cur = [poseidon([cur[i], cur[i + 1]]) for i in range(0, len(cur), 2)]
        tree.append(cur)
    return tree


def merkle_proof(tree, idx, depth):
    """``getMerkleProof`` (:225-238)."""
    sib, path = [], []
    for level in range(depth):
        sib.append(tree[level][idx ^ 1])
        path.append(idx % 2)
        idx //= 2
    return sib, path


def merkle_root_from_path(leaf, siblings, path_indices):
    """MerkleProofVerifier (src/circuits/lib/merkle.circom:34-80) evaluated off-circuit."""
    h = leaf
    for s, b in zip(siblings, path_indices):
        h = poseidon([s, h]) if int(b) else poseidon([h, s])
    return h
