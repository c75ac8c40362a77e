"""Synthetic federated-client inputs, reproducing the reference harness's generators.

Mirrors ``tests/full_system_simulation.mjs`` (Client class :244-789): the seeded JS LCG
(:118-126, evaluated in IEEE double exactly like V8 so the sequence matches), the private
dataset (:273-303), dataset commitment and Merkle proofs (:139-238, :309-335), the verified
gradient (:511-553), and the input.json objects for sgd_verified (:458-474), balance_unified
(:356-366) and secure_masked_update (:558-637).  All hashes use circomlib Poseidon.
"""

from __future__ import annotations

import math

from .field import R, poseidon_hash

CHUNK_SIZE = 16


class JsLcg:
    """``seededRandom`` / ``randomInt`` of tests/full_system_simulation.mjs:118-126."""

    def __init__(self, seed: int = 12345):
        self.seed = seed

    def random(self, client_id: int = 0) -> float:
        x = float(self.seed) * 1103515245.0 + 12345.0 + float(client_id) * 7919.0
        self.seed = int(x) & 0x7FFFFFFF          # ToInt32 of an integral double, then & mask
        return self.seed / 0x7FFFFFFF

    def randint(self, lo: int, hi: int, client_id: int = 0) -> int:
        return math.floor(self.random(client_id) * (hi - lo + 1)) + lo


def vector_hash(values) -> int:
    vals = [int(v) % R for v in values]
    if len(vals) <= CHUNK_SIZE:
        return poseidon_hash(vals)
    return poseidon_hash([poseidon_hash(vals[i:i + CHUNK_SIZE]) for i in range(0, len(vals), CHUNK_SIZE)])


def gradient_commitment(grad_field, client_id, rnd) -> int:
    return poseidon_hash([vector_hash(grad_field), poseidon_hash([client_id, rnd])])


class MerkleTree:
    """buildMerkleTree (tests/full_system_simulation.mjs:198-223) with the padding kept implicit.

    The reference pads the leaves to 2^depth with Poseidon([0]) and hashes every level.  Here level
    l stores only the nodes above real leaves; any other node is the zero-subtree hash z_l
    (z_0 = Poseidon([0]), z_{l+1} = Poseidon([z_l, z_l])), the value the full tree holds there.
    So depth 16 (BASELINE config 3) costs ~n hashes per level instead of 2^16."""

    def __init__(self, leaves, depth):
        self.depth = depth
        self.zeros = [poseidon_hash([0])]
        for _ in range(depth):
            self.zeros.append(poseidon_hash([self.zeros[-1], self.zeros[-1]]))
        level = list(leaves)
        if len(level) > 1 << depth:
            raise ValueError("more leaves than 2^depth")
        self.levels = [level]
        for lvl in range(depth):
            nxt = []
            for i in range(0, len(level), 2):
                right = level[i + 1] if i + 1 < len(level) else self.zeros[lvl]
                nxt.append(poseidon_hash([level[i], right]))
            self.levels.append(nxt)
            level = nxt

    def node(self, lvl, j):
        level = self.levels[lvl]
        return level[j] if j < len(level) else self.zeros[lvl]

    @property
    def root(self):
        return self.node(self.depth, 0)


def merkle_tree(leaves, depth) -> MerkleTree:
    return MerkleTree(leaves, depth)


def merkle_proof(tree: MerkleTree, idx, depth):
    """getMerkleProof (tests/full_system_simulation.mjs:225-238)."""
    sib, path = [], []
    for lvl in range(depth):
        sib.append(tree.node(lvl, idx ^ 1))
        path.append(idx % 2)
        idx //= 2
    return sib, path


class Client:
    """One federated client (tests/full_system_simulation.mjs:244)."""

    def __init__(self, client_id: int, n: int, dim: int, depth: int, lcg: JsLcg):
        self.id = client_id
        self.n, self.dim, self.depth = n, dim, depth
        feats, labels = [], []
        for i in range(n):                                             # :273-303
            feats.append([lcg.randint(0, 100, client_id * 1000 + i * 10 + j) for j in range(dim)])
            labels.append((i + client_id) % 2)
        self.features, self.labels = feats, labels
        self.c1 = sum(labels)
        self.c0 = n - self.c1
        leaves = [vector_hash(feats[i] + [labels[i]]) for i in range(n)]
        self.tree = merkle_tree(leaves, depth)
        self.root_D = self.tree.root

    def verified_gradient(self, weights, batch, precision):
        """_computeVerifiedGradient (:511-553)."""
        div = batch * precision
        summed = [0] * self.dim
        for i in range(batch):
            pred = sum(self.features[i][j] * weights[j] for j in range(self.dim))
            err = pred - self.labels[i] * precision
            for j in range(self.dim):
                summed[j] += err * self.features[i][j]
        grad = [s // div for s in summed]                                # Math.floor
        rem = [s - q * div for s, q in zip(summed, grad)]
        return grad, summed, rem

    def training_input(self, batch, precision, tau_sq, rnd=1, weights=None):
        """input.json for sgd_verified (:401-477)."""
        weights = list(weights) if weights is not None else [0] * self.dim
        grad, summed, rem = self.verified_gradient(weights, batch, precision)
        gp = [g if g >= 0 else 0 for g in grad]
        gn = [-g if g < 0 else 0 for g in grad]
        root_W = vector_hash(weights)
        root_G = gradient_commitment([g % R for g in grad], self.id, rnd)
        sib, pth = zip(*[merkle_proof(self.tree, i, self.depth) for i in range(batch)])
        inp = {
            "client_id": str(self.id), "round": str(rnd), "root_D": str(self.root_D),
            "root_G": str(root_G), "root_W": str(root_W), "tauSquared": str(tau_sq),
            "weights": [str(w) for w in weights], "expectedSummedGrad": [str(s) for s in summed],
            "remainder": [str(x) for x in rem], "gradPos": [str(x) for x in gp],
            "gradNeg": [str(x) for x in gn],
            "features": [[str(x) for x in row] for row in self.features[:batch]],
            "labels": [str(x) for x in self.labels[:batch]],
            "siblings": [[str(s) for s in row] for row in sib],
            "pathIndices": [[str(p) for p in row] for row in pth],
        }
        return inp, grad

    def balance_input(self):
        """input.json for balance_unified (:340-366)."""
        sib, pth = zip(*[merkle_proof(self.tree, i, self.depth) for i in range(self.n)])
        return {
            "client_id": str(self.id), "root": str(self.root_D), "N_public": str(self.n),
            "c0": str(self.c0), "c1": str(self.c1),
            "features": [[str(x) for x in row] for row in self.features],
            "labels": [str(x) for x in self.labels],
            "siblings": [[str(s) for s in row] for row in sib],
            "pathIndices": [[str(p) for p in row] for row in pth],
        }


def shared_key(i: int, j: int) -> int:
    """Simulated key exchange K_ij = Poseidon(min, max, 12345) (:1321-1336)."""
    return poseidon_hash([min(i, j), max(i, j), 12345])


def pairwise_mask(key, rnd, i, j, dim):
    """derivePairwiseMask (:181-196)."""
    lo, hi = min(i, j), max(i, j)
    return [poseidon_hash([key, rnd, lo, hi, k]) for k in range(dim)]


def secagg_input(client_id, peer_ids, gradient, rnd, tau_sq, root_D, root_W):
    """input.json for secure_masked_update (:558-637): m = g + sum_j sigma_ij r_ij mod r."""
    dim = len(gradient)
    master = poseidon_hash([client_id, 12345])
    keys = [shared_key(client_id, p) for p in peer_ids]
    root_K = poseidon_hash([master] + keys)
    g_field = [g % R for g in gradient]
    masked = list(g_field)
    for p, k in zip(peer_ids, keys):
        m = pairwise_mask(k, rnd, client_id, p, dim)
        sign = 1 if client_id < p else -1
        masked = [(a + sign * b) % R for a, b in zip(masked, m)]
    root_G = gradient_commitment(g_field, client_id, rnd)
    return {
        "client_id": str(client_id), "round": str(rnd), "root_D": str(root_D), "root_G": str(root_G),
        "root_W": str(root_W), "root_K": str(root_K), "tauSquared": str(tau_sq),
        "masked_update": [str(x) for x in masked], "peer_ids": [str(p) for p in peer_ids],
        "gradient": [str(g) for g in g_field], "master_key": str(master),
        "shared_keys": [str(k) for k in keys],
    }


def federated_round(n_clients=8, rnd=1, first_id=1, tau_sq=100000000, batch=8, dim=4, depth=3, precision=1000):
    """One round of the reference simulation (tests/full_system_simulation.mjs:1278-1343) at N clients:
    per client the sgd_verified(batch, dim, depth, precision) input.json (trainAndGenerateProof,
    :401-477) and the SecureMaskedUpdate(dim, N-1) input.json (generateSecureAggregationProof,
    :558-637) built on the gradient the training input commits to, with the pairwise keys of
    :1321-1336.  -> [(training input, secagg input, gradient)] in client order."""
    ids = list(range(first_id, first_id + n_clients))
    out = []
    for cid in ids:
        c = Client(cid, batch, dim, depth, JsLcg(12345 + cid))
        tr, grad = c.training_input(batch, precision, tau_sq, rnd=rnd)
        sa = secagg_input(cid, [j for j in ids if j != cid], grad, rnd, tau_sq, c.root_D, int(tr["root_W"]))
        out.append((tr, sa, grad))
    return out
