"""The reference's Circom circuits, expressed with the in-repo R1CS builder.

Each function mirrors one Circom template (file:line cited) and returns a ``Builder`` whose
input order matches the template's signal declaration order, so ``public.json`` carries the
same public signals at the same indices the reference harness reads
(e.g. ``tests/full_system_simulation.mjs:914-918`` for sgd_verified).
"""

from __future__ import annotations

from functools import lru_cache

from .r1cs import Builder, add, add_const, const, lc_sum, scale, sub

CHUNK_SIZE = 16


# ---------------------------------------------------------------------------
# Gadgets
# ---------------------------------------------------------------------------
def vector_hash(b: Builder, values):
    """VectorHash(DIM) — src/circuits/training/vector_hash.circom:46-89."""
    values = list(values)
    if len(values) <= CHUNK_SIZE:
        return b.poseidon(values)
    chunks = [b.poseidon(values[i:i + CHUNK_SIZE]) for i in range(0, len(values), CHUNK_SIZE)]
    return b.poseidon(chunks)


def gradient_commitment(b: Builder, gradient, client_id, rnd):
    """GradientCommitment(DIM) — vector_hash.circom:195-218."""
    g = vector_hash(b, gradient)
    meta = b.poseidon([client_id, rnd])
    return b.poseidon([g, meta])


def less_than(b: Builder, n: int, x, y):
    """circomlib LessThan(n): Num2Bits(n+1)(x + 2^n - y), out = 1 - bit[n]."""
    assert n <= 252
    bits = b.num2bits(add_const(sub(x, y), 1 << n), n + 1)
    return sub(const(1), bits[n])


def less_eq_than(b: Builder, n: int, x, y):
    """circomlib LessEqThan(n) = LessThan(n)(x, y + 1)."""
    return less_than(b, n, x, add_const(y, 1))


def merkle_root(b: Builder, leaf, siblings, path_indices):
    """MerkleProofVerifier(DEPTH) up to the final root check — src/circuits/lib/merkle.circom:34-80."""
    h = leaf
    for s, p in zip(siblings, path_indices):
        b.assert_mul(p, sub(const(1), p), {})                    # :58
        left = add(h, b.mul(p, sub(s, h)))                       # :71
        right = add(s, b.mul(p, sub(h, s)))                      # :72
        h = b.poseidon([left, right])
    return h


def batch_merkle_prehashed(b: Builder, root, leaves, siblings, path_indices):
    """BatchMerkleProofPreHashed(N, DEPTH) — merkle.circom:200-220 (root === hashes[DEPTH], :79)."""
    for leaf, sib, pth in zip(leaves, siblings, path_indices):
        b.assert_eq(root, merkle_root(b, leaf, sib, pth))


def clipping_sound(b: Builder, grad_pos, grad_neg, tau_sq, lt_bits: int):
    """VerifyClippingSound(DIM) — sgd_verified.circom:162-203 (LessThan(64)) /
    sgd_step_v5.circom:41-81 (LessThan(128)).  Returns the gradient LCs."""
    norm = {}
    for gp, gn in zip(grad_pos, grad_neg):
        b.assert_mul(gp, gn, {})
        norm = add(norm, add(b.mul(gp, gp), b.mul(gn, gn)))
    valid = less_than(b, lt_bits, norm, add_const(tau_sq, 1))
    b.assert_eq(valid, const(1))
    return [sub(gp, gn) for gp, gn in zip(grad_pos, grad_neg)]


# ---------------------------------------------------------------------------
# Main components
# ---------------------------------------------------------------------------
def poseidon_hash2() -> Builder:
    """PoseidonHash2 as a main component (src/circuits/lib/poseidon.circom:35-44):
    private left/right, public output hash.  BASELINE config 1 (plumbing)."""
    b = Builder("poseidon_hash2")
    out = b.output("hash")
    left = b.input("left")
    right = b.input("right")
    b.bind_output(out, b.poseidon([left, right]))
    return b


def training_step_verified(batch: int = 8, dim: int = 4, depth: int = 3, precision: int = 1000) -> Builder:
    """TrainingStepVerified(BATCH, DIM, DEPTH, PRECISION) — src/circuits/training/sgd_verified.circom:230-313,
    main at :316 = (8, 4, 3, 1000).  Metric circuit M = (128, 4, 7, 1000)."""
    b = Builder(f"sgd_verified_{batch}_{dim}_{depth}_{precision}")
    client_id = b.input("client_id", public=True)
    rnd = b.input("round", public=True)
    root_D = b.input("root_D", public=True)
    root_G = b.input("root_G", public=True)
    root_W = b.input("root_W", public=True)
    tau_sq = b.input("tauSquared", public=True)
    weights = b.input("weights", (dim,))
    exp_sum = b.input("expectedSummedGrad", (dim,))
    remainder = b.input("remainder", (dim,))
    grad_pos = b.input("gradPos", (dim,))
    grad_neg = b.input("gradNeg", (dim,))
    features = b.input("features", (batch, dim))
    labels = b.input("labels", (batch,))
    siblings = b.input("siblings", (batch, depth))
    path_idx = b.input("pathIndices", (batch, depth))

    # STEP 1 weight commitment (:267-272, WeightCommitmentSimple :150-160)
    b.assert_eq(root_W, vector_hash(b, weights))
    # STEP 2 batch membership (:274-292)
    leaves = [vector_hash(b, features[i] + [labels[i]]) for i in range(batch)]
    batch_merkle_prehashed(b, root_D, leaves, siblings, path_idx)
    # STEP 3 clipping (:294-301)
    gradient = clipping_sound(b, grad_pos, grad_neg, tau_sq, 64)
    # STEP 4 gradient correctness (VerifyGradientCorrectness :83-145)
    computed = [{} for _ in range(dim)]
    for i in range(batch):
        pred = lc_sum(b.mul(features[i][j], weights[j]) for j in range(dim))      # DotProduct :40-60
        err = sub(pred, scale(labels[i], precision))                               # SampleGradient :64-78
        for j in range(dim):
            computed[j] = add(computed[j], b.mul(err, features[i][j]))
    divisor = batch * precision
    for j in range(dim):
        b.assert_eq(exp_sum[j], computed[j])                                       # :125-127
        lt = less_than(b, 64, remainder[j], const(divisor))                        # :135-138
        b.assert_eq(lt, const(1))
        b.assert_eq(exp_sum[j], add(scale(gradient[j], divisor), remainder[j]))    # :141
    # STEP 5 gradient commitment (:305-311)
    b.assert_eq(root_G, gradient_commitment(b, gradient, client_id, rnd))
    # clientCheck <== client_id * 0 (:313): constant, no constraint
    return b


def training_step_v5(batch: int = 8, dim: int = 16, depth: int = 7) -> Builder:
    """TrainingStepV5(BATCH, DIM, DEPTH) — src/circuits/training/sgd_step_v5.circom:88-164, main :168 = (8,16,7);
    the circuit of the reference fixture data/test_input_v5.json."""
    b = Builder(f"sgd_step_v5_{batch}_{dim}_{depth}")
    client_id = b.input("client_id", public=True)
    rnd = b.input("round", public=True)
    root_D = b.input("root_D", public=True)
    root_G = b.input("root_G", public=True)
    tau_sq = b.input("tauSquared", public=True)
    grad_pos = b.input("gradPos", (dim,))
    grad_neg = b.input("gradNeg", (dim,))
    features = b.input("features", (batch, dim))
    labels = b.input("labels", (batch,))
    siblings = b.input("siblings", (batch, depth))
    path_idx = b.input("pathIndices", (batch, depth))
    leaves = [vector_hash(b, features[i] + [labels[i]]) for i in range(batch)]
    batch_merkle_prehashed(b, root_D, leaves, siblings, path_idx)
    gradient = clipping_sound(b, grad_pos, grad_neg, tau_sq, 128)
    max_grad = 1 << 30
    for j in range(dim):                                                           # :131-142
        b.assert_eq(less_than(b, 64, grad_pos[j], const(max_grad)), const(1))
        b.assert_eq(less_than(b, 64, grad_neg[j], const(max_grad)), const(1))
    b.assert_eq(less_than(b, 80, tau_sq, const(1 << 60)), const(1))              # :144-147
    b.assert_eq(root_G, gradient_commitment(b, gradient, client_id, rnd))
    return b


def balance_unified(n: int = 8, depth: int = 3, dim: int = 4) -> Builder:
    """BalanceProofUnified(N, DEPTH, MODEL_DIM) — src/circuits/balance/balance_unified.circom:74-180, main :188."""
    b = Builder(f"balance_unified_{n}_{depth}_{dim}")
    b.input("client_id", public=True)
    root = b.input("root", public=True)
    n_pub = b.input("N_public", public=True)
    c0 = b.input("c0", public=True)
    c1 = b.input("c1", public=True)
    features = b.input("features", (n, dim))
    labels = b.input("labels", (n,))
    siblings = b.input("siblings", (n, depth))
    path_idx = b.input("pathIndices", (n, depth))
    for lab in labels:
        b.assert_mul(lab, add_const(lab, -1), {})
    b.assert_eq(lc_sum(labels), c1)
    b.assert_eq(add(c0, c1), n_pub)
    b.assert_eq(n_pub, const(n))
    leaves = [vector_hash(b, features[i] + [labels[i]]) for i in range(n)]
    batch_merkle_prehashed(b, root, leaves, siblings, path_idx)
    return b


def secure_masked_update(dim: int = 4, peers: int = 2) -> Builder:
    """SecureMaskedUpdate(DIM, NUM_PEERS) — src/circuits/secureagg/secure_masked_update.circom:231-343, main :350-360."""
    b = Builder(f"secure_masked_update_{dim}_{peers}")
    client_id = b.input("client_id", public=True)
    rnd = b.input("round", public=True)
    b.input("root_D", public=True)
    root_G = b.input("root_G", public=True)
    b.input("root_W", public=True)
    root_K = b.input("root_K", public=True)
    tau_sq = b.input("tauSquared", public=True)
    masked = b.input("masked_update", (dim,), public=True)
    peer_ids = b.input("peer_ids", (peers,), public=True)
    gradient = b.input("gradient", (dim,))
    master_key = b.input("master_key")
    shared = b.input("shared_keys", (peers,))
    b.assert_eq(root_G, gradient_commitment(b, gradient, client_id, rnd))
    b.assert_eq(root_K, b.poseidon([master_key] + shared))                        # KeyMaterialCommitment :188-200
    norm = lc_sum(b.mul(g, g) for g in gradient)                                  # GradientNormBound :156-180
    b.assert_eq(less_eq_than(b, 128, norm, tau_sq), const(1))
    acc = list(gradient)
    for j in range(peers):
        # PairwiseMaskDerivation :55-98
        lt = less_than(b, 64, client_id, peer_ids[j])
        lt_c = b.mul(lt, client_id)
        lt_p = b.mul(lt, peer_ids[j])
        one_m = sub(const(1), lt)
        om_c = b.mul(one_m, client_id)
        om_p = b.mul(one_m, peer_ids[j])
        min_id = add(lt_c, om_p)
        max_id = add(lt_p, om_c)
        mask = [b.poseidon([shared[j], rnd, min_id, max_id, const(k)]) for k in range(dim)]
        # SignDetermination :106-118 (its own LessThan)
        is_pos = less_than(b, 64, client_id, peer_ids[j])
        # ApplySignedMask :129-146
        sign = add_const(scale(is_pos, 2), -1)
        acc = [add(acc[k], b.mul(sign, mask[k])) for k in range(dim)]
    for k in range(dim):
        b.assert_eq(masked[k], acc[k])
    return b


CIRCUITS = {
    "poseidon_hash2": poseidon_hash2,
    "sgd_verified": training_step_verified,
    "sgd_step_v5": training_step_v5,
    "balance_unified": balance_unified,
    "secure_masked_update": secure_masked_update,
}


@lru_cache(maxsize=None)
def build(name: str, *params) -> Builder:
    """Build (and cache) a circuit by reference name and template parameters."""
    return CIRCUITS[name](*params)
