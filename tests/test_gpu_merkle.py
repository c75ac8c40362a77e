"""GPU Poseidon / vectorHash / Merkle trees (zkfl_poseidon_batch, zkfl_vector_hash_batch,
zkfl_merkle_build, zkfl_dataset_commit) vs the oracle and the reference fixture — MI355X (-m gpu).

Bar: bit-exact.  Reference behaviour: tests/full_system_simulation.mjs:139-238 (vectorHash,
buildMerkleTree with Poseidon([0]) padding, getMerkleProof) and :309-335 (computeDatasetCommitment).
Pinned by data/test_input_v5.json (tests/golden/): its 8 leaves (16 features + label = 17 values,
the chunked vectorHash path), its Merkle paths and root_D.  At 2^20 leaves the tree is checked by
a size-independent property: sampled nodes of every level equal Poseidon(their two GPU children)
on the CPU oracle, the top levels are recomputed whole, and padding nodes equal the zero-subtree
hashes.
"""
import json
import os
import random

import pytest

from oracle import poseidon as op

pytestmark = pytest.mark.gpu

R = op.R
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_poseidon_every_arity_matches_oracle(gpu_ctx):
    rnd = random.Random(1)
    for arity in range(1, 17):
        rows = [[rnd.randrange(R) for _ in range(arity)] for _ in range(5)]
        rows.append([0] * arity)
        rows.append([R - 1] * arity)
        assert gpu_ctx.poseidon_batch(rows) == [op.poseidon(r) for r in rows], arity
    # circomlibjs vectors
    assert gpu_ctx.poseidon_batch([[1, 2]]) == [
        7853200120776062878684798364095072458815029376092732009249414926327459813530]
    assert gpu_ctx.poseidon_batch([[0]]) == [
        19014214495641488759237505126948346942972912379615652741039992445865937985820]


def test_poseidon_batch_large_and_ragged_counts(gpu_ctx):
    rnd = random.Random(2)
    for n in (1, 63, 64, 65, 1000, 4097):
        rows = [[rnd.randrange(R), rnd.randrange(R)] for _ in range(n)]
        got = gpu_ctx.poseidon_batch(rows)
        for i in {0, n // 2, n - 1}:
            assert got[i] == op.poseidon(rows[i])


def test_vector_hash_lengths(gpu_ctx):
    rnd = random.Random(3)
    for ln in (1, 5, 16, 17, 31, 32, 33, 100, 256):
        vecs = [[rnd.randrange(R) for _ in range(ln)] for _ in range(3)]
        assert gpu_ctx.vector_hash_batch(vecs) == [op.vector_hash(v) for v in vecs], ln


def test_fixture_leaves_paths_and_root(gpu_ctx):
    """data/test_input_v5.json holds the first 8 samples of a larger committed dataset
    (scripts/generate_test_data_v5.mjs:55-128): leaf i = vectorHash(features[i] || label[i]) (17
    values) must equal the fixture's level-0 siblings, the GPU tree over those 8 leaves its level-1
    and level-2 siblings, and hashing the subtree root up the fixture's remaining siblings on the GPU
    must give root_D."""
    d = json.load(open(os.path.join(GOLDEN, "test_input_v5.json")))
    samples = [[int(x) for x in f] + [int(lab)] for f, lab in zip(d["features"], d["labels"])]
    sib = [[int(s) for s in row] for row in d["siblings"]]
    depth = len(sib[0])
    leaves = gpu_ctx.vector_hash_batch(samples)
    tree8 = gpu_ctx.merkle_build(leaves, 3)
    assert tree8 == gpu_ctx.dataset_commit(samples, 3)
    for i in range(8):
        assert [int(p) for p in d["pathIndices"][i]][:3] == [(i >> lvl) & 1 for lvl in range(3)]
        for lvl in range(3):
            assert tree8[lvl][(i >> lvl) ^ 1] == sib[i][lvl], (i, lvl)
    h = tree8[3][0]
    for lvl in range(3, depth):            # sample 0's path: pathIndices 0 above the batch subtree
        h = gpu_ctx.poseidon_batch([[h, sib[0][lvl]]])[0]
    assert h == int(d["root_D"])
    # the same 8 samples committed alone at depth 7 (Poseidon([0]) padding): the oracle's tree
    assert gpu_ctx.dataset_commit(samples, depth) == op.build_merkle_tree(leaves, depth)


@pytest.mark.parametrize("n,depth", [(0, 3), (1, 0), (1, 4), (5, 3), (8, 3), (300, 9), (513, 10), (1000, 12)])
def test_merkle_shapes_match_oracle(gpu_ctx, n, depth):
    """Edge shapes: empty dataset, depth 0, odd counts, a full tree, the level-launch / fused-top
    switch (512 live nodes), and a tree with more padding than leaves."""
    rnd = random.Random(n * 31 + depth)
    leaves = [rnd.randrange(R) for _ in range(n)]
    assert gpu_ctx.merkle_build(leaves, depth) == op.build_merkle_tree(leaves, depth)


def test_merkle_errors(gpu_ctx):
    from zkfl import native
    with pytest.raises(native.ZkflError) as e:
        gpu_ctx.merkle_build([1] * 9, 3)           # more leaves than 2^depth
    assert e.value.code == -1
    with pytest.raises(native.ZkflError) as e:
        gpu_ctx.merkle_build([R], 2)               # a leaf >= r
    assert e.value.code == -1
    with pytest.raises(native.ZkflError):
        gpu_ctx.poseidon_batch([[1] * 17])         # arity > 16
    with pytest.raises(native.ZkflError):
        gpu_ctx.merkle_build([1], 31)              # beyond ZKFL_MERKLE_MAX_DEPTH


def test_large_tree_local_consistency(gpu_ctx):
    """2^20 - 3 leaves, depth 21: every sampled node of every level equals Poseidon of its two GPU
    children (padding child = zero-subtree hash), the top 6 levels are recomputed whole on the CPU,
    and pure-padding nodes are the zero hashes."""
    n, depth = (1 << 20) - 3, 21
    rnd = random.Random(20)
    leaves = [rnd.randrange(R) for _ in range(n)]
    tree = gpu_ctx.merkle_build(leaves, depth)
    assert tree[0][:n] == leaves
    zeros = [op.poseidon([0])]
    for _ in range(depth):
        zeros.append(op.poseidon([zeros[-1], zeros[-1]]))
    for lvl in range(1, depth + 1):
        width = len(tree[lvl])
        live = -(-n // (1 << lvl))
        for j in {0, live - 1, min(width - 1, live)} | {rnd.randrange(live) for _ in range(6)}:
            assert tree[lvl][j] == op.poseidon([tree[lvl - 1][2 * j], tree[lvl - 1][2 * j + 1]]), (lvl, j)
        if live < width:
            assert tree[lvl][width - 1] == zeros[lvl]
    top = op.build_merkle_tree(tree[depth - 6], 6)
    assert [tree[depth - 6 + k] for k in range(7)] == top
