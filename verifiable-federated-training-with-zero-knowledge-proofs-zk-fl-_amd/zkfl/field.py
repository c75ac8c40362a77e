"""BN254 scalar-field constants and the circomlib Poseidon parameter set (host side).

Host-side Fr arithmetic here is plain Python integers: it is used only to *build* circuits,
evaluate witnesses and prepare the dev ceremony — the proving hot path runs in libzkfl (HIP).

Poseidon parameters restate circomlib's ``poseidon_constants`` generation (circomlib ^2.0.5
[ext], used through ``src/circuits/lib/poseidon.circom:17``): Grain LFSR seeded with
(field=1, sbox=0, n=254, t, R_F=8, R_P), self-shrinking output, round constants by rejection
sampling below r, then a Cauchy MDS matrix M[i][j] = 1/(x_i + y_j).
"""

from __future__ import annotations

from functools import lru_cache

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583

POSEIDON_RF = 8
POSEIDON_RP = (56, 57, 56, 60, 60, 63, 64, 63, 60, 66, 60, 65, 70, 60, 64, 68)  # t = 2..17


def fr(x) -> int:
    """Reduce an input value (int / decimal string, negatives allowed) into [0, r)."""
    return int(x) % R


def _grain_stream(t: int, rp: int):
    """Yield the self-shrinking Grain LFSR output bits for a Poseidon instance."""
    seed = 0
    for val, width in ((1, 2), (0, 4), (254, 12), (t, 12), (POSEIDON_RF, 10), (rp, 10)):
        seed = (seed << width) | val
    seed = (seed << 30) | ((1 << 30) - 1)           # 80-bit register, bit 79 = oldest
    reg = seed

    def clock():
        nonlocal reg
        # taps at offsets 0, 13, 23, 38, 51, 62 from the oldest bit (bit 79)
        b = ((reg >> 79) ^ (reg >> 66) ^ (reg >> 56) ^ (reg >> 41) ^ (reg >> 28) ^ (reg >> 17)) & 1
        reg = ((reg << 1) & ((1 << 80) - 1)) | b
        return b

    for _ in range(160):
        clock()
    while True:
        first = clock()
        second = clock()
        if first:
            yield second


@lru_cache(maxsize=None)
def poseidon_params(t: int):
    """(round constants C[(R_F+R_P)*t], MDS M[t][t]) for width t (2..17)."""
    rp = POSEIDON_RP[t - 2]
    bits = _grain_stream(t, rp)

    def draw(nbits=254):
        v = 0
        for _ in range(nbits):
            v = (v << 1) | next(bits)
        return v

    consts = []
    while len(consts) < (POSEIDON_RF + rp) * t:
        v = draw()
        if v < R:
            consts.append(v)
    while True:
        xy = [draw() % R for _ in range(2 * t)]
        if len(set(xy)) < 2 * t:
            continue
        xs, ys = xy[:t], xy[t:]
        if any((a + b) % R == 0 for a in xs for b in ys):
            continue
        mds = tuple(tuple(pow((a + b) % R, R - 2, R) for b in ys) for a in xs)
        return tuple(consts), mds


def poseidon_perm_trace(state):
    """Run the permutation on integer state; return (final_state, sbox_trace) where
    sbox_trace lists (x2, x4, x5) for every S-box in circuit order (full rounds: all t lanes
    left to right; partial rounds: lane 0)."""
    t = len(state)
    C, M = poseidon_params(t)
    rp = POSEIDON_RP[t - 2]
    half = POSEIDON_RF // 2
    st = list(state)
    trace = []
    for rnd in range(POSEIDON_RF + rp):
        st = [(st[i] + C[rnd * t + i]) % R for i in range(t)]
        lanes = range(t) if (rnd < half or rnd >= half + rp) else range(1)
        for i in lanes:
            x = st[i]
            x2 = x * x % R
            x4 = x2 * x2 % R
            x5 = x4 * x % R
            trace.append((x2, x4, x5))
            st[i] = x5
        st = [sum(M[i][j] * st[j] for j in range(t)) % R for i in range(t)]
    return st, trace


def poseidon_hash(inputs) -> int:
    """circomlib Poseidon(n) on integers (state = [0, inputs...], output state[0])."""
    st, _ = poseidon_perm_trace([0] + [fr(x) for x in inputs])
    return st[0]
