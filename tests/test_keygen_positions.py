"""CPU check of the rule keygen_split_kernel uses for the error positions
(decode.hip kg_resolve_wave): after the forward shuffle (introduce_errors,
qkd_ldpc_algorithm.cpp; std::shuffle's swap a[s] <-> a[x_s], x_s <= s), a[q] for
q < ne is the last step s with x_s = q, and a position no step wrote after
its own step follows the chain back through step q. Restated here in Python
and compared with the shuffle itself on random swap sequences, including the
ne = n and tiny-n edges."""
import random

import pytest


def shuffle_prefix(xs, n, ne):
    a = list(range(n))
    for s in range(1, n):
        a[s], a[xs[s]] = a[xs[s]], a[s]
    return a[:ne]


def resolved_prefix(xs, n, ne):
    last = [0] * ne
    for s in range(1, n):
        if xs[s] < ne:
            last[xs[s]] = max(last[xs[s]], s)

    def resolve(q):
        t, p = q, xs[q]
        while True:
            for st in range(t - 1, max(p, 1) - 1, -1):
                if xs[st] == p:
                    return st
            if p == 0:
                return 0
            t, p = p, xs[p]

    return [last[q] if (last[q] or q == 0) else resolve(q) for q in range(ne)]


@pytest.mark.parametrize("seed", range(6))
def test_resolved_positions_equal_shuffle(seed):
    rnd = random.Random(seed)
    for _ in range(300):
        n = rnd.choice([1, 2, 3, 5, 64, 65, 257, 1000, rnd.randint(1, 3000)])
        ne = rnd.choice([0, 1, n, max(1, n // 50), rnd.randint(0, n)])
        xs = [None] + [rnd.randint(0, s) for s in range(1, n)]
        assert resolved_prefix(xs, n, ne) == shuffle_prefix(xs, n, ne), (seed, n, ne)


def test_rare_positions_are_few_at_config2():
    """~ne^2 / 2N positions need the walk (2 per config-2 frame): the wave-wide
    scan is off the common path."""
    rnd = random.Random(7)
    n, ne, rare = 10240, 204, 0
    for _ in range(20):
        xs = [None] + [rnd.randint(0, s) for s in range(1, n)]
        seen = set(xs[s] for s in range(1, n) if xs[s] < ne)
        rare += sum(1 for q in range(1, ne) if q not in seen)
    assert rare / 20 < 6
