"""Host (g++) builds of the device headers: the bit-exact math restatement
against glibc, and the product key generator against the oracle's full-array
std::shuffle restatement. Same source files the gfx950 kernels compile."""
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _build(tmp_path_factory, name):
    out = str(tmp_path_factory.mktemp("native") / name)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", out,
                           os.path.join(HERE, "native", name + ".cpp")])
    return out


@pytest.fixture(scope="module")
def math_bin(tmp_path_factory):
    return _build(tmp_path_factory, "math_check")


@pytest.fixture(scope="module")
def rng_bin(tmp_path_factory):
    return _build(tmp_path_factory, "rng_check")


@pytest.fixture(scope="module")
def jump_bin(tmp_path_factory):
    return _build(tmp_path_factory, "jump_check")


def test_xoshiro_jump_matrices_equal_stepping(jump_bin):
    """The key generator's jump-ahead (lane l starts at draw l * chunk) equals
    stepping the generator l * chunk times, for several chunks and seeds."""
    assert subprocess.check_output([jump_bin], text=True).strip() == "0"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_math_bit_exact_vs_glibc(math_bin, seed):
    out = subprocess.check_output([math_bin, "400000", str(seed)], text=True)
    last = out.strip().splitlines()[-1].split()
    bad, total = int(last[0]), int(last[1])
    assert total > 5_000_000
    assert bad == 0, out


def test_decoder_argument_ranges_bit_exact(math_bin):
    """Dense sampling of the ranges the decoder actually feeds (|b2c/2| <= 50,
    atanh of extrinsic products in [-1, 1])."""
    out = subprocess.check_output([math_bin, "1500000", "99"], text=True)
    assert out.strip().splitlines()[-1].split()[0] == "0", out


def test_keygen_tracking_equals_full_shuffle(rng_bin, oracle_mod):
    rng = np.random.default_rng(1234)
    cases = []
    for n in (2, 3, 6, 7, 10, 64, 65, 127, 1000, 1001, 10240):
        for q in (0.02, 0.1, 0.5, 1.0):
            if int(n * q) == 0:
                continue
            cases.append((int(rng.integers(0, 2**63)), n, q))
    cases += [(int(s), 10240, 0.08) for s in oracle_mod.seeds(777, 8)]
    stdin = "".join(f"{s} {n} {q!r}\n" for s, n, q in cases)
    out = subprocess.check_output([rng_bin], input=stdin, text=True).strip().splitlines()
    assert len(out) == len(cases)
    for (s, n, q), line in zip(cases, out):
        head, tail = line.split("|")
        vals = head.split()
        got_q = float(vals[0])
        alice = np.array([int(x) for x in vals[1:]])
        flips = [int(x) for x in tail.split()]
        wa, wb, wq = oracle_mod.keygen(s, n, q)
        assert got_q == wq
        assert (alice == wa).all()
        bob = alice.copy()
        bob[flips] ^= 1
        assert len(set(flips)) == len(flips)
        assert (bob == wb).all(), (s, n, q)
