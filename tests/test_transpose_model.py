"""Host model of the frame-syndrome kernel's butterfly bit transpose
(decode_split.hip wave_transpose32 / transpose_stage): the stage list is read
from the HIP source, and the five stages -- partner lane l ^ s (ds_swizzle xor
mode, within 32-lane halves), a rotate right by s (upper-block lanes) or
32 - s (lower-block lanes) through v_alignbit_b32, and a v_bfi_b32 keeping the
lane's own block -- must give lane 32 h + c bit r = bit c of lane 32 h + r's
input. The GPU parity tests check the kernel's outputs themselves."""
import os
import random
import re

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "qkd_ldpc_amd", "csrc", "decode_split.hip")
M32 = 0xFFFFFFFF


def stages():
    text = open(SRC).read()
    body = text[text.index("uint32_t wave_transpose32("):]
    body = body[:body.index("\n}\n")]
    return [(int(s), int(m, 16)) for s, m in re.findall(r"transpose_stage<(\d+), (0x[0-9A-Fa-f]+)u>", body)]


def rotr(y, r):
    r %= 32
    return ((y >> r) | (y << (32 - r))) & M32


def model(x, st):
    v = list(x)
    for s, mask in st:
        y = [v[l ^ s] for l in range(64)]                       # ds_swizzle, xor s
        out = []
        for l in range(64):
            hi = (l & s) != 0
            ys = rotr(y[l], s if hi else 32 - s)                  # v_alignbit_b32(y, y, r)
            k = (~mask) & M32 if hi else mask
            out.append((v[l] & k) | (ys & ~k & M32))              # v_bfi_b32(k, x, ys)
        v = out
    return v


def test_stage_list_is_the_five_butterflies():
    assert stages() == [(16, 0x0000FFFF), (8, 0x00FF00FF), (4, 0x0F0F0F0F), (2, 0x33333333), (1, 0x55555555)]


def test_model_transposes_each_half():
    st = stages()
    rng = random.Random(5)
    cases = [[rng.getrandbits(32) for _ in range(64)] for _ in range(50)]
    cases += [[1 << (l % 32) for l in range(64)], [M32] * 64, [0] * 64]
    for x in cases:
        v = model(x, st)
        for h in range(2):
            for c in range(32):
                want = sum(((x[32 * h + r] >> c) & 1) << r for r in range(32))
                assert v[32 * h + c] == want


def test_model_is_an_involution():
    # a transpose applied twice gives the input back
    st = stages()
    rng = random.Random(7)
    x = [rng.getrandbits(32) for _ in range(64)]
    assert model(model(x, st), st) == x
