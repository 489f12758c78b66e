import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_ROOT = "/root/reference"   # present only in the build container, never on the GPU box


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def probe():
    with open(os.path.join(GOLDEN, "reference_probe.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_code():
    return dict(np.load(os.path.join(GOLDEN, "code_n10240.npz")))


@pytest.fixture(scope="session")
def golden_vectors():
    return dict(np.load(os.path.join(GOLDEN, "oracle_vectors.npz")))


@pytest.fixture(scope="session")
def dense_codes():
    with open(os.path.join(GOLDEN, "dense_codes.json")) as f:
        return {k: np.array(v, np.uint8) for k, v in json.load(f).items()}


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def oracle_code(golden_code, oracle_mod):
    return oracle_mod.Code.from_lists(golden_code)


@pytest.fixture
def qkd_opt():
    """Sets process-wide debug options of the library (qkd_debug_set_option;
    the library reads no environment variable) for one test:
    qkd_opt("QKD_SPEC_CAP", 0); qkd_opt(name, None) restores the default.
    Every option it touched is restored at teardown."""
    import qkd_ldpc_amd as Q
    touched = set()

    def set_opt(name, value=None):
        touched.add(name)
        Q.set_debug_option(name, value)

    yield set_opt
    for name in touched:
        Q.set_debug_option(name, None)


def write_alist(path, n, m, bit_off, bit_idx, chk_off, chk_idx, pad=True):
    """Emit an alist file (1-based, zero-padded rows) from adjacency arrays."""
    dv = np.diff(bit_off)
    dc = np.diff(chk_off)
    with open(path, "w") as f:
        f.write(f"{n} {m}\n{int(dv.max())} {int(dc.max())}\n")
        f.write(" ".join(str(int(x)) for x in dv) + " \n")
        f.write(" ".join(str(int(x)) for x in dc) + " \n")
        for i in range(n):
            row = [int(x) + 1 for x in bit_idx[bit_off[i]:bit_off[i + 1]]]
            if pad:
                row += [0] * (int(dv.max()) - len(row))
            f.write(" ".join(map(str, row)) + " \n")
        for j in range(m):
            row = [int(x) + 1 for x in chk_idx[chk_off[j]:chk_off[j + 1]]]
            if pad:
                row += [0] * (int(dc.max()) - len(row))
            f.write(" ".join(map(str, row)) + " \n")
