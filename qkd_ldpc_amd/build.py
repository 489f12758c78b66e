"""Build the in-tree HIP library: `python -m qkd_ldpc_amd.build [--clean]`.

Compiles qkd_ldpc_amd/csrc/*.{cpp,hip} with hipcc for gfx950 into
qkd_ldpc_amd/lib/libqkd_ldpc_amd.so (git-ignored; it travels to the GPU box
with the source snapshot).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")


def build(clean: bool = False, jobs: int = 4) -> str:
    env = dict(os.environ)
    env.setdefault("HIPCC", "/opt/rocm/bin/hipcc")
    if clean:
        subprocess.check_call(["make", "-C", CSRC, "clean"], env=env)
    subprocess.check_call(["make", "-s", "-C", CSRC, f"-j{jobs}"], env=env)
    # the reference-signature C++ shim (compat/) on top of the C ABI
    subprocess.check_call(["make", "-s", "-C", os.path.join(os.path.dirname(HERE), "compat")], env=env)
    return os.path.join(HERE, "lib", "libqkd_ldpc_amd.so")


if __name__ == "__main__":
    print(build(clean="--clean" in sys.argv))
