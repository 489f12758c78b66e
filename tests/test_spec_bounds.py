"""Soundness margins of the speculative iterations (qkd_ldpc_amd/csrc/qkd_spec.h),
derived rather than sampled.

kRefSumAbs: the binary32 intervals must contain the reference's binary64 messages,
so every phi-domain check sum is widened by the largest perturbation the
reference's own roundings can cause (src/qkd_ldpc_algorithm.cpp:220-249):
  * d tanh calls (glibc, e_t ulp each) and d - 1 products + 1 division (0.5 ulp
    each) change the extrinsic product P / t_self by a relative
    (2 d e_t + d) 2^-53 at most, an ABSOLUTE change of the same size of its
    phi-domain sum S = -ln|P / t_self|;
  * atanh (e_a ulp) changes c2b = phi(S) by a relative e_a 2^-52, i.e. S by at
    most e_a 2^-52 max_S phi(S) sinh(S) (computed below; < 1).
e_t and e_a are measured here against 80-bit x87 tanhl / atanhl
(tests/native/libm_ulp.c; glibc documents <= 2 ulp for both on x86_64, and the
sweep finds tanh at 2.15, so the derivation assumes 3 ulp for both).

The exhaustive binary32 sweep of the phi bounds themselves is a GPU test
(tests/test_spec.py::test_phi_bounds_exhaustive)."""
import os
import re
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPEC_H = os.path.join(ROOT, "qkd_ldpc_amd", "csrc", "qkd_spec.h")


def spec_constant(name):
    m = re.search(rf"constexpr float {name} = ([0-9.eE+\-x]+)f;", open(SPEC_H).read())
    assert m, name
    v = m.group(1)
    return float.fromhex(v) if "x" in v else float(v)


def glibc_ulp_errors(tmp_path, points=4_000_000):
    exe = str(tmp_path / "libm_ulp")
    subprocess.check_call(["gcc", "-O2", "-o", exe, os.path.join(ROOT, "tests", "native", "libm_ulp.c"), "-lm"])
    out = subprocess.check_output([exe, str(points)], text=True).split()
    return float(out[1]), float(out[4])


def max_phi_sinh():
    """max over S > 0 of phi(S) sinh(S), phi(S) = -ln tanh(S/2): the factor from a
    relative error of c2b to an absolute error of its phi-domain sum."""
    S = np.concatenate([np.geomspace(1e-12, 1.0, 200000), np.linspace(1.0, 700.0, 2000000)])
    u = np.exp(-S)
    phi = np.log1p(2 * u / -np.expm1(-S))
    return float(np.max(phi * np.sinh(S)))


def test_ref_sum_allowance_covers_reference_roundings(tmp_path, golden_code):
    e_t, e_a = glibc_ulp_errors(tmp_path)
    assert e_t <= 3.0 and e_a <= 3.0, (e_t, e_a)          # the bound the derivation assumes
    d = int(np.diff(golden_code["chk_off"]).max())           # max check degree of the code
    k = max_phi_sinh()
    assert 0.99 < k <= 1.0 + 1e-9, k
    # worst case of the reference's own rounding of one c2b, in nep units of S
    delta = (2 * d * e_t + d) * 2.0 ** -53 + e_a * 2.0 ** -52 * k
    # the same with the assumed 3-ulp bounds instead of the measured maxima
    delta_doc = (2 * d * 3.0 + d) * 2.0 ** -53 + 3.0 * 2.0 ** -52 * k
    allow = spec_constant("kRefSumAbs") * np.log(2.0)           # psi units -> nep
    print(f"glibc max error: tanh {e_t:.3f} ulp, atanh {e_a:.3f} ulp; degree {d}; "
          f"reference perturbation <= {delta:.3g} (3-ulp bounds {delta_doc:.3g}); "
          f"kRefSumAbs = {allow:.3g} nep: headroom x{allow / delta:.1f} (x{allow / delta_doc:.1f})")
    assert allow >= 2 * delta_doc


def test_ref_sum_allowance_in_kernel_degree_buckets():
    """The kernel keeps kRefSumAbs per check, independent of degree, so the bound must
    hold for the largest degree the speculative kernel accepts (DC = 16 at most)."""
    d = 16
    delta_doc = (2 * d * 3.0 + d) * 2.0 ** -53 + 3.0 * 2.0 ** -52
    assert spec_constant("kRefSumAbs") * np.log(2.0) >= 2 * delta_doc
