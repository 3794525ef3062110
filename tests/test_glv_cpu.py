"""The secp256k1 GLV constants the device's k_ecdsa_comb_q uses (ecdsa.hip K1_BETA / K1_GLV_*): derived and checked
by tools/glv_constants.py — lambda G = (beta Gx, Gy), the split's identity u = a1 + lambda a2 (mod n) and its bound
|a1|, |a2| < 2^128 over random and edge scalars — and the words in the kernel source equal to the derived ones."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import glv_constants as glv  # noqa: E402


def test_glv_split_identity_and_bound():
    assert glv.check(samples=3000, seed=7)


def test_glv_constants_in_kernel_source():
    assert glv.check_source(os.path.join(ROOT, "corda_amd", "csrc", "ecdsa.hip"))


def test_glv_split_edge_values():
    for u in (0, 1, glv.N - 1, glv.LAMBDA, glv.N // 2, glv.N // 2 + 1):
        a1, n1, a2, n2 = glv.split(u)
        assert ((-a1 if n1 else a1) + glv.LAMBDA * (-a2 if n2 else a2) - u) % glv.N == 0
        assert a1 < 2**128 and a2 < 2**128
