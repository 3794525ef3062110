"""GPU check of the ECDSA field / scalar arithmetic (corda_amd/csrc/ec_dev.hpp) against Python
integers, through the test harness tools/libectest.so (tools/ec_field_test.hip).  Operands include
the values that take the rare carry / borrow branches of the redundant-form reductions: 0, 1, p - 1,
p, p + 1, K - 1, K, 2^224 multiples, 2^256 - 1 (K = 2^256 - p), plus seeded random 256-bit values.
Results must be congruent mod p (or mod n for mn_mul) and below 2^256; canon must be < p."""
import ctypes
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = {0: 2**256 - 2**224 + 2**192 + 2**96 - 1, 1: 2**256 - 2**32 - 977}
N = {0: 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551,
     1: 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141}
OPS = {"mul": 0, "sqr": 1, "add": 2, "sub": 3, "inv": 4, "mn_mul": 5, "canon": 6, "mn_inv": 7}


@pytest.fixture(scope="module")
def lib():
    path = os.path.join(ROOT, "tools", "libectest.so")
    if not os.path.exists(path):
        pytest.fail("tools/libectest.so not built (python __graft_entry__.py)")
    L = ctypes.CDLL(path)
    L.ec_field_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]
    return L


def words(vals):
    a = np.zeros((len(vals), 8), dtype=np.uint32)
    for i, v in enumerate(vals):
        for k in range(8):
            a[i, k] = (v >> (32 * k)) & 0xFFFFFFFF
    return a


def ints(a):
    return [sum(int(a[i, k]) << (32 * k) for k in range(8)) for i in range(a.shape[0])]


def run(lib, curve, op, xs, ys):
    a, b = words(xs), words(ys)
    out = np.zeros_like(a)
    assert lib.ec_field_run(curve, OPS[op], len(xs), a.ctypes.data, b.ctypes.data, out.ctypes.data) == 0
    return ints(out)


def operands(curve, n_random=4000, seed=7):
    p = P[curve]
    K = 2**256 - p
    edge = {0, 1, 2, 3, p - 1, p - 2, p, p + 1, p + 2, K - 1, K, K + 1, 2**256 - 1, 2**256 - 2, 2**255,
            2**224, 2**224 - 1, 2**192, 2**96, 2**32, 2**32 - 1, 2**256 - K - 1, 2**256 - 2**224, 7 * 2**224,
            2**256 - 7 * 2**224}
    edge = sorted(v for v in edge if 0 <= v < 2**256)
    rng = random.Random(seed + curve)
    xs, ys = [], []
    for u in edge:
        for v in edge:
            xs.append(u)
            ys.append(v)
    for _ in range(n_random):
        xs.append(rng.getrandbits(256))
        ys.append(rng.getrandbits(256))
    # values just below / above multiples of p inside [0, 2^256)
    for _ in range(500):
        xs.append(p - rng.getrandbits(40) if rng.random() < 0.5 else min(2**256 - 1, p + rng.getrandbits(40)))
        ys.append(2**256 - 1 - rng.getrandbits(rng.choice([8, 32, 200])))
    return xs, ys


@pytest.mark.parametrize("curve", [0, 1])
@pytest.mark.parametrize("op", ["mul", "sqr", "add", "sub"])
def test_field_ops_congruent(lib, curve, op):
    p = P[curve]
    xs, ys = operands(curve)
    got = run(lib, curve, op, xs, ys)
    for x, y, r in zip(xs, ys, got):
        want = {"mul": x * y, "sqr": x * x, "add": x + y, "sub": x - y}[op] % p
        assert 0 <= r < 2**256 and r % p == want, (op, hex(x), hex(y), hex(r))


@pytest.mark.parametrize("curve", [0, 1])
def test_field_inv_and_canon(lib, curve):
    p = P[curve]
    xs, ys = operands(curve, n_random=500)
    xs = [x for x in xs if x % p][:3000]
    got = run(lib, curve, "inv", xs, xs)
    for x, r in zip(xs, got):
        assert r < 2**256 and (r * x) % p == 1, hex(x)
    got = run(lib, curve, "canon", xs, xs)
    for x, r in zip(xs, got):
        assert r == x % p


@pytest.mark.parametrize("curve", [0, 1])
def test_montgomery_scalar_mul(lib, curve):
    n = N[curve]
    R = 2**256
    rinv = pow(R, -1, n)
    rng = random.Random(11 + curve)
    xs = [0, 1, n - 1, n - 2, 2**255 % n] + [rng.randrange(n) for _ in range(3000)]
    ys = [n - 1, 1, n - 1, 2, 1] + [rng.randrange(n) for _ in range(3000)]
    got = run(lib, curve, "mn_mul", xs, ys)
    for x, y, r in zip(xs, ys, got):
        assert r == x * y * rinv % n, (hex(x), hex(y), hex(r))


@pytest.mark.parametrize("curve", [0, 1])
def test_montgomery_scalar_inverse(lib, curve):
    """mn_inv (binary extended Euclid): Montgomery form in and out, (aR)^-1 -> a^-1 R."""
    n = N[curve]
    R = 2**256
    rng = random.Random(13 + curve)
    xs = [1, 2, 3, n - 1, n - 2, 2**255 % n, 2**128, (R * 5) % n] + [rng.randrange(1, n) for _ in range(3000)]
    xs += [1 << k for k in range(0, 256, 7)]
    xs = [x % n for x in xs if x % n]
    got = run(lib, curve, "mn_inv", xs, xs)
    for x, r in zip(xs, got):
        a = x * pow(R, -1, n) % n           # x is the Montgomery form of a
        assert r == pow(a, -1, n) * R % n, hex(x)
