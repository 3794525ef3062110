#!/usr/bin/env python3
"""The secp256k1 GLV constants of ecdsa.hip (K1_BETA, K1_GLV_*), derived and checked here.

lambda^3 = 1 (mod n), beta^3 = 1 (mod p), lambda G = (beta Gx, Gy); the rounded-lattice split (g1, g2 = round
2^384 b / n, -b1, -b2 the short basis) gives u = a1 + lambda a2 (mod n) with |a1|, |a2| < 2^128, checked over
random scalars and edge values.  The device multiplies through mn_mul (Montgomery, R = 2^256), so -b1, -b2 and
-lambda are kept times R mod n.  Run: python3 tools/glv_constants.py [--check-source corda_amd/csrc/ecdsa.hip]"""
import random
import re
import sys

P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
LAMBDA = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
BETA = 0x7AE96A2B657C07106E64479EAC3434E99CF0497512F58995C1396C28719501EE
MINUS_B1 = 0xE4437ED6010E88286F547FA90ABFE4C3
MINUS_B2 = (-0x3086D221A7D46BCDE86C90E49284EB15) % N
G1 = 0x3086D221A7D46BCDE86C90E49284EB153DAA8A1471E8CA7FE893209A45DBB031
G2 = 0xE4437ED6010E88286F547FA90ABFE4C4221208AC9DF506C61571B4AE8AC47F71
R = 2**256

CONSTS = {
    "K1_BETA": BETA, "K1_GLV_G1": G1, "K1_GLV_G2": G2, "K1_GLV_MB1R": MINUS_B1 * R % N,
    "K1_GLV_MB2R": MINUS_B2 * R % N, "K1_GLV_MLR": (-LAMBDA) * R % N, "K1_N_HALF": N // 2,
}


def _add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0] and (a[1] + b[1]) % P == 0:
        return None
    if a == b:
        m = 3 * a[0] * a[0] * pow(2 * a[1], -1, P) % P
    else:
        m = (b[1] - a[1]) * pow(b[0] - a[0], -1, P) % P
    x = (m * m - a[0] - b[0]) % P
    return (x, (m * (a[0] - x) - a[1]) % P)


def _mul(k, pt):
    r = None
    while k:
        if k & 1:
            r = _add(r, pt)
        pt = _add(pt, pt)
        k >>= 1
    return r


def split(u):
    """The device's glv_split: (|a1|, neg1, |a2|, neg2) with u = s1 |a1| + lambda s2 |a2| (mod n)."""
    c1 = (u * G1 + (1 << 383)) >> 384
    c2 = (u * G2 + (1 << 383)) >> 384
    r2 = (c1 * MINUS_B1 + c2 * MINUS_B2) % N
    r1 = (r2 * (-LAMBDA) + u) % N
    n1, n2 = r1 > N // 2, r2 > N // 2
    return (N - r1 if n1 else r1), n1, (N - r2 if n2 else r2), n2


def check(samples=20000, seed=1):
    assert pow(LAMBDA, 3, N) == 1 and pow(BETA, 3, P) == 1
    assert _mul(LAMBDA, (GX, GY)) == (BETA * GX % P, GY)
    rng = random.Random(seed)
    edge = [0, 1, 2, N - 1, N - 2, LAMBDA, N - LAMBDA, 2**128, 2**128 - 1, 2**255, N // 2, N // 2 + 1]
    for t in range(samples + len(edge)):
        u = edge[t] if t < len(edge) else rng.randrange(N)
        a1, n1, a2, n2 = split(u)
        assert a1 < 2**128 and a2 < 2**128, hex(u)
        assert ((-a1 if n1 else a1) + LAMBDA * (-a2 if n2 else a2) - u) % N == 0
    return True


def words(v):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def check_source(path):
    src = open(path).read()
    for name, v in CONSTS.items():
        m = re.search(r"%s\[8\]\s*=\s*\{([^}]*)\}" % name, src)
        assert m, name
        got = [int(x.strip().rstrip("u"), 16) for x in m.group(1).split(",") if x.strip()]
        assert got == words(v), (name, [hex(x) for x in got], [hex(x) for x in words(v)])
    return True


if __name__ == "__main__":
    check()
    if len(sys.argv) > 2 and sys.argv[1] == "--check-source":
        check_source(sys.argv[2])
    for name, v in CONSTS.items():
        print(name, ", ".join("0x%08xu" % w for w in words(v)))
