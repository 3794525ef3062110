#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Sources of truth, per fixture:
  * OpenSSL 3.0.2 (tools/cordagen.c) signs and verifies every canonical case; its verdict is
    recorded as `openssl` and must equal `expected` wherever the reference semantics agree with
    OpenSSL (canonical inputs).
  * The reference's own deterministic test material: TestConstants.kt:27-72
    (entropyToKeyPair(20..100) -> seed = BigInteger.toByteArray() right-padded to 32 bytes,
    Crypto.kt:828-834) and X509EdDSAEngineTest.kt:27-60 (SEED 20170920, 2000 bytes from
    java.util.Random(SEED), restated below).
  * i2p/BC-specific cases where OpenSSL disagrees (S >= L, slide() carry drop, small-order and
    non-canonical keys, DER non-minimal integers) carry `expected` from the construction and
    are marked `unpinned` where no reference test covers them.
  * Tx-id vectors use Python hashlib only (independent of oracle/ and of the GPU path).
Re-run:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cordagen as G  # noqa: E402

P = 2**255 - 19
L = G.L_ED


def java_random_bytes(seed, n):
    """java.util.Random(seed).nextBytes(n) — the LCG specified in the Java SE API."""
    mask = (1 << 48) - 1
    s = (seed ^ 0x5DEECE66D) & mask
    out = bytearray()

    def next_int():
        nonlocal s
        s = (s * 0x5DEECE66D + 0xB) & mask
        v = s >> 16
        return v - (1 << 32) if v >= (1 << 31) else v

    while len(out) < n:
        r = next_int()
        for _ in range(min(n - len(out), 4)):
            out.append(r & 0xFF)
            r >>= 8
    return bytes(out)


def entropy_seed(v: int) -> bytes:
    """BigInteger.valueOf(v).toByteArray().copyOf(32) (Crypto.kt:830)."""
    b = v.to_bytes((v.bit_length() + 8) // 8, "big", signed=True)
    return (b + bytes(32))[:32]


def slide_drops(s: int) -> int:
    """Independent Python restatement of i2p GroupElement.slide(): dropped carries."""
    r = [(s >> i) & 1 for i in range(256)]
    drops = 0
    for i in range(256):
        if not r[i]:
            continue
        for b in range(1, 7):
            if i + b >= 256:
                break
            if not r[i + b]:
                continue
            if r[i] + (r[i + b] << b) <= 15:
                r[i] += r[i + b] << b
                r[i + b] = 0
            elif r[i] - (r[i + b] << b) >= -15:
                r[i] -= r[i + b] << b
                k = i + b
                while k < 256:
                    if not r[k]:
                        r[k] = 1
                        break
                    r[k] = 0
                    k += 1
                if k == 256:
                    drops += 1
            else:
                break
    return drops


def clamp_scalar(seed: bytes) -> int:
    h = bytearray(hashlib.sha512(seed).digest()[:32])
    h[0] &= 248
    h[31] &= 127
    h[31] |= 64
    return int.from_bytes(h, "little")


def ed_case(label, spki, sig, msg, expected, source, unpinned=False, msg_repeat=None):
    """msg_repeat=(pattern, count) stores a long message compactly (the test expands it)."""
    d = dict(label=label, spki=spki.hex(), sig=sig.hex(), expected=expected, source=source, unpinned=unpinned,
             openssl=G.ossl_verify(spki, sig, msg) if sig and msg else None)
    if msg_repeat:
        d["msg_repeat"] = [msg_repeat[0].hex(), msg_repeat[1]]
    else:
        d["msg"] = msg.hex()
    return d


def ed25519_cases():
    cases = []
    msg = b"corda\x00\x00\x01" + hashlib.sha256(b"golden-msg").digest() * 6
    # reference deterministic keys (TestConstants.kt:27-72)
    for v in (20, 30, 40, 50, 60, 70, 80, 90, 100):
        seed = entropy_seed(v)
        a = G.ed25519_pub(seed)
        sig = G.ed25519_sign(seed, msg)
        cases.append(ed_case("entropyToKeyPair(%d)" % v, G.spki_ed25519(a), sig, msg, 0, "TestConstants.kt:27-72"))
        bad = bytearray(sig)
        bad[0] ^= 1   # signedData[0]++ style corruption (CryptoUtilsTest.kt:123-286)
        cases.append(ed_case("entropyToKeyPair(%d) R corrupted" % v, G.spki_ed25519(a), bytes(bad), msg, 1,
                             "CryptoUtilsTest.kt:123-286"))
    # X509EdDSAEngineTest: SEED, 2000 random bytes from java.util.Random(SEED)
    for sd in (20170920, 20170921):
        seed = entropy_seed(sd)
        data = java_random_bytes(20170920, 2000)
        a = G.ed25519_pub(seed)
        sig = G.ed25519_sign(seed, data)
        cases.append(ed_case("X509EdDSAEngineTest seed %d" % sd, G.spki_ed25519(a), sig, data, 0,
                             "X509EdDSAEngineTest.kt:27-75"))
    # 100 zero bytes and 1 MB messages (CryptoUtilsTest full process)
    seed = entropy_seed(70)
    a = G.ed25519_pub(seed)
    for pat, cnt in ((bytes(100), 1), (bytes(range(256)), 4096)):
        m = pat * cnt
        cases.append(ed_case("message len %d" % len(m), G.spki_ed25519(a), G.ed25519_sign(seed, m), m, 0,
                             "CryptoUtilsTest.kt:123-286", msg_repeat=(pat, cnt)))
    # doVerify argument checks (Crypto.kt:528-529) and engine length check
    sig = G.ed25519_sign(seed, msg)
    cases.append(ed_case("empty signature", G.spki_ed25519(a), b"", msg, 3, "Crypto.kt:528"))
    cases.append(ed_case("empty clear data", G.spki_ed25519(a), sig, b"", 4, "Crypto.kt:529"))
    cases.append(ed_case("signature 63 bytes", G.spki_ed25519(a), sig[:63], msg, 2, "i2p engineVerify length"))
    cases.append(ed_case("signature 65 bytes", G.spki_ed25519(a), sig + b"\x00", msg, 2, "i2p engineVerify length"))
    # unsupported key algorithm (RSA SPKI prefix) and a key that is not a curve point
    rsa_spki = bytes.fromhex("30820122300d06092a864886f70d01010105000382010f00") + bytes(270)
    cases.append(ed_case("RSA key -> unsupported", rsa_spki, sig, msg, 5, "Crypto.kt:263-267"))
    y = 2
    while True:   # smallest y with no square root for x
        u = (y * y - 1) % P
        v = (G_D * y * y + 1) % P
        x2 = u * pow(v, P - 2, P) % P
        if pow(x2, (P - 1) // 2, P) not in (0, 1):
            break
        y += 1
    cases.append(ed_case("key not on curve (y=%d)" % y, G.spki_ed25519(y.to_bytes(32, "little")), sig, msg, 6,
                         "i2p GroupElement decode"))
    # S + L: i2p 0.2.0 has no S < L check (CVE-2020-36843) -> VALID; OpenSSL rejects
    S = int.from_bytes(sig[32:], "little")
    for k in (1, 2, 3):
        s2 = S + k * L
        if s2 < 2**256:
            exp = 0 if slide_drops(s2) == 0 else 1
            cases.append(ed_case("S + %dL" % k, G.spki_ed25519(a), sig[:32] + s2.to_bytes(32, "little"), msg, exp,
                                 "i2p 0.2.0 no S<L check", unpinned=True))
    # S >= 2^255: multiples S + kL whose slide() recoding drops a carry (effective scalar
    # S + kL - 2^256 -> INVALID) or does not (-> VALID), over several signatures
    found_drop = found_nodrop = 0
    for j in range(200):
        if found_drop >= 4 and found_nodrop >= 3:
            break
        mj = msg + struct.pack(">I", j)
        sj = G.ed25519_sign(seed, mj)
        Sj = int.from_bytes(sj[32:], "little")
        for k in range(8, 20):
            s2 = Sj + k * L
            if s2 >= 2**256:
                break
            if s2 < 2**255:
                continue
            d = slide_drops(s2)
            if d and found_drop < 4:
                found_drop += 1
                cases.append(ed_case("S + %dL >= 2^255 with slide carry drop (msg %d)" % (k, j), G.spki_ed25519(a),
                                     sj[:32] + s2.to_bytes(32, "little"), mj, 1, "i2p slide() carry drop",
                                     unpinned=True))
            elif not d and found_nodrop < 3:
                found_nodrop += 1
                cases.append(ed_case("S + %dL >= 2^255 no carry drop (msg %d)" % (k, j), G.spki_ed25519(a),
                                     sj[:32] + s2.to_bytes(32, "little"), mj, 0, "i2p slide()", unpinned=True))
    # identity key (small order 1) forgeries: R = [S]B for any S -> VALID in i2p
    ident = bytes([1] + [0] * 31)
    for j, s_seed in enumerate([b"f1", b"f2"]):
        sd = hashlib.sha256(s_seed).digest()
        R = G.ed25519_pub(sd)
        s = clamp_scalar(sd)
        cases.append(ed_case("identity key forgery %d" % j, G.spki_ed25519(ident), R + s.to_bytes(32, "little"), msg,
                             0, "no small-order check (Crypto.kt:874-924 unused)", unpinned=True))
    # non-canonical encodings of the identity key: y = 1 + p, and x = 0 with the sign bit set
    sd = hashlib.sha256(b"f3").digest()
    R = G.ed25519_pub(sd)
    s = clamp_scalar(sd)
    noncanon_1 = (1 + P).to_bytes(32, "little")
    signed_0 = bytes([1] + [0] * 30 + [0x80])
    cases.append(ed_case("key y = 1 + p (non-canonical)", G.spki_ed25519(noncanon_1), R + s.to_bytes(32, "little"),
                         msg, 0, "i2p decode tolerates y >= p; h over canonical Abyte", unpinned=True))
    cases.append(ed_case("key x = 0 with sign bit", G.spki_ed25519(signed_0), R + s.to_bytes(32, "little"), msg, 0,
                         "i2p decode tolerates -0", unpinned=True))
    # non-canonical R: identity as y = 1 + p with identity key and S = 0 -> canonical(R') != R
    cases.append(ed_case("R non-canonical (1 + p)", G.spki_ed25519(ident), noncanon_1 + bytes(32), msg, 1,
                         "bytewise compare with canonical encode", unpinned=True))
    cases.append(ed_case("R canonical identity, S = 0", G.spki_ed25519(ident), ident + bytes(32), msg, 0,
                         "identity key, S = 0", unpinned=True))
    cases.append(ed_case("all-zero signature", G.spki_ed25519(ident), bytes(64), msg, 1, "R = 00.. (y = 0)",
                         unpinned=True))
    # order-4 key (y = 0) and order-2 key (y = -1): decodes fine, arithmetic decides
    for lab, enc in (("order-4 key (y=0)", bytes(32)), ("order-2 key (y=-1)", (P - 1).to_bytes(32, "little"))):
        cases.append(ed_case(lab + " with random sig", G.spki_ed25519(enc), sig, msg, 1, "no small-order check",
                             unpinned=True))
    return cases


G_D = (-121665 * pow(121666, P - 2, P)) % P


def txid_reference(salt, groups):
    """hashlib-only restatement of WireTransaction.id (WireTransaction.kt:139-189)."""
    def sha(b):
        return hashlib.sha256(b).digest()

    def merkle(leaves):
        n = 1
        while n < len(leaves):
            n *= 2
        lvl = list(leaves) + [bytes(32)] * (n - len(leaves))
        while len(lvl) > 1:
            lvl = [sha(lvl[i] + lvl[i + 1]) for i in range(0, len(lvl), 2)]
        return lvl[0]

    present = {g: comps for g, comps in groups}
    maxg = max(present)
    tops = []
    for g in range(maxg + 1):
        if g in present:
            leaves = []
            for i, c in enumerate(present[g]):
                nonce = sha(sha(salt + struct.pack(">ii", g, i)))
                leaves.append(sha(sha(nonce + c)))
            tops.append(merkle(leaves))
        else:
            tops.append(b"\xff" * 32)
    return merkle(tops)


def txid_cases():
    cases = []
    rng = G.PRNG(0xC0DA, b"txid")
    def rb(n):
        return rng.bytes(n)
    shapes = [
        ("issue: outputs, commands, notary", [(1, [rb(640)]), (2, [rb(320)]), (4, [rb(384)])]),
        ("move: inputs, outputs, commands, notary", [(0, [rb(96), rb(96)]), (1, [rb(640), rb(640)]), (2, [rb(320)]),
                                                      (4, [rb(384)])]),
        ("cfg4 profile (6 groups, 8 components)", [(0, [rb(96), rb(96)]), (1, [rb(640), rb(640)]), (2, [rb(320)]),
                                                   (3, [rb(96)]), (4, [rb(384)]), (5, [rb(96)])]),
        ("single component (1-leaf tree = leaf)", [(0, [rb(1)])]),
        ("odd group sizes 3 and 5", [(0, [rb(10), rb(20), rb(30)]), (1, [rb(5)] * 5)]),
        ("unknown group ordinal 20 (CompatibleTransactionTests.kt:151-164)", [(0, [rb(40)]), (2, [rb(50)]),
                                                                               (20, [rb(60)])]),
        ("group order of insertion irrelevant (sorted here)", [(1, [rb(33)]), (3, [rb(64)])]),
        ("component lengths around SHA block edges", [(0, [rb(n) for n in (0, 22, 23, 55, 56, 64, 87, 88, 119, 120)])]),
        ("large component 64 KB", [(1, [rb(1 << 16)])]),
        ("max group ordinal 63", [(63, [rb(8)])]),
    ]
    for label, groups in shapes:
        salt = rb(32)
        cases.append(dict(label=label, salt=salt.hex(), groups=[[g, [c.hex() for c in comps]] for g, comps in groups],
                          id=txid_reference(salt, groups).hex()))
    return cases


# ---------------- ECDSA (BC 1.57 SHA256withECDSA) ----------------
EC = {
    G.SCHEME_R1: dict(p=0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF, n=G.N_R1,
                      a=-3, b=0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B,
                      g=(0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
                         0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5)),
    G.SCHEME_K1: dict(p=2**256 - 2**32 - 977, n=G.N_K1, a=0, b=7,
                      g=(0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
                         0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)),
}


def ec_add(c, P1, P2):
    p = c["p"]
    if P1 is None:
        return P2
    if P2 is None:
        return P1
    (x1, y1), (x2, y2) = P1, P2
    if x1 == x2:
        if (y1 + y2) % p == 0:
            return None
        lam = (3 * x1 * x1 + c["a"]) * pow(2 * y1, -1, p) % p
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, p) % p
    x3 = (lam * lam - x1 - x2) % p
    return (x3, (lam * (x1 - x3) - y1) % p)


def ec_mul(c, k, P):
    R = None
    for bit in bin(k)[2:]:
        R = ec_add(c, R, R)
        if bit == "1":
            R = ec_add(c, R, P)
    return R


def ec_spki(scheme, P, compressed=False):
    if compressed:
        pt = bytes([2 + (P[1] & 1)]) + P[0].to_bytes(32, "big")
        pfx = bytes.fromhex("3039301306072a8648ce3d020106082a8648ce3d030107032200") if scheme == G.SCHEME_R1 else \
            bytes.fromhex("3036301006072a8648ce3d020106052b8104000a032200")
        return pfx + pt
    return G.spki_ec(scheme, b"\x04" + P[0].to_bytes(32, "big") + P[1].to_bytes(32, "big"))


def ec_case(label, spki, sig, msg, expected, source, unpinned=False):
    return dict(label=label, spki=spki.hex(), sig=sig.hex(), msg=msg.hex(), expected=expected, source=source,
                unpinned=unpinned, openssl=G.ossl_verify(spki, sig, msg) if sig and msg else None)


def ecdsa_cases():
    cases = []
    msg = b"corda\x00\x00\x01" + hashlib.sha256(b"golden-ec").digest() * 6
    for scheme, name in ((G.SCHEME_R1, "r1"), (G.SCHEME_K1, "k1")):
        c = EC[scheme]
        n = c["n"]
        d = int.from_bytes(hashlib.sha256(b"ec-golden-key" + name.encode()).digest(), "big") % (n - 1) + 1
        pub = G.ec_pub(scheme, d.to_bytes(32, "big"))
        P = (int.from_bytes(pub[1:33], "big"), int.from_bytes(pub[33:], "big"))
        assert ec_mul(c, d, c["g"]) == P
        spki = G.spki_ec(scheme, pub)
        k = hashlib.sha256(b"nonce" + name.encode()).digest()
        der, rb, sb = G.ec_sign(scheme, d.to_bytes(32, "big"), k, msg)
        r, s_ = int.from_bytes(rb, "big"), int.from_bytes(sb, "big")
        src = "CryptoUtilsTest.kt:123-286 (%s full process)" % name
        cases.append(ec_case("%s valid" % name, spki, der, msg, 0, src))
        cases.append(ec_case("%s valid, compressed key" % name, ec_spki(scheme, P, True), der, msg, 0,
                             "BC decodePoint compressed"))
        cases.append(ec_case("%s 100 zero-byte message" % name, spki,
                             G.ec_sign(scheme, d.to_bytes(32, "big"), k, bytes(100))[0], bytes(100), 0, src))
        cases.append(ec_case("%s message changed" % name, spki, der, msg + b"x", 1, src))
        cases.append(ec_case("%s r+1" % name, spki, G.der_sig(r + 1 if r + 1 < n else r - 1, s_), msg, 1, src))
        cases.append(ec_case("%s high-s (n - s) is valid in BC" % name, spki, G.der_sig(r, n - s_), msg, 0,
                             "ECDSASigner.verifySignature has no low-s rule"))
        cases.append(ec_case("%s r = 0" % name, spki, G.der_sig(0, s_), msg, 1, "r in [1, n-1]"))
        cases.append(ec_case("%s s = 0" % name, spki, G.der_sig(r, 0), msg, 1, "s in [1, n-1]"))
        cases.append(ec_case("%s r = n" % name, spki, G.der_sig(n, s_), msg, 1, "r in [1, n-1]"))
        cases.append(ec_case("%s s = n + s" % name, spki, G.der_sig(r, n + s_), msg, 1, "s in [1, n-1]"))
        rneg = b"\x02\x20" + (r | (1 << 255)).to_bytes(32, "big")   # top bit set, no 00 pad: negative INTEGER
        body = rneg + G.der_encode_int(s_)
        cases.append(ec_case("%s negative r (two's complement)" % name, spki, b"\x30" + bytes([len(body)]) + body, msg,
                             1, "BigInteger negative -> r < 1"))
        big = b"\x02\x21\x01" + r.to_bytes(32, "big")   # 2^256 + r
        body = big + G.der_encode_int(s_)
        cases.append(ec_case("%s r >= 2^256" % name, spki, b"\x30" + bytes([len(body)]) + body, msg, 1, "r >= n"))
        # DER structure (StdDSAEncoder.decode + re-encode equality) -> SignatureException
        cases.append(ec_case("%s DER long-form length" % name, spki, b"\x30\x81" + der[1:2] + der[2:], msg, 2,
                             "DER re-encode mismatch (BC 1.56+)"))
        cases.append(ec_case("%s DER indefinite length" % name, spki, b"\x30\x80" + der[2:] + b"\x00\x00", msg, 2,
                             "BER indefinite length"))
        body = G.der_encode_int(r) + G.der_encode_int(s_) + G.der_encode_int(5)
        cases.append(ec_case("%s DER three elements" % name, spki, b"\x30" + bytes([len(body)]) + body, msg, 2,
                             "s.size() != 2"))
        body = G.der_encode_int(r)
        cases.append(ec_case("%s DER one element" % name, spki, b"\x30" + bytes([len(body)]) + body, msg, 2,
                             "s.size() != 2"))
        cases.append(ec_case("%s DER trailing byte" % name, spki, der + b"\x00", msg, 2, "re-encode mismatch"))
        cases.append(ec_case("%s DER truncated" % name, spki, der[:-1], msg, 2, "parse error"))
        cases.append(ec_case("%s DER outer tag SET" % name, spki, b"\x31" + der[1:], msg, 2, "not a SEQUENCE"))
        cases.append(ec_case("%s DER BIT STRING element" % name, spki, der[:2] + b"\x03" + der[3:], msg, 2,
                             "ASN1Integer.getInstance fails"))
        body = b"\x02\x00" + G.der_encode_int(s_)
        cases.append(ec_case("%s DER empty INTEGER" % name, spki, b"\x30" + bytes([len(body)]) + body, msg, 2,
                             "BigInteger of zero length"))
        rpad = b"\x00\x00" + r.to_bytes(32, "big")
        body = b"\x02" + bytes([len(rpad)]) + rpad + G.der_encode_int(s_)
        cases.append(ec_case("%s DER non-minimal INTEGER padding" % name, spki, b"\x30" + bytes([len(body)]) + body,
                             msg, 2, "ASN1Integer rejects a malformed (non-minimal) INTEGER -> 'error decoding signature "
                             "bytes.' (BC 1.57 as restated; unpinned: no reference test)", unpinned=True))
        cases.append(ec_case("%s raw r||s (not DER)" % name, spki, rb + sb, msg, 2, "not DER"))
        cases.append(ec_case("%s empty signature" % name, spki, b"", msg, 3, "Crypto.kt:528"))
        cases.append(ec_case("%s empty clear data" % name, spki, der, b"", 4, "Crypto.kt:529"))
        # keys
        bad = b"\x04" + P[0].to_bytes(32, "big") + ((P[1] + 1) % c["p"]).to_bytes(32, "big")
        cases.append(ec_case("%s key not on curve" % name, G.spki_ec(scheme, bad), der, msg, 6, "ECPoint.isValid"))
        bad = b"\x04" + (P[0] + c["p"]).to_bytes(33, "big")[1:] + P[1].to_bytes(32, "big") \
            if P[0] + c["p"] < 2**256 else b"\x04" + bytes([0xff] * 32) + P[1].to_bytes(32, "big")
        cases.append(ec_case("%s key x >= p" % name, G.spki_ec(scheme, bad), der, msg, 6, "fromBigInteger range"))
        cases.append(ec_case("%s key infinity encoding" % name, G.spki_ec(scheme, b"\x00" * 65), der, msg, 6,
                             "point at infinity"))
        # generator and -generator as keys (exceptional additions inside the joint mult)
        for dd, lab in ((1, "key = G"), (n - 1, "key = -G"), (2, "key = 2G")):
            pk = ec_mul(c, dd, c["g"])
            kk = hashlib.sha256(b"nk" + lab.encode() + name.encode()).digest()
            dder = G.ec_sign(scheme, dd.to_bytes(32, "big"), kk, msg)[0]
            cases.append(ec_case("%s %s" % (name, lab), ec_spki(scheme, pk), dder, msg, 0, "exceptional point adds"))
        # x(R) in [n, p): accept through the r + n branch (Q constructed from a chosen R)
        x = n + 1
        while True:
            rhs = (x ** 3 + c["a"] * x + c["b"]) % c["p"]
            y = pow(rhs, (c["p"] + 1) // 4, c["p"])
            if y * y % c["p"] == rhs:
                break
            x += 1
        Rpt = (x, y)
        rr = x % n
        ss = int.from_bytes(hashlib.sha256(b"s" + name.encode()).digest(), "big") % n
        e = int.from_bytes(hashlib.sha256(msg).digest(), "big") % n
        w = pow(ss, -1, n)
        u1, u2 = e * w % n, rr * w % n
        # Q = (R - u1 G) * u2^-1
        negu1G = ec_mul(c, (n - u1) % n, c["g"])
        Qpt = ec_mul(c, pow(u2, -1, n), ec_add(c, Rpt, negu1G))
        cases.append(ec_case("%s x(R) >= n accepted via r + n" % name, ec_spki(scheme, Qpt), G.der_sig(rr, ss), msg, 0,
                             "ECDSASigner r*Z^2 loop at r, r+n"))
    # wrong-curve key: r1 signature checked against the k1 key with the same scalar
    return cases


def uniq_cases():
    """Hand-built notary scenarios; `expected` restates the reference semantics (not the oracle):
    PersistentUniquenessProviderTests.kt:35-61, NotaryServiceTests.kt:98-145, SURVEY.md §8a."""
    def ref(name, i):
        return G.state_ref(hashlib.sha256(name.encode()).digest(), i).hex()

    def tx(name):
        return hashlib.sha256(b"tx:" + name.encode()).hexdigest()
    a, b_, c, d = ref("a", 0), ref("b", 0), ref("c", 1), ref("d", 2)
    cases = [
        dict(label="commit then re-commit by another tx -> conflict",
             source="PersistentUniquenessProviderTests.kt:35-61",
             batches=[[[tx("t1"), [a], 1]], [[tx("t2"), [a], 2]]], expected=[[0], [2]]),
        dict(label="double spend across txs in one batch", source="NotaryServiceTests.kt:118-145",
             batches=[[[tx("t1"), [a, b_], 1], [tx("t2"), [b_, c], 1]]], expected=[[0, 2]]),
        dict(label="identical tx notarised twice is idempotent", source="NotaryServiceTests.kt:98-116",
             batches=[[[tx("t1"), [a, b_], 7]], [[tx("t1"), [a, b_], 7]]], expected=[[0], [1]]),
        dict(label="identical tx twice in one batch", source="NotaryServiceTests.kt:98-116",
             batches=[[[tx("t1"), [a, b_], 7], [tx("t1"), [a, b_], 7]]], expected=[[0, 1]]),
        dict(label="same tx id, other caller -> conflict", source="ConsumingTx equality incl. requestingParty",
             batches=[[[tx("t1"), [a], 1], [tx("t1"), [a], 2]]], expected=[[0, 2]]),
        dict(label="failed tx consumes nothing: tx1{a}, tx2{a,b}, tx3{b}", source="SURVEY.md §7 / §8a",
             batches=[[[tx("t1"), [a], 1], [tx("t2"), [a, b_], 1], [tx("t3"), [b_], 1]]], expected=[[0, 2, 0]]),
        dict(label="chain of failures: tx2 blocked by tx1, tx3 by nothing, tx4 by tx3",
             source="sequential commit order",
             batches=[[[tx("t1"), [a], 1], [tx("t2"), [a, b_], 1], [tx("t3"), [b_, c], 1], [tx("t4"), [c, d], 1]]],
             expected=[[0, 2, 0, 2]]),
        dict(label="duplicate input inside one tx commits (first index wins)",
             source="AppendOnlyPersistentMap.kt:51-92", batches=[[[tx("t1"), [a, a], 1]]], expected=[[0]]),
        dict(label="re-submitting a tx with a duplicated input is a real conflict (index 1 != 0)",
             source="NotaryService.kt:61-75 index-aware idempotency",
             batches=[[[tx("t1"), [a, a], 1]], [[tx("t1"), [a, a], 1]]], expected=[[0], [2]]),
        dict(label="partial overlap with own earlier commit is idempotent, inserts nothing",
             source="NotaryService.kt:61-75", batches=[[[tx("t1"), [a, b_], 3]], [[tx("t1"), [a, b_], 3],
                                                                                  [tx("t5"), [b_], 3]]],
             expected=[[0], [1, 2]]),
        dict(label="tx with no inputs commits", source="commit(emptyList)",
             batches=[[[tx("t1"), [], 1]]], expected=[[0]]),
    ]
    return cases


def main():
    G.build()
    uq = uniq_cases()
    with open(os.path.join(HERE, "uniq_cases.json"), "w") as f:
        json.dump(uq, f, indent=1)
    print("uniq cases:", len(uq))
    ec = ecdsa_cases()
    with open(os.path.join(HERE, "ecdsa_cases.json"), "w") as f:
        json.dump(ec, f, indent=1)
    print("ecdsa cases:", len(ec))
    ed = ed25519_cases()
    with open(os.path.join(HERE, "ed25519_cases.json"), "w") as f:
        json.dump(ed, f, indent=1)
    tx = txid_cases()
    with open(os.path.join(HERE, "txid_cases.json"), "w") as f:
        json.dump(tx, f, indent=1)
    print("ed25519 cases:", len(ed), " txid cases:", len(tx))


if __name__ == "__main__":
    main()
