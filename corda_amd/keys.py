"""Public-key decoding as the Kryo front end needs it (host mirror of the device checks in kryo.hip).

When a SignedTransaction is deserialised, every PublicKey in it goes through PublicKeySerializer.read ->
Crypto.decodePublicKey(encoded) (Kryo.kt:302-311, Crypto.kt:343-348): a key that does not decode throws
and the transaction never reaches verifySignaturesExcept.  The device front end therefore checks every
key it reads (command signers, the notary's owningKey, CompositeKey leaves) and hands a transaction with
a key outside what it can decide to the JVM path (CHIP_STX_UNSUPPORTED):

  * Ed25519 / ECDSA secp256r1 / secp256k1 SubjectPublicKeyInfo in the encodings the verify path reads
    (oracle orc_spki_scheme): the point must decode — i2p eddsa 0.2.0 GroupElement(curve, bytes): y from
    the low 255 bits (not range-checked), x^2 = (y^2 - 1) / (d y^2 + 1) must be a square; BC 1.57
    decodePoint: coordinates < p and the point on the curve (compressed: x^3 + ax + b a square);
  * a CompositeKey SPKI (CompositeKey.kt:37-55, 166-212) decoded into its post-order tree, accepted only
    in its canonical DER (what CompositeKey.encoded re-encodes: minimal lengths and INTEGERs, children
    sorted by (weight, encoded) strictly — which is also the no-duplicate rule of checkConstraints —,
    every leaf in the encoding its key class re-encodes), with checkConstraints' rules (>= 2 children,
    weights > 0 with an Int sum, 0 < threshold <= total) and the device's limits (<= 64 nodes, nesting
    <= 8 levels);
  * anything else (RSA, SPHINCS, other encodings) -> unsupported.

Byte equality of canonical encodings is key equality on the JVM, so the device compares keys by bytes.
"""
from typing import List, Optional, Tuple

P25519 = 2**255 - 19
D25519 = (-121665 * pow(121666, P25519 - 2, P25519)) % P25519

SPKI_ED25519 = bytes.fromhex("302a300506032b6570032100")
SPKI_R1_U = bytes.fromhex("3059301306072a8648ce3d020106082a8648ce3d03010703420004")[:26]
SPKI_R1_C = bytes.fromhex("3039301306072a8648ce3d020106082a8648ce3d030107032200")
SPKI_K1_U = bytes.fromhex("3056301006072a8648ce3d020106052b8104000a03420004")[:23]
SPKI_K1_C = bytes.fromhex("3036301006072a8648ce3d020106052b8104000a032200")

CURVES = {
    3: (0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF,
        0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFC,
        0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B),
    2: (0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F, 0, 7),
}
ED25519, K1, R1 = 4, 2, 3
COMPOSITE_OID_TLV = bytes.fromhex("0613" "69ada2af89d5b8e2aff38d93ac9de6969bd05a")
COMPOSITE_MAX_NODES = 64
COMPOSITE_MAX_DEPTH = 8
INT_MAX = 2**31 - 1


class KeyUnsupported(ValueError):
    """The key is not one the device front end decides (-> CHIP_STX_UNSUPPORTED)."""


def spki_scheme(spki: bytes) -> Tuple[int, Optional[bytes]]:
    """(scheme, raw point) for the encodings the verify path reads (oracle orc_spki_scheme), else (0, None)."""
    n = len(spki)
    if n == 44 and spki[:12] == SPKI_ED25519:
        return ED25519, spki[12:]
    if n == 91 and spki[:26] == SPKI_R1_U:
        return R1, spki[26:]
    if n == 59 and spki[:26] == SPKI_R1_C:
        return R1, spki[26:]
    if n == 88 and spki[:23] == SPKI_K1_U:
        return K1, spki[23:]
    if n == 56 and spki[:23] == SPKI_K1_C:
        return K1, spki[23:]
    return 0, None


def ed25519_point_ok(a: bytes) -> bool:
    """i2p GroupElement(curve, a) does not throw."""
    y = (int.from_bytes(a, "little") & ((1 << 255) - 1)) % P25519
    u = (y * y - 1) % P25519
    v = (D25519 * y * y + 1) % P25519
    x2 = u * pow(v, P25519 - 2, P25519) % P25519
    return x2 == 0 or pow(x2, (P25519 - 1) // 2, P25519) == 1


def ed25519_canonical(a: bytes) -> bool:
    """EdDSAPublicKey re-encodes A as A.toByteArray(): y < p, sign bit = parity of x (0 when x = 0)."""
    y = int.from_bytes(a, "little") & ((1 << 255) - 1)
    if y >= P25519:
        return False
    return not (a[31] >> 7 and (y * y - 1) % P25519 == 0)


def ec_point_ok(scheme: int, raw: bytes) -> bool:
    """BC ECCurve.decodePoint does not throw."""
    p, a, b = CURVES[scheme]
    if len(raw) == 65 and raw[0] == 4:
        x, y = int.from_bytes(raw[1:33], "big"), int.from_bytes(raw[33:], "big")
        return x < p and y < p and (y * y - (x ** 3 + a * x + b)) % p == 0
    if len(raw) == 33 and raw[0] in (2, 3):
        x = int.from_bytes(raw[1:], "big")
        if x >= p:
            return False
        rhs = (x ** 3 + a * x + b) % p
        return rhs == 0 or pow(rhs, (p - 1) // 2, p) == 1
    return False


def plain_key_ok(spki: bytes) -> bool:
    """Crypto.decodePublicKey succeeds on a plain (non-composite) key the verify path reads."""
    scheme, raw = spki_scheme(spki)
    if scheme == ED25519:
        return ed25519_point_ok(raw)
    if scheme in (R1, K1):
        return ec_point_ok(scheme, raw)
    return False


def plain_key_canonical(spki: bytes) -> bool:
    """A decodable plain key in the encoding its JVM key class re-encodes (EdDSAPublicKey: 44 bytes,
    canonical A; BCECPublicKey: the uncompressed named-curve SPKI)."""
    scheme, raw = spki_scheme(spki)
    if scheme == ED25519:
        return ed25519_point_ok(raw) and ed25519_canonical(raw)
    if scheme in (R1, K1):
        return len(raw) == 65 and ec_point_ok(scheme, raw)
    return False


def is_composite(spki: bytes) -> bool:
    """SubjectPublicKeyInfo whose AlgorithmIdentifier is exactly SEQUENCE { the CompositeKey OID } (the
    prefix the device matches; anything else is not taken for a composite)."""
    try:
        tag, c0, c1 = _tlv(spki, 0, len(spki))
        if tag != 0x30 or c1 != len(spki):
            return False
        tag, a0, a1 = _tlv(spki, c0, c1)
        return tag == 0x30 and spki[a0:a1] == COMPOSITE_OID_TLV
    except KeyUnsupported:
        return False


# ---- canonical DER ----
def _tlv(buf: bytes, pos: int, end: int) -> Tuple[int, int, int]:
    """(tag, content start, content end) of a TLV with a minimal definite length inside [pos, end)."""
    if pos + 2 > end:
        raise KeyUnsupported("truncated DER")
    tag, ln = buf[pos], buf[pos + 1]
    if ln < 0x80:
        n, h = ln, 2
    elif ln == 0x81:
        if pos + 3 > end or buf[pos + 2] < 0x80:
            raise KeyUnsupported("non-minimal DER length")
        n, h = buf[pos + 2], 3
    elif ln == 0x82:
        if pos + 4 > end:
            raise KeyUnsupported("truncated DER")
        n, h = (buf[pos + 2] << 8) | buf[pos + 3], 4
        if n < 0x100:
            raise KeyUnsupported("non-minimal DER length")
    else:
        raise KeyUnsupported("DER length form")
    if pos + h + n > end:
        raise KeyUnsupported("truncated DER")
    return tag, pos + h, pos + h + n


def _pos_int(buf: bytes, c0: int, c1: int) -> int:
    """A minimal DER INTEGER in [1, 2^31 - 1] (what ASN1Integer(weight.toLong()) writes for a valid key)."""
    n = c1 - c0
    if n < 1 or n > 4 or buf[c0] >= 0x80 or (n > 1 and buf[c0] == 0 and buf[c0 + 1] < 0x80):
        raise KeyUnsupported("INTEGER")
    v = int.from_bytes(buf[c0:c1], "big")
    if v < 1:
        raise KeyUnsupported("INTEGER < 1")
    return v


# node = (leaf SPKI bytes or None, threshold (composite) or 0, child count, weight in the parent)
Node = Tuple[Optional[bytes], int, int, int]


def composite_tree(spki: bytes, weight: int = 1, depth: int = 0) -> List[Node]:
    """The post-order nodes of a canonical CompositeKey SPKI (root last, its weight = `weight`)."""
    n = len(spki)
    tag, s0, s1 = _tlv(spki, 0, n)
    if tag != 0x30 or s1 != n:
        raise KeyUnsupported("SPKI")
    tag, a0, a1 = _tlv(spki, s0, s1)
    if tag != 0x30 or spki[a0:a1] != COMPOSITE_OID_TLV:
        raise KeyUnsupported("algorithm")
    tag, b0, b1 = _tlv(spki, a1, s1)
    if tag != 0x03 or b1 != s1 or b0 >= b1 or spki[b0] != 0:
        raise KeyUnsupported("BIT STRING")
    tag, q0, q1 = _tlv(spki, b0 + 1, b1)
    if tag != 0x30 or q1 != b1:
        raise KeyUnsupported("key body")
    tag, t0, t1 = _tlv(spki, q0, q1)
    if tag != 0x02:
        raise KeyUnsupported("threshold")
    threshold = _pos_int(spki, t0, t1)
    tag, c0, c1 = _tlv(spki, t1, q1)
    if tag != 0x30 or c1 != q1:
        raise KeyUnsupported("children")
    nodes: List[Node] = []
    kids, total, prev = 0, 0, None
    pos = c0
    while pos < c1:
        tag, k0, k1 = _tlv(spki, pos, c1)
        if tag != 0x30:
            raise KeyUnsupported("child")
        tag, e0, e1 = _tlv(spki, k0, k1)
        if tag != 0x03 or e0 >= e1 or spki[e0] != 0:
            raise KeyUnsupported("child BIT STRING")
        tag, w0, w1 = _tlv(spki, e1, k1)
        if tag != 0x02 or w1 != k1:
            raise KeyUnsupported("child weight")
        w = _pos_int(spki, w0, w1)
        child = spki[e0 + 1:e1]
        key = (w, child)
        if prev is not None and not prev < key:   # NodeAndWeight order (weight, ByteSequence), no duplicates
            raise KeyUnsupported("children not in canonical order")
        prev = key
        if is_composite(child):
            if depth + 1 >= COMPOSITE_MAX_DEPTH:
                raise KeyUnsupported("nesting")
            nodes += composite_tree(child, w, depth + 1)
        elif plain_key_canonical(child):
            nodes.append((child, 0, 0, w))
        else:
            raise KeyUnsupported("leaf key")
        kids += 1
        total += w
        if total > INT_MAX:
            raise KeyUnsupported("weight overflow")   # exactAdd -> ArithmeticException
        pos = k1
    if kids < 2 or threshold > total:
        raise KeyUnsupported("CompositeKey constraints")
    nodes.append((None, threshold, kids, weight))
    if len(nodes) > COMPOSITE_MAX_NODES:
        raise KeyUnsupported("too many nodes")
    return nodes
