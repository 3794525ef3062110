"""CompositeKey: weighted-threshold signing requirements over leaf keys (host side).

Mirrors net.corda.core.crypto.CompositeKey (CompositeKey.kt:22-270), the PublicKey extensions
`keys` / `isFulfilledBy` / `containsAny` (CryptoUtils.kt:100-112) and CompositeSignature's verify
(CompositeSignature.kt:77-86).  Fulfilment is set logic over the signers of a transaction and stays on
the host; the signatures themselves go through the engine in one batch.

Leaf keys are their X.509 SubjectPublicKeyInfo bytes (the form the C-ABI takes); a CompositeKey's
`encoded` is the reference's DER SPKI with algorithm OID 2.25.30086077608615255153862931087626791002
(CordaSecurityProvider.kt:35) and a SEQUENCE { threshold INTEGER, SEQUENCE OF SEQUENCE { BIT STRING
node.encoded, INTEGER weight } } (CompositeKey.kt:161-170), so `get_instance(k.encoded) == k`.
"""
from typing import Iterable, List, Optional, Sequence, Tuple, Union

COMPOSITE_KEY_OID = "2.25.30086077608615255153862931087626791002"
INT_MAX = 2**31 - 1


class IllegalArgumentException(ValueError):
    """Kotlin require() failure."""


class ArithmeticException(ArithmeticError):
    """Math.addExact overflow (KotlinUtils.kt:23)."""


# --------------------------------------------------------------------------------------------
# minimal DER (only what the composite SPKI needs)

def _der_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def _tlv(tag: int, body: bytes) -> bytes:
    return bytes([tag]) + _der_len(len(body)) + body


def _der_int(v: int) -> bytes:
    n = max(1, (v.bit_length() + 8) // 8)          # minimal two's complement (ASN1Integer)
    return _tlv(0x02, v.to_bytes(n, "big", signed=True))


def _der_oid(dotted: str) -> bytes:
    arcs = [int(a) for a in dotted.split(".")]
    out = bytearray()
    for v in [arcs[0] * 40 + arcs[1]] + arcs[2:]:
        enc = [v & 0x7F]
        v >>= 7
        while v:
            enc.append(0x80 | (v & 0x7F))
            v >>= 7
        out += bytes(reversed(enc))
    return _tlv(0x06, bytes(out))


def _der_read(buf: bytes, pos: int) -> Tuple[int, bytes, int]:
    """(tag, contents, next position); raises IllegalArgumentException on malformed input."""
    if pos + 2 > len(buf):
        raise IllegalArgumentException("truncated DER")
    tag, ln = buf[pos], buf[pos + 1]
    pos += 2
    if ln & 0x80:
        k = ln & 0x7F
        if k == 0 or k > 4 or pos + k > len(buf):
            raise IllegalArgumentException("bad DER length")
        ln = int.from_bytes(buf[pos:pos + k], "big")
        pos += k
    if pos + ln > len(buf):
        raise IllegalArgumentException("truncated DER")
    return tag, buf[pos:pos + ln], pos + ln


def _der_seq_items(body: bytes) -> List[Tuple[int, bytes]]:
    items, pos = [], 0
    while pos < len(body):
        tag, val, pos = _der_read(body, pos)
        items.append((tag, val))
    return items


def _spki_oid(encoded: bytes) -> Optional[bytes]:
    """The algorithm OID TLV of an SPKI, or None if `encoded` is not one."""
    try:
        tag, body, end = _der_read(encoded, 0)
        if tag != 0x30 or end != len(encoded):
            return None
        items = _der_seq_items(body)
        if len(items) != 2 or items[0][0] != 0x30 or items[1][0] != 0x03:
            return None
        alg = _der_seq_items(items[0][1])
        if not alg or alg[0][0] != 0x06:
            return None
        return _tlv(0x06, alg[0][1])
    except IllegalArgumentException:
        return None


_COMPOSITE_OID_TLV = _der_oid(COMPOSITE_KEY_OID)

Key = Union[bytes, "CompositeKey"]


def _encoded(key: Key) -> bytes:
    return key.encoded if isinstance(key, CompositeKey) else bytes(key)


# --------------------------------------------------------------------------------------------

class NodeAndWeight:
    """CompositeKey.kt:128-152: ordered by weight, then by the node's encoding (unsigned
    lexicographic, shorter first — ByteSequence.compareTo, ByteArrays.kt:74-86)."""
    __slots__ = ("node", "weight")

    def __init__(self, node: Key, weight: int):
        if weight <= 0:
            raise IllegalArgumentException("A non-positive weight was detected. Node info: %r" % (weight,))
        self.node = node
        self.weight = weight

    def _sort_key(self):
        return (self.weight, _encoded(self.node))

    def __eq__(self, other):
        return isinstance(other, NodeAndWeight) and self.weight == other.weight and self.node == other.node

    def __hash__(self):
        return hash((self.node, self.weight))

    def __iter__(self):
        yield self.node
        yield self.weight

    def __repr__(self):
        return "NodeAndWeight(weight=%d)" % self.weight


class CompositeKey:
    """CompositeKey.kt:22-221.  Construct through CompositeKey.Builder."""
    KEY_ALGORITHM = "COMPOSITE"

    def __init__(self, threshold: int, children: Sequence[NodeAndWeight]):
        self.threshold = threshold
        self.children: List[NodeAndWeight] = sorted(children, key=NodeAndWeight._sort_key)
        self._validated = False
        self._check_constraints()

    # CompositeKey.kt:60-72
    def _check_constraints(self):
        if len(self.children) != len(set(self.children)):
            raise IllegalArgumentException("CompositeKey with duplicated child nodes detected.")
        if len(self.children) <= 1:
            raise IllegalArgumentException("CompositeKey must consist of two or more child nodes.")
        if self.threshold <= 0:
            raise IllegalArgumentException(
                "CompositeKey threshold is set to %d, but it should be a positive integer." % self.threshold)
        total = self._total_weight()
        if self.threshold > total:
            raise IllegalArgumentException(
                "CompositeKey threshold: %d cannot be bigger than aggregated weight of child nodes: %d"
                % (self.threshold, total))

    # CompositeKey.kt:115-122 (Math.addExact on Int)
    def _total_weight(self) -> int:
        s = 0
        for _, w in self.children:
            if w <= 0:
                raise IllegalArgumentException("Non-positive weight: %d detected." % w)
            s += w
            if s > INT_MAX:
                raise ArithmeticException("integer overflow")
        return s

    # CompositeKey.kt:77-89 (identity-based, as the reference's IdentityHashMap)
    def _cycle_detection(self, visited: frozenset):
        for node, _ in self.children:
            if isinstance(node, CompositeKey):
                if id(node) in visited:
                    raise IllegalArgumentException("Cycle detected for CompositeKey")
                node._cycle_detection(visited | {id(node)})

    def check_validity(self):
        """CompositeKey.kt:99-111."""
        self._cycle_detection(frozenset({id(self)}))
        self._check_constraints()
        for node, _ in self.children:
            if isinstance(node, CompositeKey):
                node._check_constraints()
        self._validated = True

    # CompositeKey.kt:175-185
    def _check_fulfilled_by(self, keys: List[Key]) -> bool:
        if any(isinstance(k, CompositeKey) for k in keys):
            return False
        total = 0
        for node, weight in self.children:
            if isinstance(node, CompositeKey):
                total += weight if node._check_fulfilled_by(keys) else 0
            else:
                total += weight if node in keys else 0
        return total >= self.threshold

    def is_fulfilled_by(self, keys: Union[Key, Iterable[Key]]) -> bool:
        """CompositeKey.kt:157,192-198."""
        ks = [keys] if isinstance(keys, (bytes, bytearray, CompositeKey)) else list(keys)
        ks = [bytes(k) if isinstance(k, bytearray) else k for k in ks]
        if not self._validated:
            self.check_validity()
        return self._check_fulfilled_by(ks)

    @property
    def leaf_keys(self) -> set:
        """CompositeKey.kt:203-204."""
        out = set()
        for node, _ in self.children:
            out |= keys_of(node)
        return out

    @property
    def encoded(self) -> bytes:
        """CompositeKey.kt:161-170: DER SubjectPublicKeyInfo(AlgorithmIdentifier(COMPOSITE_KEY), ...)."""
        kids = b"".join(_tlv(0x30, _tlv(0x03, b"\x00" + _encoded(n)) + _der_int(w)) for n, w in self.children)
        body = _der_int(self.threshold) + _tlv(0x30, kids)
        return _tlv(0x30, _tlv(0x30, _COMPOSITE_OID_TLV) + _tlv(0x03, b"\x00" + _tlv(0x30, body)))

    @staticmethod
    def get_instance(encoded: bytes) -> Key:
        """CompositeKey.kt:28-46: DER SPKI -> Builder(children).build(threshold)."""
        if _spki_oid(encoded) != _COMPOSITE_OID_TLV:
            raise IllegalArgumentException("not a composite key")
        _, spki, _ = _der_read(encoded, 0)
        bits = _der_seq_items(spki)[1][1]
        if not bits or bits[0] != 0:
            raise IllegalArgumentException("bad BIT STRING")
        tag, seq, end = _der_read(bits[1:], 0)
        if tag != 0x30 or end != len(bits) - 1:
            raise IllegalArgumentException("bad composite key body")
        items = _der_seq_items(seq)
        if len(items) < 2 or items[0][0] != 0x02 or items[1][0] != 0x30:
            raise IllegalArgumentException("bad composite key body")
        threshold = int.from_bytes(items[0][1], "big", signed=True)   # positiveValue for valid keys
        b = CompositeKey.Builder()
        for tag, child in _der_seq_items(items[1][1]):
            if tag != 0x30:
                raise IllegalArgumentException("child is not a SEQUENCE")
            parts = _der_seq_items(child)
            if len(parts) < 2 or parts[0][0] != 0x03 or parts[1][0] != 0x02 or parts[0][1][:1] != b"\x00":
                raise IllegalArgumentException("bad child node")
            b.add_key(decode_public_key(parts[0][1][1:]), int.from_bytes(parts[1][1], "big", signed=True))
        return b.build(threshold)

    def __eq__(self, other):
        return (isinstance(other, CompositeKey) and self.threshold == other.threshold
                and self.children == other.children)

    def __hash__(self):
        return hash((self.threshold, tuple(self.children)))

    def __repr__(self):
        return "CompositeKey(threshold=%d, %r)" % (self.threshold, self.children)

    class Builder:
        """CompositeKey.kt:224-268."""

        def __init__(self):
            self._children: List[NodeAndWeight] = []

        def add_key(self, key: Key, weight: int = 1) -> "CompositeKey.Builder":
            self._children.append(NodeAndWeight(key, weight))
            return self

        def add_keys(self, *keys: Key) -> "CompositeKey.Builder":
            for k in keys:
                self.add_key(k)
            return self

        def build(self, threshold: Optional[int] = None) -> Key:
            if threshold is not None and threshold <= 0:
                raise IllegalArgumentException("Failed requirement.")
            n = len(self._children)
            if n > 1:
                if threshold is None:   # Kotlin Int sum: wraps on overflow (then fails threshold > 0)
                    threshold = sum(w for _, w in self._children)
                    threshold = (threshold + 2**31) % 2**32 - 2**31
                return CompositeKey(threshold, self._children)
            if n == 1:
                if threshold is not None and threshold != self._children[0].weight:
                    raise IllegalArgumentException("Trying to build invalid CompositeKey, threshold value different "
                                                   "than weight of single child node.")
                return self._children[0].node   # single keys are never wrapped
            raise RuntimeError("Trying to build CompositeKey without child nodes.")


def decode_public_key(encoded: bytes) -> Key:
    """Crypto.decodePublicKey as far as composites go: a composite SPKI becomes a CompositeKey, any
    other key stays its SPKI bytes."""
    encoded = bytes(encoded)
    if _spki_oid(encoded) == _COMPOSITE_OID_TLV:
        return CompositeKey.get_instance(encoded)
    return encoded


def as_key(key: Key) -> Key:
    """Normalise a key given as bytes: composite SPKI bytes are decoded to a CompositeKey."""
    if isinstance(key, CompositeKey):
        return key
    return decode_public_key(key)


def keys_of(key: Key) -> set:
    """PublicKey.keys (CryptoUtils.kt:100)."""
    key = as_key(key)
    return key.leaf_keys if isinstance(key, CompositeKey) else {key}


def is_fulfilled_by(key: Key, other_keys: Union[Key, Iterable[Key]]) -> bool:
    """PublicKey.isFulfilledBy (CryptoUtils.kt:103-105)."""
    key = as_key(key)
    if isinstance(key, CompositeKey):
        return key.is_fulfilled_by(other_keys)
    if isinstance(other_keys, (bytes, bytearray, CompositeKey)):
        other_keys = [other_keys]
    return key in [bytes(k) if isinstance(k, bytearray) else k for k in other_keys]


def contains_any(key: Key, other_keys: Iterable[Key]) -> bool:
    """PublicKey.containsAny (CryptoUtils.kt:108-112)."""
    key = as_key(key)
    others = set(other_keys)
    if isinstance(key, CompositeKey):
        return bool(key.leaf_keys & others)
    return key in others
