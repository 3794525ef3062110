"""Kryo 4.0.0 wire format, restated for the bytes the signature path signs.

The signed message of every transaction signature is `SignableData(txId, signatureMetadata)
.serialize().bytes` (Crypto.kt:550-578 -> SerializationAPI.kt:193), produced on a node by the Kryo
P2P context (Node.kt:372: SerializationDefaults.P2P_CONTEXT = KRYO_P2P_CONTEXT).  This module writes
and reads those bytes without a JVM, from the published Kryo 4.0.0 algorithms as Corda configures
them (node-api/build.gradle:25 pins Kryo 4.0.0):

  header      "corda" 00 00 01                                    SerializationScheme.kt:251 (KryoHeaderV0_1)
  object      kryo.writeClassAndObject(output, obj)               SerializationScheme.kt:218-239
  class       unregistered @CordaSerializable classes are registered implicitly by NAME
              (CordaClassResolver.registerImplicit, CordaClassResolver.kt:76-99):
              varint(NAME + 2 = 1), varint(name id), name string the first time per graph, just the
              id afterwards (Kryo DefaultClassResolver.writeName; ids restart every graph)
  reference   references on (KRYO_P2P_CONTEXT objectReferencesEnabled = true; MapReferenceResolver):
              a first-seen object is preceded by varint(NOT_NULL = 1)
  serializer  default CompatibleFieldSerializer with CachedFieldNameStrategy.EXTENDED
              (DefaultKryoCustomizer.kt:59-62): the first time a class is written in a graph,
              varint(field count) + every cached field name ("DeclaringSimpleName.field", sorted);
              then each field's bytes through one OutputChunked(1024): varint(chunk length), bytes,
              and a 0 end marker per field
  fields      int: zig-zag varint (CachedField.varIntsEnabled); byte[]: varint(length + 1) + bytes
              (DefaultArraySerializers.ByteArraySerializer); a field of a final class (Kotlin
              classes are final) writes reference + object; of an abstract type (SecureHash is
              sealed) writes the concrete class first
  strings     Output.writeString: ASCII with 1 < length < 64 -> the bytes with bit 7 set on the last;
              otherwise varint(UTF-16 length + 1) with bit 7 of the first byte set, then UTF-8

SignableData (SignableData.kt:12-13) has fields signatureMetadata (SignatureMetadata.kt:14-15: two
ints) and txId (SecureHash.SHA256 -> OpaqueBytes.bytes, ByteArrays.kt:121).  For one metadata value
the serialized form is a fixed byte string with the 32-byte id at a fixed offset, which is what the
fused tx-verify kernel (chip_verify_tx_batch templates) relies on.

PARITY UNPINNED: the reference holds no serialized SignableData bytes and no JVM runs here, so these
bytes follow the Kryo 4.0.0 source semantics as restated above; tests pin only self-consistency
(write -> read round trips, template offsets, field order).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

KRYO_HEADER_V0_1 = b"corda\x00\x00\x01"
NULL, NOT_NULL, NAME = 0, 1, -1
CHUNK = 1024

SIGNABLE_DATA = "net.corda.core.crypto.SignableData"
SECURE_HASH_SHA256 = "net.corda.core.crypto.SecureHash$SHA256"
SIGNATURE_METADATA = "net.corda.core.crypto.SignatureMetadata"


class KryoException(Exception):
    pass


# ---- primitives (com.esotericsoftware.kryo.io.Output) ----
def varint(v: int, optimize_positive: bool = True) -> bytes:
    """Output.writeVarInt: zig-zag when optimize_positive is false, then 7-bit groups, LSB first."""
    if not optimize_positive:
        v = ((v << 1) ^ (v >> 31)) & 0xFFFFFFFF
    v &= 0xFFFFFFFF
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def string(s: str) -> bytes:
    """Output.writeString."""
    n = len(s)
    if n == 0:
        return b"\x81"
    if 1 < n < 64 and all(ord(c) < 128 for c in s):
        b = bytearray(s.encode("ascii"))
        b[-1] |= 0x80
        return bytes(b)
    # writeUtf8Length(charCount + 1): 6 bits in the first byte (bit 7 = UTF-8 flag, bit 6 = more)
    v = n + 1
    head = bytearray()
    first = 0x80 | (v & 0x3F)
    v >>= 6
    if v:
        first |= 0x40
    head.append(first)
    while v:
        b = v & 0x7F
        v >>= 7
        head.append(b | (0x80 if v else 0))
    return bytes(head) + s.encode("utf-8")


class Graph:
    """Per-graph state of one writeClassAndObject call: class-name ids and the classes whose
    CompatibleFieldSerializer field-name header is already out (both reset per graph)."""

    def __init__(self):
        self.name_ids: Dict[str, int] = {}
        self.headers: set = set()

    def write_class(self, name: str) -> bytes:
        if name in self.name_ids:
            return varint(NAME + 2) + varint(self.name_ids[name])
        nid = len(self.name_ids)
        self.name_ids[name] = nid
        return varint(NAME + 2) + varint(nid) + string(name)

    def compatible(self, cls: str, fields: List[Tuple[str, bytes]]) -> bytes:
        """CompatibleFieldSerializer.write: fields = [(cached name, field bytes)], sorted here by
        cached name (FieldSerializer orders its CachedFields by name)."""
        fields = sorted(fields, key=lambda f: f[0])
        out = bytearray()
        if cls not in self.headers:
            self.headers.add(cls)
            out += varint(len(fields))
            for name, _ in fields:
                out += string(name)
        for _, data in fields:
            out += chunked(data)
        return bytes(out)


def chunked(data: bytes) -> bytes:
    """OutputChunked(output, 1024) for one field then endChunks(): chunks of at most 1024 bytes,
    each prefixed by its varint length, then a 0 end marker."""
    out = bytearray()
    for i in range(0, len(data), CHUNK):
        part = data[i:i + CHUNK]
        out += varint(len(part)) + part
    out.append(0)
    return bytes(out)


# ---- SignableData ----
def _sha256_object(g: Graph, tx_id: bytes) -> bytes:
    if len(tx_id) != 32:   # SecureHash.SHA256 init { require(bytes.size == 32) }
        raise KryoException("SecureHash.SHA256 needs 32 bytes")
    arr = varint(NOT_NULL) + varint(len(tx_id) + 1) + bytes(tx_id)
    return (g.write_class(SECURE_HASH_SHA256) + varint(NOT_NULL)
            + g.compatible(SECURE_HASH_SHA256, [("OpaqueBytes.bytes", arr)]))


def _metadata_object(g: Graph, platform_version: int, scheme_number_id: int) -> bytes:
    return varint(NOT_NULL) + g.compatible(SIGNATURE_METADATA, [
        ("SignatureMetadata.platformVersion", varint(platform_version, False)),
        ("SignatureMetadata.schemeNumberID", varint(scheme_number_id, False))])


def signable_data(tx_id: bytes, platform_version: int, scheme_number_id: int) -> bytes:
    """SignableData(SecureHash.SHA256(tx_id), SignatureMetadata(platformVersion, schemeNumberID))
    .serialize().bytes under the Kryo P2P context."""
    g = Graph()
    body = g.write_class(SIGNABLE_DATA) + varint(NOT_NULL) + g.compatible(SIGNABLE_DATA, [
        ("SignableData.signatureMetadata", _metadata_object(g, platform_version, scheme_number_id)),
        ("SignableData.txId", _sha256_object(g, tx_id))])
    return KRYO_HEADER_V0_1 + body


def signable_data_template(platform_version: int, scheme_number_id: int) -> Tuple[bytes, int]:
    """(template bytes without the id, id offset) — the chip_msg_templates convention: the message
    of every transaction signed with this metadata is t[:at] + txId + t[at:]."""
    a = signable_data(b"\x00" * 32, platform_version, scheme_number_id)
    b = signable_data(b"\xff" * 32, platform_version, scheme_number_id)
    diff = [i for i in range(len(a)) if a[i] != b[i]]
    at = diff[0]
    assert diff == list(range(at, at + 32)) and len(a) == len(b)
    return a[:at] + a[at + 32:], at


# ---- reader (front end: SignableData bytes -> (txId, platformVersion, schemeNumberID)) ----
class Reader:
    def __init__(self, buf: bytes, pos: int = 0):
        self.buf = buf
        self.pos = pos
        self.names: Dict[int, str] = {}
        self.headers: Dict[str, List[str]] = {}

    def byte(self) -> int:
        if self.pos >= len(self.buf):
            raise KryoException("buffer underflow")
        b = self.buf[self.pos]
        self.pos += 1
        return b

    def varint(self, optimize_positive: bool = True) -> int:
        v, shift = 0, 0
        while True:
            b = self.byte()
            v |= (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                break
            if shift > 35:
                raise KryoException("malformed varint")
        v &= 0xFFFFFFFF
        if not optimize_positive:
            v = (v >> 1) ^ -(v & 1)
        return v

    def string(self) -> str:
        b = self.byte()
        if b & 0x80 == 0:                  # ASCII run, last byte flagged
            out = bytearray([b])
            while True:
                c = self.byte()
                if c & 0x80:
                    out.append(c & 0x7F)
                    return out.decode("ascii")
                out.append(c)
        v = b & 0x3F
        if b & 0x40:
            shift = 6
            while True:
                c = self.byte()
                v |= (c & 0x7F) << shift
                shift += 7
                if not c & 0x80:
                    break
        if v == 0:
            raise KryoException("null string")
        n = v - 1
        s = self.buf[self.pos:].decode("utf-8", errors="strict")[:n]
        self.pos += len(s.encode("utf-8"))
        return s

    def read_class(self) -> str:
        tag = self.varint()
        if tag != NAME + 2:
            raise KryoException("expected a class written by name, got registration id %d" % (tag - 2))
        nid = self.varint()
        if nid not in self.names:
            self.names[nid] = self.string()
        return self.names[nid]

    def not_null(self):
        if self.varint() != NOT_NULL:
            raise KryoException("expected a first-seen object")

    def field_names(self, cls: str) -> List[str]:
        if cls not in self.headers:
            self.headers[cls] = [self.string() for _ in range(self.varint())]
        return self.headers[cls]

    def chunk(self) -> "Reader":
        data = bytearray()
        while True:
            n = self.varint()
            if n == 0:
                break
            data += self.buf[self.pos:self.pos + n]
            if self.pos + n > len(self.buf):
                raise KryoException("truncated chunk")
            self.pos += n
        r = Reader(bytes(data))
        r.names, r.headers = self.names, self.headers   # one graph
        return r


def parse_signable_data(buf: bytes) -> Tuple[bytes, int, int]:
    """Inverse of signable_data: (txId, platformVersion, schemeNumberID); KryoException on any
    other layout (trailing bytes included)."""
    if buf[:8] != KRYO_HEADER_V0_1:
        raise KryoException("Serialized bytes header does not match expected format.")
    r = Reader(buf, 8)
    if r.read_class() != SIGNABLE_DATA:
        raise KryoException("not a SignableData")
    r.not_null()
    names = r.field_names(SIGNABLE_DATA)
    if names != ["SignableData.signatureMetadata", "SignableData.txId"]:
        raise KryoException("unexpected SignableData fields %r" % names)
    m = r.chunk()
    m.not_null()
    if m.field_names(SIGNATURE_METADATA) != ["SignatureMetadata.platformVersion", "SignatureMetadata.schemeNumberID"]:
        raise KryoException("unexpected SignatureMetadata fields")
    pv = m.chunk().varint(False)
    sch = m.chunk().varint(False)
    t = r.chunk()
    if t.read_class() != SECURE_HASH_SHA256:
        raise KryoException("txId is not a SecureHash.SHA256")
    t.not_null()
    if t.field_names(SECURE_HASH_SHA256) != ["OpaqueBytes.bytes"]:
        raise KryoException("unexpected SecureHash fields")
    a = t.chunk()
    a.not_null()
    n = a.varint() - 1
    tx_id = a.buf[a.pos:a.pos + n]
    if n != 32 or len(tx_id) != 32:
        raise KryoException("txId is not 32 bytes")
    if r.pos != len(buf):
        raise KryoException("trailing bytes")
    return bytes(tx_id), pv, sch
