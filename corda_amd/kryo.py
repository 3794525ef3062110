"""Kryo 4.0.0 wire format, restated for the bytes on the signature path.

Two uses:
  * the signed message of every transaction signature, `SignableData(txId, signatureMetadata)
    .serialize().bytes` (Crypto.kt:550-578 -> SerializationAPI.kt:193);
  * the front end of a batch: `SignedTransaction` / `WireTransaction` bytes as nodes store and send
    them (Kryo.kt:236-280 serializers), parsed into component groups and signatures.  The product
    parser is the device kernel (corda_amd/csrc/kryo.hip, chip_stx_parse_device); the reader here is
    its host mirror and the writer builds the test and bench inputs.

Both are produced on a node by the Kryo P2P context (Node.kt:372: SerializationDefaults.P2P_CONTEXT =
KRYO_P2P_CONTEXT, references on) from the published Kryo 4.0.0 algorithms as Corda configures them
(node-api/build.gradle:25 pins Kryo 4.0.0):

  header      "corda" 00 00 01                                    SerializationScheme.kt:251 (KryoHeaderV0_1)
  object      kryo.writeClassAndObject(output, obj)               SerializationScheme.kt:218-239
  class       registered classes as varint(id + 2).  The Kryo constructor registers 10 primitives
              (ids 0-9); DefaultKryoCustomizer.kt:77-80 then registers Arrays$ArrayList (10),
              SignedTransaction (11), WireTransaction (12), SerializedBytes (13).  Every later id
              follows from the registration ORDER of DefaultKryoCustomizer.kt:81-122 (REGISTRATION_ORDER
              below: Kryo.register gives a new class the next free id, a class registered twice keeps
              its first id).  The javakaffee / Guava blocks (:81-86) register library-dependent class
              sets (kryo-serializers 0.41, Guava 21.0 — neither jar is under /root/reference): their
              counts are restated from those versions' published sources, so the ids from PrivacySalt
              and the PublicKey classes on are UNPINNED defaults.  They live in a Registry that a
              deployment overwrites with its JVM's own ids (chip_set_kryo_registry);
              readers accept exactly the registry's id where the position fixes the class and fail
              closed (KryoUnsupported -> the JVM path) on any other id.
              Unregistered @CordaSerializable / whitelisted classes are registered implicitly by
              NAME (CordaClassResolver.registerImplicit, CordaClassResolver.kt:76-99): varint(1),
              varint(name id), the name string the first time per graph (ids restart every graph)
  reference   references on (MapReferenceResolver): a first-seen object written through
              writeClassAndObject / writeObject(OrNull) is preceded by varint(NOT_NULL = 1).
              WireTransaction's serializer runs with references off (noReferencesWithin,
              DefaultKryoCustomizer.kt:88, Kryo.kt:425-437): no markers inside it
  serializer  default CompatibleFieldSerializer, CachedFieldNameStrategy.EXTENDED
              (DefaultKryoCustomizer.kt:59-62): the first time a class is written in a graph,
              varint(field count) + every cached field name ("DeclaringSimpleName.field", sorted);
              then each field through ONE OutputChunked(output, 1024) and endChunks() per field
  chunks      OutputChunked flushes a chunk (varint size + bytes, size > 0) when its 1024-byte buffer
              cannot take the next primitive (Output.require: a varint / byte never straddles a
              chunk, writeBytes fills the buffer first), and at endChunks, then writes the 0 end
              marker.  Output.flush also flushes the stream it writes to, so a nested
              CompatibleFieldSerializer (a field value with its own chunked fields) makes the
              enclosing field emit a chunk at every inner chunk: the writer below simulates the
              Output / OutputChunked buffers exactly instead of chunking flat byte strings
  fields      int: zig-zag varint (varIntsEnabled); byte[] field (final type): reference marker +
              varint(length + 1) + bytes (ByteArraySerializer); a field of a final class writes the
              reference marker + object; of an abstract / interface type (SecureHash, PublicKey,
              List) the concrete class first
  strings     Output.writeString: ASCII with 1 < length < 64 -> the bytes with bit 7 set on the last;
              otherwise varint(UTF-16 length + 1) with bit 7 of the first byte set, then UTF-8
  lists       ArrayList: CollectionSerializer, varint(size) + writeClassAndObject per element;
              Collections$SingletonList: writeClassAndObject(element); Arrays$ArrayList (id 10,
              javakaffee ArraysAsListSerializer): varint(size), the component class, elements

PARITY UNPINNED: the reference holds no serialized bytes and no JVM runs here, so these bytes follow
the Kryo 4.0.0 source semantics as restated above; tests pin self-consistency (write -> read round
trips, Python == C++ == the device parser, template offsets, chunk placement rules).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

KRYO_HEADER_V0_1 = b"corda\x00\x00\x01"
NULL, NOT_NULL, NAME = 0, 1, -1
CHUNK = 1024

# ---- class registrations (DefaultKryoCustomizer.kt:56-136) ----
# The Kryo constructor registers int, String, float, boolean, byte, char, short, long, double, void
# (ids 0-9); customize() then registers, in this order (file:line of the register call), one id per NEW
# class.  The javakaffee blocks list the classes their registerSerializers(kryo) registers under
# kryo-serializers 0.41 with Guava 21.0 (node-api/build.gradle:26, constants.properties:3), already
# reduced to distinct classes: e.g. ImmutableList.of() and .of().reverse() are both RegularImmutableList
# in Guava 21, .subList(1, 2) of a 3-list is a SingletonImmutableList.  Those two libraries are not
# under /root/reference, so from :81 on the ids are restated, not pinned (see the module docstring).
REGISTRATION_ORDER = [
    ("java.util.Arrays$ArrayList", "DefaultKryoCustomizer.kt:77"),
    ("net.corda.core.transactions.SignedTransaction", ":78"),
    ("net.corda.core.transactions.WireTransaction", ":79"),
    ("net.corda.core.serialization.SerializedBytes", ":80"),
    # :81 UnmodifiableCollectionsSerializer: one class per UnmodifiableCollection constant
    ("java.util.Collections$UnmodifiableCollection", ":81"),
    ("java.util.Collections$UnmodifiableRandomAccessList", ":81"),
    ("java.util.Collections$UnmodifiableList", ":81"),
    ("java.util.Collections$UnmodifiableSet", ":81"),
    ("java.util.Collections$UnmodifiableSortedSet", ":81"),
    ("java.util.Collections$UnmodifiableMap", ":81"),
    ("java.util.Collections$UnmodifiableSortedMap", ":81"),
    # :82 ImmutableListSerializer: ImmutableList, of(), of(1), of(1,2,3).subList(1,2), of().reverse(),
    # Lists.charactersOf(..), ImmutableTable.copyOf(..).values()
    ("com.google.common.collect.ImmutableList", ":82"),
    ("com.google.common.collect.RegularImmutableList", ":82"),
    ("com.google.common.collect.SingletonImmutableList", ":82"),
    ("com.google.common.collect.Lists$StringAsImmutableList", ":82"),
    ("com.google.common.collect.RegularImmutableTable$Values", ":82"),
    # :83 ImmutableSetSerializer: ImmutableSet, of(), of(1), of(1,2,3), Sets.immutableEnumSet(..)
    ("com.google.common.collect.ImmutableSet", ":83"),
    ("com.google.common.collect.RegularImmutableSet", ":83"),
    ("com.google.common.collect.SingletonImmutableSet", ":83"),
    ("com.google.common.collect.ImmutableEnumSet", ":83"),
    # :84 ImmutableSortedSetSerializer: ImmutableSortedSet, of(), of(""), of().descendingSet()
    ("com.google.common.collect.ImmutableSortedSet", ":84"),
    ("com.google.common.collect.RegularImmutableSortedSet", ":84"),
    # :85 ImmutableMapSerializer: ImmutableMap, of(), of(k, v), of(k, v, k, v), copyOf(EnumMap)
    ("com.google.common.collect.ImmutableMap", ":85"),
    ("com.google.common.collect.RegularImmutableBiMap", ":85"),
    ("com.google.common.collect.SingletonImmutableBiMap", ":85"),
    ("com.google.common.collect.RegularImmutableMap", ":85"),
    ("com.google.common.collect.ImmutableEnumMap", ":85"),
    # :86 ImmutableMultimapSerializer: ImmutableMultimap, ImmutableListMultimap.of() / .of(a, b),
    # ImmutableSetMultimap.of() / .of(a, b)
    ("com.google.common.collect.ImmutableMultimap", ":86"),
    ("com.google.common.collect.EmptyImmutableListMultimap", ":86"),
    ("com.google.common.collect.ImmutableListMultimap", ":86"),
    ("com.google.common.collect.EmptyImmutableSetMultimap", ":86"),
    ("com.google.common.collect.ImmutableSetMultimap", ":86"),
    ("java.io.BufferedInputStream", ":88"),
    ("sun.net.www.protocol.jar.JarURLConnection$JarURLInputStream", ":89"),
    ("sun.security.ec.ECPublicKeyImpl", ":91"),
    ("net.i2p.crypto.eddsa.EdDSAPublicKey", ":92"),
    ("net.i2p.crypto.eddsa.EdDSAPrivateKey", ":93"),
    ("net.corda.core.crypto.CompositeKey", ":94"),
    ("[Ljava.lang.StackTraceElement;", ":96"),
    ("net.corda.core.utilities.NonEmptySet", ":98"),
    ("java.util.BitSet", ":99"),
    ("java.lang.Class", ":100"),
    ("java.io.FileInputStream", ":101"),
    ("java.security.cert.CertPath", ":102"),
    ("sun.security.provider.certpath.X509CertPath", ":103"),
    ("org.bouncycastle.asn1.x500.X500Name", ":104"),
    ("org.bouncycastle.cert.X509CertificateHolder", ":105"),
    ("org.bouncycastle.jcajce.provider.asymmetric.ec.BCECPrivateKey", ":106"),
    ("org.bouncycastle.jcajce.provider.asymmetric.ec.BCECPublicKey", ":107"),
    ("org.bouncycastle.jcajce.provider.asymmetric.rsa.BCRSAPrivateCrtKey", ":108"),
    ("org.bouncycastle.jcajce.provider.asymmetric.rsa.BCRSAPublicKey", ":109"),
    ("org.bouncycastle.pqc.jcajce.provider.sphincs.BCSphincs256PrivateKey", ":110"),
    ("org.bouncycastle.pqc.jcajce.provider.sphincs.BCSphincs256PublicKey", ":111"),
    ("net.corda.core.transactions.NotaryChangeWireTransaction", ":112"),
    ("net.corda.core.identity.PartyAndCertificate", ":113"),
    ("net.corda.core.contracts.PrivacySalt", ":116"),
    ("net.corda.core.contracts.ContractAttachment", ":119"),
    ("java.lang.invoke.SerializedLambda", ":121"),
    ("com.esotericsoftware.kryo.serializers.ClosureSerializer$Closure", ":122"),
]
FIRST_CUSTOM_ID = 10


def registration_ids(order=REGISTRATION_ORDER) -> Dict[str, int]:
    """class name -> id: Kryo.register assigns the next free id to a class not registered yet."""
    ids: Dict[str, int] = {}
    for name, _ in order:
        ids.setdefault(name, FIRST_CUSTOM_ID + len(ids))
    return ids


# the classes registered with PublicKeySerializer (DefaultKryoCustomizer.kt:91,92,94,107,109,111): whichever
# of them a key slot names, the JVM reads writeBytesWithLength(encoded) -> Crypto.decodePublicKey (Kryo.kt:302-311)
PUBLIC_KEY_CLASSES = ["sun.security.ec.ECPublicKeyImpl", "net.i2p.crypto.eddsa.EdDSAPublicKey",
                      "net.corda.core.crypto.CompositeKey",
                      "org.bouncycastle.jcajce.provider.asymmetric.ec.BCECPublicKey",
                      "org.bouncycastle.jcajce.provider.asymmetric.rsa.BCRSAPublicKey",
                      "org.bouncycastle.pqc.jcajce.provider.sphincs.BCSphincs256PublicKey"]
MAX_PUBLIC_KEY_IDS = 8   # chip_kryo_registry.public_key[]


class Registry:
    """The registration ids the front end depends on (the C-ABI's chip_kryo_registry): the four pinned
    ones, PrivacySalt's, and every id whose serializer is PublicKeySerializer.  Defaults: the restated
    REGISTRATION_ORDER; a deployment passes its JVM's Kryo ids (kryo.getRegistration(cls).id)."""

    def __init__(self, ids: Optional[Dict[str, int]] = None):
        ids = registration_ids() if ids is None else ids
        self.arrays_aslist = ids["java.util.Arrays$ArrayList"]
        self.signed_tx = ids["net.corda.core.transactions.SignedTransaction"]
        self.wire_tx = ids["net.corda.core.transactions.WireTransaction"]
        self.serialized_bytes = ids["net.corda.core.serialization.SerializedBytes"]
        self.privacy_salt = ids["net.corda.core.contracts.PrivacySalt"]
        self.eddsa_public_key = ids["net.i2p.crypto.eddsa.EdDSAPublicKey"]
        self.bcec_public_key = ids["org.bouncycastle.jcajce.provider.asymmetric.ec.BCECPublicKey"]
        self.composite_key = ids["net.corda.core.crypto.CompositeKey"]
        self.public_key = [ids[c] for c in PUBLIC_KEY_CLASSES if c in ids][:MAX_PUBLIC_KEY_IDS]

    def as_tuple(self):
        return (self.arrays_aslist, self.signed_tx, self.wire_tx, self.serialized_bytes, self.privacy_salt,
                tuple(self.public_key))

    def key_class_for(self, spki: bytes) -> int:
        """The class a JVM writes for a key with this encoding (EdDSAPublicKey / BCECPublicKey / CompositeKey)."""
        if len(spki) == 44:
            return self.eddsa_public_key
        if _spki_oid_is_composite(spki):
            return self.composite_key
        return self.bcec_public_key


DEFAULT_REGISTRY = Registry()
REG_ARRAYS_ASLIST = DEFAULT_REGISTRY.arrays_aslist       # 10: pinned by DefaultKryoCustomizer.kt:77-80
REG_SIGNED_TX = DEFAULT_REGISTRY.signed_tx               # 11
REG_WIRE_TX = DEFAULT_REGISTRY.wire_tx                   # 12
REG_SERIALIZED_BYTES = DEFAULT_REGISTRY.serialized_bytes # 13
DEFAULT_IDS = {"privacy_salt": DEFAULT_REGISTRY.privacy_salt, "eddsa_public_key": DEFAULT_REGISTRY.eddsa_public_key,
               "bcec_public_key": DEFAULT_REGISTRY.bcec_public_key, "composite_key": DEFAULT_REGISTRY.composite_key}


def _spki_oid_is_composite(spki: bytes) -> bool:
    from corda_amd import composite as CK
    return CK._spki_oid(bytes(spki)) == CK._COMPOSITE_OID_TLV

SIGNABLE_DATA = "net.corda.core.crypto.SignableData"
SECURE_HASH_SHA256 = "net.corda.core.crypto.SecureHash$SHA256"
SIGNATURE_METADATA = "net.corda.core.crypto.SignatureMetadata"
TRANSACTION_SIGNATURE = "net.corda.core.crypto.TransactionSignature"
COMPONENT_GROUP = "net.corda.core.transactions.ComponentGroup"
ARRAY_LIST = "java.util.ArrayList"
SINGLETON_LIST = "java.util.Collections$SingletonList"

TXSIG_FIELDS = ["OpaqueBytes.bytes", "TransactionSignature.by", "TransactionSignature.signatureMetadata"]
META_FIELDS = ["SignatureMetadata.platformVersion", "SignatureMetadata.schemeNumberID"]
GROUP_FIELDS = ["ComponentGroup.components", "ComponentGroup.groupIndex"]


class KryoException(Exception):
    pass


class KryoUnsupported(KryoException):
    """Well-formed input outside the front end's grammar (device status CHIP_STX_UNSUPPORTED): the
    caller verifies that transaction on the JVM path."""


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


def chunked(data: bytes) -> bytes:
    """One OutputChunked(1024) field holding `data` written with writeBytes, then endChunks(), over a
    plain (non-chunked) output: chunks of 1024 bytes, the rest, the 0 end marker."""
    o = Out()
    c = Out(o)
    c.write_bytes(data)
    c.end_chunks()
    return o.getvalue()


class Out:
    """Kryo 4.0.0 Output / OutputChunked.  parent None = the top-level Output (its 64 KB buffer and
    ByteArrayOutputStream never change the bytes: modelled as unbounded); otherwise an
    OutputChunked(parent, 1024) whose OutputStream is the parent Output."""

    def __init__(self, parent: Optional["Out"] = None):
        self.parent = parent
        self.cap = CHUNK if parent is not None else None
        self.buf = bytearray()

    def getvalue(self) -> bytes:
        return bytes(self.buf)

    def _require(self, n: int):       # Output.require: flush when the buffer cannot take n more
        if self.cap is not None and self.cap - len(self.buf) < n:
            self.flush()

    def write_byte(self, b: int):      # Output.write(int) / writeByte
        if self.cap is not None and len(self.buf) == self.cap:
            self._require(1)
        self.buf.append(b & 0xFF)

    def write_varint(self, v: int, optimize_positive: bool = True):
        enc = varint(v, optimize_positive)
        self._require(len(enc))
        self.buf += enc

    def write_bytes(self, data: bytes):   # Output.writeBytes: fill the buffer, then whole buffers
        data = bytes(data)
        if self.cap is None:
            self.buf += data
            return
        i, n = 0, len(data)
        k = min(self.cap - len(self.buf), n)
        while True:
            self.buf += data[i:i + k]
            i += k
            if i == n:
                return
            k = min(self.cap, n - i)
            self._require(k)

    def write_string(self, s: str):
        enc = string(s)
        if len(enc) == len(s) and len(s) > 1:   # ASCII path: bytes (slow path = writeBytes), flag last
            self.write_bytes(enc[:-1] + bytes([enc[-1] & 0x7F]))
            self.buf[-1] |= 0x80
        else:
            for b in enc:
                self.write_byte(b)

    def flush(self):                   # OutputChunked.flush -> Output.flush -> parent.flush
        if self.parent is None:
            return
        if self.buf:
            for b in varint(len(self.buf)):   # writeChunkSize: outputStream.write(int) per byte
                self.parent.write_byte(b)
            self.parent.write_bytes(bytes(self.buf))
            self.buf.clear()
        self.parent.flush()

    def end_chunks(self):
        self.flush()
        self.parent.write_byte(0)


class Graph:
    """Per-graph state of one top-level writeClassAndObject: class-name ids, the classes whose
    CompatibleFieldSerializer field-name header is already out, and whether references are on."""

    def __init__(self, references: bool = True):
        self.name_ids: Dict[str, int] = {}
        self.headers: set = set()
        self.references = references

    def write_class(self, o: Out, cls) -> None:
        """DefaultClassResolver.writeClass: int = registered id, str = written by NAME."""
        if isinstance(cls, int):
            o.write_varint(cls + 2)
            return
        o.write_varint(NAME + 2)
        if cls in self.name_ids:
            o.write_varint(self.name_ids[cls])
            return
        nid = len(self.name_ids)
        self.name_ids[cls] = nid
        o.write_varint(nid)
        o.write_string(cls)

    def marker(self, o: Out) -> None:
        """writeReferenceOrNull for a first-seen object (references on only)."""
        if self.references:
            o.write_varint(NOT_NULL)

    def compatible(self, o: Out, cls: str, fields: List[Tuple[str, Callable[[Out], None]]]) -> None:
        """CompatibleFieldSerializer.write: fields = [(cached name, writer)], in cached-name order."""
        fields = sorted(fields, key=lambda f: f[0])
        if cls not in self.headers:
            self.headers.add(cls)
            o.write_varint(len(fields))
            for name, _ in fields:
                o.write_string(name)
        c = Out(o)
        for _, fn in fields:
            fn(c)
            c.end_chunks()


# ---- SignableData ----
def _bytes_field(g: Graph, data: bytes) -> Callable[[Out], None]:
    def w(o: Out):
        g.marker(o)                              # writeObjectOrNull of a final byte[] field
        o.write_varint(len(data) + 1)            # ByteArraySerializer: length + 1 (0 = null)
        o.write_bytes(data)
    return w


def _metadata_field(g: Graph, platform_version: int, scheme_number_id: int) -> Callable[[Out], None]:
    def w(o: Out):
        g.marker(o)                              # SignatureMetadata is final: marker + object
        g.compatible(o, SIGNATURE_METADATA, [
            ("SignatureMetadata.platformVersion", lambda c: c.write_varint(platform_version, False)),
            ("SignatureMetadata.schemeNumberID", lambda c: c.write_varint(scheme_number_id, False))])
    return w


def signable_data(tx_id: bytes, platform_version: int, scheme_number_id: int) -> bytes:
    """SignableData(SecureHash.SHA256(tx_id), SignatureMetadata(platformVersion, schemeNumberID))
    .serialize().bytes under the Kryo P2P context."""
    if len(tx_id) != 32:   # SecureHash.SHA256 init { require(bytes.size == 32) }
        raise KryoException("SecureHash.SHA256 needs 32 bytes")
    g = Graph()
    o = Out()
    o.write_bytes(KRYO_HEADER_V0_1)
    g.write_class(o, SIGNABLE_DATA)
    g.marker(o)

    def tx_field(c: Out):                        # SecureHash is sealed (abstract): class first
        g.write_class(c, SECURE_HASH_SHA256)
        g.marker(c)
        g.compatible(c, SECURE_HASH_SHA256, [("OpaqueBytes.bytes", _bytes_field(g, tx_id))])

    g.compatible(o, SIGNABLE_DATA, [
        ("SignableData.signatureMetadata", _metadata_field(g, platform_version, scheme_number_id)),
        ("SignableData.txId", tx_field)])
    return o.getvalue()


def signable_data_template(platform_version: int, scheme_number_id: int) -> Tuple[bytes, int]:
    """(template bytes without the id, id offset) — the chip_msg_templates convention: the message
    of every transaction signed with this metadata is t[:at] + txId + t[at:]."""
    a = signable_data(b"\x00" * 32, platform_version, scheme_number_id)
    b = signable_data(b"\xff" * 32, platform_version, scheme_number_id)
    diff = [i for i in range(len(a)) if a[i] != b[i]]
    at = diff[0]
    assert diff == list(range(at, at + 32)) and len(a) == len(b)
    return a[:at] + a[at + 32:], at


# ---- WireTransaction / SignedTransaction (Kryo.kt:236-280) ----
def _list(g: Graph, o: Out, items: Sequence, write_item: Callable[[Out, object], None], kind: str = "auto"):
    """writeClassAndObject(list): kind 'array' = ArrayList, 'single' = Collections$SingletonList,
    ('aslist', component class) = Arrays$ArrayList (listOf(a, b)); 'auto': singleton for one element
    (listOf(x)), else ArrayList (mutableListOf / map / plus)."""
    if kind == "auto":
        kind = "single" if len(items) == 1 else "array"
    if kind == "single":
        assert len(items) == 1
        g.write_class(o, SINGLETON_LIST)
        g.marker(o)
        write_item(o, items[0])                  # CollectionsSingletonListSerializer
    elif isinstance(kind, tuple) and kind[0] == "aslist":
        g.write_class(o, REG_ARRAYS_ASLIST)      # ArraysAsListSerializer: size, component class, elements
        g.marker(o)
        o.write_varint(len(items))
        g.write_class(o, kind[1])
        for it in items:
            write_item(o, it)
    else:
        g.write_class(o, ARRAY_LIST)
        g.marker(o)
        o.write_varint(len(items))               # CollectionSerializer: size, then class + object
        for it in items:
            write_item(o, it)


def wire_transaction(groups: Sequence[Tuple[int, Sequence[bytes]]], salt: bytes,
                     privacy_salt_id: int = DEFAULT_IDS["privacy_salt"], list_kinds: Optional[Dict] = None) -> bytes:
    """WireTransaction(componentGroups, privacySalt).serialize().bytes: groups = [(groupIndex,
    [component bytes = SerializedBytes of the component]), ...] in list order (createComponentGroups,
    WireTransaction.kt:207-221).  list_kinds optionally forces the list class per group index
    ('array' / 'single'); -1 = the componentGroups list itself."""
    kinds = list_kinds or {}
    g = Graph()
    o = Out()
    o.write_bytes(KRYO_HEADER_V0_1)
    g.write_class(o, REG_WIRE_TX)
    g.marker(o)                                  # references are still on for the top object
    g.references = False                         # NoReferencesSerializer (Kryo.kt:429-437)

    def ser_bytes(c: Out, b):                    # element: SerializedBytes, SerializedBytesSerializer
        g.write_class(c, REG_SERIALIZED_BYTES)
        g.marker(c)
        c.write_varint(len(b))
        c.write_bytes(b)

    def group(c: Out, gi_comps):
        gi, comps = gi_comps
        g.write_class(c, COMPONENT_GROUP)
        g.marker(c)
        g.compatible(c, COMPONENT_GROUP, [
            ("ComponentGroup.components", lambda f: _list(g, f, list(comps), ser_bytes, kinds.get(gi, "auto"))),
            ("ComponentGroup.groupIndex", lambda f: f.write_varint(gi, False))])

    _list(g, o, list(groups), group, kinds.get(-1, "array"))
    if len(salt) != 32:
        raise KryoException("Privacy salt should be 32 bytes.")
    g.write_class(o, privacy_salt_id)            # PrivacySaltSerializer: writeBytesWithLength
    o.write_varint(32)
    o.write_bytes(salt)
    return o.getvalue()


class Sig:
    """A TransactionSignature as the front end sees it."""

    def __init__(self, sig: bytes, key: bytes, platform_version: int = 1, scheme_number_id: int = 4,
                 key_class_id: Optional[int] = None):
        self.sig, self.key = bytes(sig), bytes(key)
        self.platform_version, self.scheme_number_id = platform_version, scheme_number_id
        self.key_class_id = key_class_id

    def tuple(self):
        return (self.sig, self.key, self.platform_version, self.scheme_number_id)


def signed_transaction(tx_bits: bytes, sigs: Sequence[Sig], list_kind: str = "auto") -> bytes:
    """SignedTransaction(txBits, sigs).serialize().bytes (SignedTransactionSerializer, Kryo.kt:266-280)."""
    g = Graph()
    o = Out()
    o.write_bytes(KRYO_HEADER_V0_1)
    g.write_class(o, REG_SIGNED_TX)
    g.marker(o)
    g.write_class(o, REG_SERIALIZED_BYTES)       # txBits
    g.marker(o)
    o.write_varint(len(tx_bits))
    o.write_bytes(tx_bits)

    def txsig(c: Out, s: Sig):
        g.write_class(c, TRANSACTION_SIGNATURE)
        g.marker(c)

        def by(f: Out):                          # PublicKey (interface): class, marker, PublicKeySerializer
            kid = s.key_class_id if s.key_class_id is not None else DEFAULT_REGISTRY.key_class_for(s.key)
            g.write_class(f, kid)
            g.marker(f)
            f.write_varint(len(s.key))
            f.write_bytes(s.key)

        g.compatible(c, TRANSACTION_SIGNATURE, [
            ("OpaqueBytes.bytes", _bytes_field(g, s.sig)),
            ("TransactionSignature.by", by),
            ("TransactionSignature.signatureMetadata", _metadata_field(g, s.platform_version, s.scheme_number_id))])

    _list(g, o, list(sigs), txsig, list_kind)
    return o.getvalue()


# ---- reader (host mirror of the device front end) ----
class Reader:
    """Input / InputChunked over one graph: chunk() returns the de-chunked bytes of one field as a
    reader sharing the graph's name ids and headers (InputChunked.nextChunks semantics: unread
    bytes of a field are skipped)."""

    def __init__(self, buf: bytes, pos: int = 0, end: Optional[int] = None, reg: Registry = DEFAULT_REGISTRY):
        self.buf = buf
        self.pos = pos
        self.end = len(buf) if end is None else end
        self.names: Dict[int, str] = {}
        self.headers: Dict[str, List[str]] = {}
        self.reg = reg
        self.bounds: List[int] = []      # a de-chunked field: where its chunks end

    def byte(self) -> int:
        if self.pos >= self.end:
            raise KryoException("buffer underflow")
        b = self.buf[self.pos]
        self.pos += 1
        return b

    def take(self, n: int) -> bytes:
        if n < 0 or self.pos + n > self.end:
            raise KryoException("buffer underflow")
        b = self.buf[self.pos:self.pos + n]
        self.pos += n
        return bytes(b)

    def varint(self, optimize_positive: bool = True) -> int:
        """Input.readVarInt: at most 5 bytes; the 5th byte's 7 bits all shift in (bits >= 32 drop)."""
        v = 0
        for i in range(5):
            b = self.byte()
            v |= (b & 0x7F) << (7 * i)
            if not b & 0x80:
                break
        v &= 0xFFFFFFFF
        if not optimize_positive:
            v = (v >> 1) ^ -(v & 1)
        return v

    def string(self, max_chars: int = 64) -> str:
        """Input.readString restricted to the form the grammar's names take (Output.writeString's ASCII
        form: bit 7 on the last byte): a UTF-8-form string, or one running past max_chars + 1 characters
        without its last byte, is outside the device grammar (KryoUnsupported)."""
        out = bytearray()
        for i in range(max_chars + 2):
            c = self.byte()
            if i == 0 and c & 0x80:
                raise KryoUnsupported("UTF-8 form string")
            out.append(c & 0x7F)
            if c & 0x80:
                return out.decode("ascii")
        raise KryoUnsupported("string longer than %d characters" % (max_chars + 1))

    def read_class(self):
        """-> registered id (int) or class name (str); None for a null."""
        tag = self.varint()
        if tag == NULL:
            return None
        if tag != NAME + 2:
            return tag - 2
        nid = self.varint()
        if nid not in self.names:
            if nid != len(self.names) or nid >= 8:     # the device keeps 8 name ids per graph
                raise KryoUnsupported("class name id %d" % nid)
            self.names[nid] = self.string(200)
        return self.names[nid]

    def not_null(self):
        if self.varint() != NOT_NULL:
            raise KryoUnsupported("expected a first-seen object (back-references / null unsupported)")

    def chunk(self) -> "Reader":
        data = bytearray()
        bounds = []
        while True:
            n = self.varint()
            if n == 0:
                break
            data += self.take(n)
            bounds.append(len(data))
        r = Reader(bytes(data), reg=self.reg)
        r.names, r.headers = self.names, self.headers   # one graph
        r.bounds = bounds
        return r

    def spans(self, n: int) -> bool:
        """The next n bytes cross a chunk boundary of this (de-chunked) field."""
        return any(self.pos < b < self.pos + n for b in self.bounds)


def _header(buf: bytes, reg: Registry = DEFAULT_REGISTRY) -> Reader:
    if bytes(buf[:8]) != KRYO_HEADER_V0_1:
        raise KryoException("Serialized bytes header does not match expected format.")
    return Reader(buf, 8, reg=reg)


def _expect_fields(r: Reader, cls: str, names: List[str]):
    if cls not in r.headers:
        n = r.varint()
        if n != len(names):
            raise KryoUnsupported("unexpected %s field count %d" % (cls, n))
        got = []
        for want in names:
            got.append(r.string())
            if got[-1] != want:
                raise KryoUnsupported("unexpected %s field %r" % (cls, got[-1]))
        r.headers[cls] = got


def _read_metadata(r: Reader) -> Tuple[int, int]:
    r.not_null()
    _expect_fields(r, SIGNATURE_METADATA, META_FIELDS)
    pv = r.chunk().varint(False)
    sch = r.chunk().varint(False)
    return pv, sch


def _read_list(r: Reader, references: bool, read_item: Callable[[Reader], object]) -> list:
    cls = r.read_class()
    if references:
        r.not_null()
    if cls == SINGLETON_LIST:
        return [read_item(r)]
    if cls == ARRAY_LIST:
        return [read_item(r) for _ in range(r.varint())]
    if cls == r.reg.arrays_aslist:
        n = r.varint()
        r.read_class()                           # the array's component class
        return [read_item(r) for _ in range(n)]
    raise KryoUnsupported("unsupported list class %r" % (cls,))


def parse_signable_data(buf: bytes) -> Tuple[bytes, int, int]:
    """Inverse of signable_data: (txId, platformVersion, schemeNumberID); KryoException on any
    other layout (trailing bytes included)."""
    r = _header(buf)
    if r.read_class() != SIGNABLE_DATA:
        raise KryoException("not a SignableData")
    r.not_null()
    _expect_fields(r, SIGNABLE_DATA, ["SignableData.signatureMetadata", "SignableData.txId"])
    pv, sch = _read_metadata(r.chunk())
    t = r.chunk()
    if t.read_class() != SECURE_HASH_SHA256:
        raise KryoException("txId is not a SecureHash.SHA256")
    t.not_null()
    _expect_fields(t, SECURE_HASH_SHA256, ["OpaqueBytes.bytes"])
    a = t.chunk()
    a.not_null()
    n = a.varint() - 1
    if n != 32:
        raise KryoException("txId is not 32 bytes")
    tx_id = a.take(32)
    if r.pos != len(buf):
        raise KryoException("trailing bytes")
    return tx_id, pv, sch


def parse_wire_transaction(buf: bytes, reg: Registry = DEFAULT_REGISTRY) -> Tuple[List[Tuple[int, List[bytes]]], bytes]:
    """WireTransactionSerializer.read (Kryo.kt:242-246): ([(groupIndex, [component bytes])], salt)."""
    r = _header(buf, reg)
    if r.read_class() != reg.wire_tx:
        raise KryoUnsupported("not a WireTransaction")
    r.not_null()

    def comp(c: Reader) -> bytes:
        if c.read_class() != reg.serialized_bytes:
            raise KryoUnsupported("component is not SerializedBytes")
        return c.take(c.varint())

    def group(c: Reader):
        if c.read_class() != COMPONENT_GROUP:
            raise KryoUnsupported("not a ComponentGroup")
        _expect_fields(c, COMPONENT_GROUP, GROUP_FIELDS)
        comps = _read_list(c.chunk(), False, comp)
        gi = c.chunk().varint(False)
        if not 0 <= gi < 64:                     # the device tracks group presence in 64 bits
            raise KryoUnsupported("group index %d" % gi)
        return gi, comps

    groups = _read_list(r, False, group)
    if r.read_class() != reg.privacy_salt:       # another registered class: another serializer
        raise KryoUnsupported("privacySalt is not the registered PrivacySalt class")
    if r.varint() != 32:                         # PrivacySalt.init require: left to the JVM path
        raise KryoUnsupported("Privacy salt should be 32 bytes.")
    salt = r.take(32)
    return groups, salt


def _key_class_ok(reg: Registry, kid) -> bool:
    """A key slot names a class registered with PublicKeySerializer (the same decode for all of them)."""
    return isinstance(kid, int) and kid in reg.public_key


def parse_signed_transaction(buf: bytes, reg: Registry = DEFAULT_REGISTRY) -> Tuple[bytes, List[Tuple[bytes, bytes, int, int]]]:
    """SignedTransactionSerializer.read (Kryo.kt:273-278): (txBits, [(sig, key SPKI, pv, scheme)])."""
    r = _header(buf, reg)
    if r.read_class() != reg.signed_tx:
        raise KryoUnsupported("not a SignedTransaction")
    r.not_null()
    if r.read_class() != reg.serialized_bytes:
        raise KryoUnsupported("txBits is not SerializedBytes")
    r.not_null()
    tx_bits = r.take(r.varint())

    def txsig(c: Reader):
        if c.read_class() != TRANSACTION_SIGNATURE:
            raise KryoUnsupported("not a TransactionSignature")
        c.not_null()
        _expect_fields(c, TRANSACTION_SIGNATURE, TXSIG_FIELDS)
        f = c.chunk()
        f.not_null()
        n = f.varint()
        if n == 0:
            raise KryoUnsupported("null signature bytes")
        sig = f.take(n - 1)
        f = c.chunk()
        if not _key_class_ok(reg, f.read_class()):
            raise KryoUnsupported("key class is not registered with PublicKeySerializer")
        f.not_null()
        key = f.take(f.varint())
        pv, sch = _read_metadata(c.chunk())
        return sig, key, pv, sch

    sigs = _read_list(r, True, txsig)
    return tx_bits, sigs


# ---- StateRef components (the inputs group: SerializedBytes<StateRef>, MerkleTransaction.kt:23) ----
STATE_REF = "net.corda.core.contracts.StateRef"
STATEREF_FIELDS = ["StateRef.index", "StateRef.txhash"]


def state_ref(txhash: bytes, index: int) -> bytes:
    """StateRef(SecureHash.SHA256(txhash), index).serialize().bytes (Structures.kt:143-145): fields sort as
    StateRef.index (zig-zag int), StateRef.txhash (SecureHash is sealed: class, marker, OpaqueBytes.bytes)."""
    if len(txhash) != 32:
        raise KryoException("SecureHash.SHA256 needs 32 bytes")
    g = Graph()
    o = Out()
    o.write_bytes(KRYO_HEADER_V0_1)
    g.write_class(o, STATE_REF)
    g.marker(o)

    def txh(c: Out):
        g.write_class(c, SECURE_HASH_SHA256)
        g.marker(c)
        g.compatible(c, SECURE_HASH_SHA256, [("OpaqueBytes.bytes", _bytes_field(g, txhash))])

    g.compatible(o, STATE_REF, [("StateRef.index", lambda c: c.write_varint(index, False)), ("StateRef.txhash", txh)])
    return o.getvalue()


def state_ref_of(comp: bytes) -> Optional[Tuple[bytes, int]]:
    """(txhash, index) when `comp` is the canonical encoding of a StateRef (what a JVM writes for it), else
    None.  checkNoDuplicateInputs compares decoded StateRefs (BaseTransaction.kt:37); requiring the
    canonical encoding makes byte equality of two inputs the same as StateRef equality, so the device
    compares bytes and hands anything else to the JVM path."""
    try:
        r = _header(comp)
        if r.read_class() != STATE_REF:
            return None
        r.not_null()
        _expect_fields(r, STATE_REF, STATEREF_FIELDS)
        index = r.chunk().varint(False)
        t = r.chunk()
        if t.read_class() != SECURE_HASH_SHA256:
            return None
        t.not_null()
        _expect_fields(t, SECURE_HASH_SHA256, ["OpaqueBytes.bytes"])
        a = t.chunk()
        a.not_null()
        if a.varint() != 33:
            return None
        h = a.take(32)
    except KryoException:
        return None
    return (h, index) if bytes(comp) == state_ref(h, index) else None


# ---- WireTransaction.init / SignedTransaction.init checks the device front end applies ----
GROUP_INPUTS, GROUP_OUTPUTS, GROUP_COMMANDS, GROUP_ATTACHMENTS, GROUP_NOTARY, GROUP_TIMEWINDOW = range(6)


def wire_invariant_error(groups: Sequence[Tuple[int, Sequence[bytes]]], check_duplicates: bool = True) -> Optional[str]:
    """The structural checks of WireTransaction deserialisation in the order the JVM meets them:
    TraversableTransaction's notary / time-window initialisers (MerkleTransaction.kt:30-40, the first group
    of each index), then WireTransaction.init (WireTransaction.kt:53-60, BaseTransaction.kt:30-37): the
    message of the IllegalStateException, or None."""
    first = {}
    for gi, comps in groups:
        first.setdefault(gi, comps)
    if len(first.get(GROUP_NOTARY, ())) > 1:
        return "Invalid Transaction. More than 1 notary party detected."
    if len(first.get(GROUP_TIMEWINDOW, ())) > 1:
        return "Invalid Transaction. More than 1 time-window detected."
    if not all(len(c) for _, c in groups):
        return "Empty component groups are not allowed"
    idx = [gi for gi, _ in groups]
    if len(set(idx)) != len(idx):
        return "Duplicated component groups detected"
    present = set(idx)
    if GROUP_INPUTS in present and GROUP_NOTARY not in present:
        return "The notary must be specified explicitly for any transaction that has inputs"
    inputs = [bytes(c) for gi, comps in groups if gi == GROUP_INPUTS for c in comps]
    if check_duplicates and len(set(inputs)) != len(inputs):      # canonical StateRefs: bytes = value
        return "Duplicate input states detected"
    if GROUP_INPUTS not in present and GROUP_OUTPUTS not in present:
        return "A transaction must contain at least one input or output state"
    if GROUP_COMMANDS not in present:
        return "A transaction must contain at least one command"
    if GROUP_TIMEWINDOW in present and GROUP_NOTARY not in present:
        return "Transactions with time-windows must be notarised"
    return None


# ---- the front end's verdict per SignedTransaction (host mirror of chip_stx_parse_device) ----
STX_OK, STX_KRYO, STX_NO_SIGS, STX_INVARIANT, STX_UNSUPPORTED = range(5)
MAX_INPUTS = 64          # the device's duplicate-input check covers <= 64 inputs
MAX_SIGNER_ENTRIES = 64  # commands' signers + the notary, before de-duplication


def stx_parse(buf: bytes, reg: Registry = DEFAULT_REGISTRY):
    """-> (status, groups, salt, sigs): what SignedTransaction deserialisation, the lazy WireTransaction
    deserialisation and their init checks make of `buf`, in the order the JVM meets them (cordahip.h
    chip_stx_status).  groups / salt / sigs are None unless status is STX_OK.  After the structural
    checks: an input that is not a canonical StateRef, or more than 64 inputs -> STX_UNSUPPORTED; then
    duplicate inputs -> STX_INVARIANT."""
    try:
        tx_bits, sigs = parse_signed_transaction(buf, reg)
    except KryoUnsupported:
        return STX_UNSUPPORTED, None, None, None
    except KryoException:
        return STX_KRYO, None, None, None
    if not sigs:                                 # SignedTransaction.init require(sigs.isNotEmpty())
        return STX_NO_SIGS, None, None, None
    try:
        groups, salt = parse_wire_transaction(tx_bits, reg)
    except KryoUnsupported:
        return STX_UNSUPPORTED, None, None, None
    except KryoException:
        return STX_KRYO, None, None, None
    if wire_invariant_error(groups, check_duplicates=False) is not None:
        return STX_INVARIANT, None, None, None
    inputs = [c for gi, cs in groups if gi == GROUP_INPUTS for c in cs]
    if any(state_ref_of(c) is None for c in inputs) or len(inputs) > MAX_INPUTS:
        return STX_UNSUPPORTED, None, None, None
    if wire_invariant_error(groups) is not None:
        return STX_INVARIANT, None, None, None
    return STX_OK, groups, salt, sigs


# ---- component contents the front end reads: Command.signers, the notary Party's owningKey ----
COMMAND = "net.corda.core.contracts.Command"
PARTY = "net.corda.core.identity.Party"
CORDA_X500_NAME = "net.corda.core.identity.CordaX500Name"
COMMAND_FIELDS = ["Command.signers", "Command.value"]
PARTY_FIELDS = ["AbstractParty.owningKey", "Party.name"]


def _key_object(g: Graph, o: Out, key: bytes, key_class_id) -> None:
    """A PublicKey through an interface-typed slot: class, marker, PublicKeySerializer
    (writeBytesWithLength of the X.509 encoding, Kryo.kt:299-310)."""
    g.write_class(o, key_class_id)
    g.marker(o)
    o.write_varint(len(key))
    o.write_bytes(key)


def command(signers: Sequence[bytes], value_class: str = "net.corda.finance.contracts.asset.Cash$Commands$Move",
            key_class_id=None, list_kind="auto") -> bytes:
    """Command(value, signers).serialize().bytes (Structures.kt:179-185): a CompatibleFieldSerializer
    object whose fields sort as Command.signers, Command.value; the value here is an object of
    `value_class` with no fields (the front end reads only the signers).  key_class_id None = the class
    a JVM writes for each key (EdDSAPublicKey / BCECPublicKey / CompositeKey)."""
    g = Graph()
    o = Out()
    o.write_bytes(KRYO_HEADER_V0_1)
    g.write_class(o, COMMAND)
    g.marker(o)

    def value(c: Out):
        g.write_class(c, value_class)
        g.marker(c)
        g.compatible(c, value_class, [])

    g.compatible(o, COMMAND, [
        ("Command.signers", lambda c: _list(g, c, list(signers), lambda f, k: _key_object(
            g, f, k, DEFAULT_REGISTRY.key_class_for(k) if key_class_id is None else key_class_id), list_kind)),
        ("Command.value", value)])
    return o.getvalue()


def party(owning_key: bytes, name: str = "O=Notary Service,L=Zurich,C=CH", key_class_id=None) -> bytes:
    """Party(name, owningKey).serialize().bytes (Party.kt:29, AbstractParty.kt:13): fields sort as
    AbstractParty.owningKey, Party.name; the name is a CordaX500Name with its string fields."""
    g = Graph()
    o = Out()
    o.write_bytes(KRYO_HEADER_V0_1)
    g.write_class(o, PARTY)
    g.marker(o)

    def name_field(c: Out):
        g.marker(c)                              # CordaX500Name is final: marker + object
        parts = dict(p.split("=", 1) for p in name.split(","))

        def s(v):
            def w(f: Out):
                if v is None:
                    f.write_byte(0x80)           # writeString(null)
                else:
                    f.write_string(v)
            return w
        g.compatible(c, CORDA_X500_NAME, [
            ("CordaX500Name.commonName", s(parts.get("CN"))), ("CordaX500Name.country", s(parts.get("C"))),
            ("CordaX500Name.locality", s(parts.get("L"))), ("CordaX500Name.organisation", s(parts.get("O"))),
            ("CordaX500Name.organisationUnit", s(parts.get("OU"))), ("CordaX500Name.state", s(parts.get("ST")))])

    g.compatible(o, PARTY, [
        ("AbstractParty.owningKey", lambda c: _key_object(
            g, c, owning_key, DEFAULT_REGISTRY.key_class_for(owning_key) if key_class_id is None else key_class_id)),
        ("Party.name", name_field)])
    return o.getvalue()


def _read_key_object(r: Reader) -> bytes:
    """A command signer / the notary's owningKey.  The device reads these keys in place in the component:
    one whose bytes cross a chunk boundary of their field is outside its grammar (the JVM path decides)."""
    if not _key_class_ok(r.reg, r.read_class()):
        raise KryoUnsupported("key class is not registered with PublicKeySerializer")
    r.not_null()
    n = r.varint()
    if r.spans(n):
        raise KryoUnsupported("key spans a chunk boundary")
    return r.take(n)


def command_signers(buf: bytes, reg: Registry = DEFAULT_REGISTRY) -> List[bytes]:
    """Command.signers of a command component (the value is not read).  An empty list is what Command.init
    rejects (require(signers.isNotEmpty()), Structures.kt:183): the JVM path decides that transaction."""
    r = _header(buf, reg)
    if r.read_class() != COMMAND:
        raise KryoUnsupported("not a Command")
    r.not_null()
    _expect_fields(r, COMMAND, COMMAND_FIELDS)
    out = _read_list(r.chunk(), True, _read_key_object)
    if not out:
        raise KryoUnsupported("Command with no signers")
    return out


def party_owning_key(buf: bytes, reg: Registry = DEFAULT_REGISTRY) -> bytes:
    """AbstractParty.owningKey of a notary component."""
    r = _header(buf, reg)
    if r.read_class() != PARTY:
        raise KryoUnsupported("not a Party")
    r.not_null()
    _expect_fields(r, PARTY, PARTY_FIELDS)
    return _read_key_object(r.chunk())


def required_signing_keys(groups: Sequence[Tuple[int, Sequence[bytes]]], reg: Registry = DEFAULT_REGISTRY) -> List[bytes]:
    """WireTransaction.requiredSigningKeys (WireTransaction.kt:66-75): commands.flatMap { signers }.toSet()
    + notary.owningKey when the transaction has inputs or a time-window, in first-appearance order (the
    order of the device's required-key ranges).  Keys compare by their encoding."""
    out: List[bytes] = []
    seen = set()
    for k in _signer_entries(groups, reg)[0]:
        if k not in seen:
            seen.add(k)
            out.append(k)
    return out


def _signer_entries(groups, reg):
    """(commands' signers then the notary when required, the notary key or None)."""
    entries: List[bytes] = []
    present = {gi for gi, _ in groups}
    for gi, comps in groups:
        if gi == GROUP_COMMANDS:
            for c in comps:
                entries += command_signers(c, reg)
    notary = None
    for gi, comps in groups:
        if gi == GROUP_NOTARY:
            notary = party_owning_key(comps[0], reg)
            break
    if notary is not None and (GROUP_INPUTS in present or GROUP_TIMEWINDOW in present):
        entries.append(notary)
    return entries, notary


def required_key_trees(groups, sig_keys, reg: Registry = DEFAULT_REGISTRY):
    """requiredSigningKeys as the device derives them (CHIP_STX_REQUIRED): per distinct key its tree of
    post-order nodes (keys.Node: a plain key is one leaf, a CompositeKey its canonical tree).  Raises
    KryoUnsupported for what the device hands to the JVM path: a command / notary component outside the
    grammar, an empty signers list, more than 64 signer entries, a key that is neither a decodable
    Ed25519 / ECDSA key nor a canonical CompositeKey (keys.py).  A plain key that signs none of this
    transaction's signatures (`sig_keys`: its signatures' key bytes) is decoded here — the verify path
    decodes the others — and so is the notary's key when the notary is not required."""
    from corda_amd import keys as KS

    def tree_of(k: bytes):
        if KS.is_composite(k):
            return KS.composite_tree(k)
        if KS.spki_scheme(k)[0]:
            if k not in sig_keys and not KS.plain_key_ok(k):
                raise KryoUnsupported("undecodable key")
            return [(k, 0, 0, 1)]
        raise KryoUnsupported("key type")

    try:
        entries, notary = _signer_entries(groups, reg)
        if len(entries) > MAX_SIGNER_ENTRIES:
            raise KryoUnsupported("more than %d signer entries" % MAX_SIGNER_ENTRIES)
        if notary is not None:
            tree_of(notary)                      # deserialised whether or not it must sign
        trees, seen = [], set()
        for k in entries:
            t = tree_of(k)
            if k not in seen:
                seen.add(k)
                trees.append(t)
        return trees
    except KS.KeyUnsupported as e:
        raise KryoUnsupported(str(e))
