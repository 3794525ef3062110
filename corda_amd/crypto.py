"""Host-side mirror of the reference's hot-path API over the libcordahip engine (Python).

Same names, argument meaning and exceptions as the Kotlin it mirrors, so call sites and tests read
like the reference's:

  Crypto.findSignatureScheme / doVerify / isValid      core/.../crypto/Crypto.kt:235-267,502-625
  TransactionSignature.verify                          core/.../crypto/TransactionSignature.kt:26-40
  SignedTransaction / TransactionWithSignatures        core/.../transactions/TransactionWithSignatures.kt:29-85,
    .checkSignaturesAreValid / getMissingSigners /       SignedTransaction.kt:37-76,136-173,228-229
     verifySignaturesExcept / verifyRequiredSignatures
  WireTransaction.id / requiredSigningKeys / invariants core/.../transactions/WireTransaction.kt:53-75,139-189
  PersistentUniquenessProvider.commit                  node/.../transactions/PersistentUniquenessProvider.kt:92-113
  TrustedAuthorityNotaryService.commitInputStates      core/.../node/services/NotaryService.kt:61-75

Every cryptographic operation is one batched engine call.  `engine` is a corda_amd.Context (the HIP
path); any object with the same verify_batch / txid_batch / uniq_open methods can stand in (the CPU
tests plug the oracle in to exercise the host logic without a GPU).  There is no CPU fallback here.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Set, Tuple

import numpy as np

from .native import (VALID, INVALID, SIG_DECODE, EMPTY_SIG, EMPTY_CLEAR, UNSUPPORTED, KEY_INVALID)
from .composite import CompositeKey, IllegalArgumentException, as_key, is_fulfilled_by
from . import kryo


# ---- exceptions (java.security / IllegalArgumentException / Corda exceptions) ----
class SignatureException(Exception):
    pass


class InvalidKeyException(Exception):
    pass


class UnsupportedSchemeError(IllegalArgumentException):
    """CHIP_UNSUPPORTED: RSA / SPHINCS / composite keys stay on the JCA path (not accelerated)."""


class SignaturesMissingException(SignatureException):
    """SignedTransaction.SignaturesMissingException (SignedTransaction.kt:228-229)."""

    def __init__(self, missing: Set[bytes], descriptions: List[str], id: bytes):
        super().__init__("Missing signatures for %s on transaction %s for %s" %
                         (len(missing), id.hex().upper(), ", ".join(descriptions)))
        self.missing = missing
        self.descriptions = descriptions
        self.id = id


class UniquenessException(Exception):
    def __init__(self, conflict: "Conflict"):
        super().__init__("UniquenessException")
        self.error = conflict


class CommitLogFailure(RuntimeError):
    """The commit log could not be made durable: the provider stops accepting commits (fail-stop)
    and must be reopened, which rebuilds the table from the rows that did reach the log."""


class NotaryException(Exception):
    def __init__(self, tx_id: bytes, conflict: "Conflict"):
        super().__init__("Notary conflict for %s" % tx_id.hex())
        self.tx_id = tx_id
        self.conflict = conflict


# ---- signature schemes (Crypto.kt:84-128) and key -> scheme (Crypto.findSignatureScheme) ----
@dataclass(frozen=True)
class SignatureScheme:
    scheme_number_id: int
    scheme_code_name: str


ECDSA_SECP256K1_SHA256 = SignatureScheme(2, "ECDSA_SECP256K1_SHA256")
ECDSA_SECP256R1_SHA256 = SignatureScheme(3, "ECDSA_SECP256R1_SHA256")
EDDSA_ED25519_SHA512 = SignatureScheme(4, "EDDSA_ED25519_SHA512")

_SPKI_ED25519 = bytes.fromhex("302a300506032b6570032100")
_OID_R1 = bytes.fromhex("06082a8648ce3d030107")
_OID_K1 = bytes.fromhex("06052b8104000a")


def find_signature_scheme(key: bytes) -> SignatureScheme:
    """The scheme of an X.509 SubjectPublicKeyInfo (PublicKey.encoded), from its algorithm OID."""
    if len(key) == 44 and key[:12] == _SPKI_ED25519:
        return EDDSA_ED25519_SHA512
    if len(key) in (91, 59) and key[13:23] == _OID_R1:
        return ECDSA_SECP256R1_SHA256
    if len(key) in (88, 56) and key[13:20] == _OID_K1:
        return ECDSA_SECP256K1_SHA256
    raise IllegalArgumentException("Unsupported key/algorithm for schemeCodeName")


def _raise_for(status: int, key: bytes):
    """The exception Crypto.doVerify throws for a non-VALID status byte."""
    if status == INVALID:
        raise SignatureException("Signature Verification failed!")
    if status == SIG_DECODE:
        try:
            ed = find_signature_scheme(key) == EDDSA_ED25519_SHA512
        except IllegalArgumentException:
            ed = False
        raise SignatureException("signature length is wrong" if ed else "error decoding signature bytes.")
    if status == EMPTY_SIG:
        raise IllegalArgumentException("Signature data is empty!")
    if status == EMPTY_CLEAR:
        raise IllegalArgumentException("Clear data is empty, nothing to verify!")
    if status == KEY_INVALID:
        raise InvalidKeyException("invalid key: not a valid curve point")
    if status == UNSUPPORTED:
        raise UnsupportedSchemeError("Unsupported key/algorithm (JCA path)")
    raise SignatureException("unknown status %d" % status)


# ---- batch packing (chip_sig_batch SoA layout; keys and messages de-duplicated) ----
class SigBatch:
    def __init__(self, items: Sequence[Tuple[bytes, bytes, bytes]]):
        kid: Dict[bytes, int] = {}
        mid: Dict[bytes, int] = {}
        keys: List[bytes] = []
        msgs: List[bytes] = []
        key_idx, msg_idx, sigs = [], [], []
        for k, s, m in items:
            if k not in kid:
                kid[k] = len(keys)
                keys.append(k)
            if m not in mid:
                mid[m] = len(msgs)
                msgs.append(m)
            key_idx.append(kid[k])
            msg_idx.append(mid[m])
            sigs.append(s)
        self.key_index = kid                  # SPKI bytes -> key pool index
        self.key_idx = np.array(key_idx, dtype=np.uint32)
        self.msg_idx = np.array(msg_idx, dtype=np.uint32)
        self.sig_data, self.sig_off, self.sig_len = _pool(sigs)
        self.key_data, self.key_off, self.key_len = _pool(keys)
        self.msg_data, self.msg_off, self.msg_len = _pool(msgs)

    @property
    def n(self):
        return len(self.key_idx)


def _pool(items: List[bytes]):
    lens = np.fromiter((len(x) for x in items), dtype=np.uint32, count=len(items))
    off = np.zeros(len(items), dtype=np.uint64)
    if len(items) > 1:
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    data = np.frombuffer(b"".join(items), dtype=np.uint8).copy() if items else np.zeros(0, np.uint8)
    if len(data) == 0:
        data = np.zeros(1, dtype=np.uint8)
    return data, off, lens


def verify_statuses(engine, items: Sequence[Tuple[bytes, bytes, bytes]], is_valid: bool = False) -> np.ndarray:
    """CHIP_* status of every (key, signature, clear data) triple, one engine call.  is_valid=True:
    Crypto.isValid semantics (chip_is_valid_batch: no empty-input checks, Crypto.kt:615-625)."""
    if not items:
        return np.zeros(0, dtype=np.uint8)
    if is_valid:
        status, _ = engine.verify_batch(SigBatch(items), is_valid=True)
    else:
        status, _ = engine.verify_batch(SigBatch(items))
    return status


class Crypto:
    """net.corda.core.crypto.Crypto (verification half)."""

    @staticmethod
    def find_signature_scheme(key: bytes) -> SignatureScheme:
        return find_signature_scheme(key)

    @staticmethod
    def do_verify(engine, public_key: bytes, signature_data: bytes, clear_data: bytes) -> bool:
        """True, or the exception Crypto.doVerify(PublicKey, ByteArray, ByteArray) throws (Crypto.kt:502-536)."""
        st = int(verify_statuses(engine, [(public_key, signature_data, clear_data)])[0])
        if st != VALID:
            _raise_for(st, public_key)
        return True

    @staticmethod
    def is_valid(engine, public_key: bytes, signature_data: bytes, clear_data: bytes) -> bool:
        """False on a bad signature; engine decode errors still throw (Crypto.kt:600-625).  No empty
        checks: an empty signature is the engine's decode SignatureException, empty clear data is
        verified as the empty message."""
        st = int(verify_statuses(engine, [(public_key, signature_data, clear_data)], is_valid=True)[0])
        if st == VALID:
            return True
        if st == INVALID:
            return False
        _raise_for(st, public_key)


# ---- SignableData(txId, SignatureMetadata).serialize() ----
@dataclass(frozen=True)
class SignatureMetadata:
    platform_version: int = 1
    scheme_number_id: int = 4


def signable_template(meta: SignatureMetadata) -> Tuple[bytes, int]:
    """(template bytes without the id, id offset) of SignableData(txId, meta).serialize() — the Kryo
    4.0.0 P2P-context bytes restated in corda_amd.kryo (parity unpinned: no JVM, no reference-held
    bytes).  For one metadata value the message is a fixed byte string with the 32-byte id at a fixed
    offset, which is what chip_verify_tx_batch relies on."""
    return kryo.signable_data_template(meta.platform_version, meta.scheme_number_id)


def signable_data_bytes(tx_id: bytes, meta: SignatureMetadata) -> bytes:
    """SignableData(txId, meta).serialize().bytes (Crypto.kt:550-578, SignableData.kt:12-13)."""
    return kryo.signable_data(tx_id, meta.platform_version, meta.scheme_number_id)


Serializer = Callable[[bytes, SignatureMetadata], bytes]


@dataclass
class TransactionSignature:
    bytes: bytes
    by: bytes                                  # PublicKey.encoded (SPKI)
    signature_metadata: SignatureMetadata = field(default_factory=SignatureMetadata)

    def verify(self, engine, tx_id: bytes, serializer: Serializer = signable_data_bytes) -> bool:
        """TransactionSignature.verify(txId) = Crypto.doVerify(txId, this) (TransactionSignature.kt:26-30)."""
        return Crypto.do_verify(engine, self.by, self.bytes, serializer(tx_id, self.signature_metadata))


class SignedTransaction:
    """The signature half of SignedTransaction / TransactionWithSignatures."""

    def __init__(self, id: bytes, sigs: List[TransactionSignature], required_signing_keys: Iterable[bytes],
                 serializer: Serializer = signable_data_bytes, key_descriptions: Optional[Dict[bytes, str]] = None):
        if not sigs:   # SignedTransaction.kt:46
            raise IllegalArgumentException("Tried to instantiate a SignedTransaction without any signatures ")
        self.id = id
        self.sigs = sigs
        self.required_signing_keys = set(required_signing_keys)
        self.serializer = serializer
        self.key_descriptions = key_descriptions or {}

    def _items(self):
        return [(s.by, s.bytes, self.serializer(self.id, s.signature_metadata)) for s in self.sigs]

    def check_signatures_are_valid(self, engine):
        """TransactionWithSignatures.kt:62-66: the first failing signature in list order throws."""
        for st, s in zip(verify_statuses(engine, self._items()), self.sigs):
            if st != VALID:
                _raise_for(int(st), s.by)

    def get_missing_signers(self) -> Set[bytes]:
        """TransactionWithSignatures.kt:79-85: required keys not fulfilled by the signers' keys (set
        membership for a plain key; weighted thresholds for a CompositeKey, corda_amd.composite)."""
        sig_keys = [s.by for s in self.sigs]
        return {k for k in self.required_signing_keys if not is_fulfilled_by(k, sig_keys)}

    def verify_signatures_except(self, engine, *allowed_to_be_missing: bytes):
        """TransactionWithSignatures.kt:44-50."""
        self.check_signatures_are_valid(engine)
        self._check_missing(allowed_to_be_missing)

    def verify_required_signatures(self, engine):
        self.verify_signatures_except(engine)

    def _check_missing(self, allowed):
        needed = self.get_missing_signers() - set(allowed)
        if needed:
            desc = sorted(self.key_descriptions.get(k, _short(k)) for k in needed)
            raise SignaturesMissingException(needed, desc, self.id)


def _short(k) -> str:
    return ("composite:" + k.encoded.hex()[-16:]) if isinstance(k, CompositeKey) else k.hex()[-16:]


def composite_signature_verify(engine, verify_key, sigs: Sequence[TransactionSignature], clear_data: bytes,
                               serializer: Serializer = signable_data_bytes) -> bool:
    """CompositeSignature.State.engineVerify (CompositeSignature.kt:77-86): the composite key must be
    fulfilled by the signers; then the buffered clear data IS the transaction id —
    SecureHash.SHA256(bytes) wraps the 32 bytes without hashing and requires size == 32
    (SecureHash.kt:16-19) — and every component signature must pass TransactionSignature.isValid(id)
    (Crypto.isValid semantics), all of them in one engine call.  `sigs.all {}` stops at the first
    false, so a decode failure after an invalid signature does not throw."""
    key = as_key(verify_key)
    if not isinstance(key, CompositeKey):
        raise IllegalArgumentException("verify key is not a CompositeKey")
    if not key.is_fulfilled_by([s.by for s in sigs]):
        return False
    if len(clear_data) != 32:
        raise IllegalArgumentException("Provided bytes are not 32 bytes long")
    tx_id = bytes(clear_data)
    items = [(s.by, s.bytes, serializer(tx_id, s.signature_metadata)) for s in sigs]
    for st, s in zip(verify_statuses(engine, items, is_valid=True), sigs):
        if st == INVALID:
            return False
        if st != VALID:
            _raise_for(int(st), s.by)
    return True


REQ_NO_SIGNER = 0xFFFFFFFF
REQ_MAX_PENDING = 64      # CHIP_REQ_MAX_PENDING: pending subtrees of one key tree on the device
TXV_OK, TXV_SIGNATURE, TXV_MISSING, TXV_MALFORMED = range(4)


class ReqBatch:
    """chip_req_batch layout: every transaction's required signing keys as post-order key trees over
    the key pool of the signature batch `sigs` (a SigBatch over the same transactions' signatures,
    in order), plus the allowedToBeMissing flags.  A CompositeKey is validated here
    (CompositeKey.checkValidity, which isFulfilledBy runs first, CompositeKey.kt:192-198); a transaction
    whose required key fails validation gets no required keys and its exception in `errors[t]`."""

    def __init__(self, txs: Sequence["SignedTransaction"], sigs: "SigBatch", allowed_to_be_missing: Iterable = ()):
        allowed = {as_key(k) for k in allowed_to_be_missing}
        sig_start, req_start, node_start = [0], [0], [0]
        val, nk, w, allow = [], [], [], []
        self.required: List[List] = []
        self.errors: List[Optional[Exception]] = []
        pos = 0
        for tx in txs:
            pos += len(tx.sigs)
            sig_start.append(pos)
            keys = [as_key(k) for k in tx.required_signing_keys]
            err = None
            try:
                for k in keys:
                    if isinstance(k, CompositeKey):
                        k.check_validity()
            except (IllegalArgumentException, ArithmeticError) as e:
                err, keys = e, []
            self.errors.append(err)
            self.required.append(keys)
            for k in keys:
                self._flatten(k, 1, sigs.key_index, val, nk, w)
                node_start.append(len(val))
                allow.append(1 if k in allowed else 0)
            req_start.append(len(allow))
        self.ntx = len(txs)
        self.sig_start = np.array(sig_start, dtype=np.uint64)
        self.req_start = np.array(req_start, dtype=np.uint64)
        self.node_start = np.array(node_start, dtype=np.uint64)
        self.allowed = np.array(allow or [0], dtype=np.uint8)
        self.node_val = np.array(val or [0], dtype=np.uint32)
        self.node_nkids = np.array(nk or [0], dtype=np.uint32)
        self.node_weight = np.array(w or [0], dtype=np.uint32)
        if not val:       # keep array lengths = node counts (n_nodes is taken from node_val)
            self.node_val, self.node_nkids, self.node_weight = (np.zeros(0, np.uint32),) * 3
        if not allow:
            self.allowed = np.zeros(0, np.uint8)

    @staticmethod
    def _flatten(key, weight, kid, val, nk, w, depth=0):
        """Post-order: children (each with its weight in this node), then the node itself."""
        if isinstance(key, CompositeKey):
            for child, cw in key.children:
                ReqBatch._flatten(child, cw, kid, val, nk, w, depth + 1)
            val.append(key.threshold)
            nk.append(len(key.children))
        else:
            val.append(kid.get(bytes(key), REQ_NO_SIGNER))
            nk.append(0)
        w.append(weight)

    def check_limits(self):
        """The device evaluates a key tree with at most REQ_MAX_PENDING pending subtrees (a CompositeKey
        node with that many children, or that deep a left spine): wider trees are refused up front."""
        sp, starts = 0, set(self.node_start.tolist())
        for j, n in enumerate(self.node_nkids.tolist()):
            if j in starts:
                sp = 0
            sp = sp - n + 1
            if sp > REQ_MAX_PENDING:
                raise IllegalArgumentException("key tree needs more than %d pending subtrees" % REQ_MAX_PENDING)


def verify_signatures_except_batch(engine, txs: Sequence[SignedTransaction],
                                   allowed_to_be_missing: Iterable[bytes] = ()) -> List[Optional[Exception]]:
    """Batch site (ResolveTransactionsFlow.kt:91-98 style): every transaction's signatures in ONE
    engine call, then the required-signer check of every transaction in one more (chip_required_signers:
    first failing signature, getMissingSigners with CompositeKey thresholds, minus allowedToBeMissing,
    TransactionWithSignatures.kt:44-50,62-66,79-85).  result[i] is None when transaction i passes
    verifySignaturesExcept, else the exception its own sequential call would have raised first."""
    items = [it for tx in txs for it in tx._items()]
    res: List[Optional[Exception]] = [None] * len(txs)
    if not txs:
        return res
    sb = SigBatch(items)
    st, _ = engine.verify_batch(sb) if items else (np.zeros(0, np.uint8), None)
    q = ReqBatch(txs, sb, allowed_to_be_missing)
    q.check_limits()
    verdict, arg, missing = engine.required_signers(q, sb, st)
    sig_base = q.sig_start
    for t, tx in enumerate(txs):
        v = int(verdict[t])
        if v == TXV_SIGNATURE:
            j = int(arg[t])
            try:
                _raise_for(int(st[j]), tx.sigs[j - int(sig_base[t])].by)
            except Exception as e:   # noqa: BLE001 - the reference exception is the result
                res[t] = e
        elif q.errors[t] is not None:
            res[t] = q.errors[t]     # CompositeKey.checkValidity inside isFulfilledBy
        elif v == TXV_MISSING:
            r0 = int(q.req_start[t])
            needed = {k for i, k in enumerate(q.required[t]) if missing[r0 + i]}
            desc = sorted(tx.key_descriptions.get(k, _short(k)) for k in needed)
            res[t] = SignaturesMissingException(needed, desc, tx.id)
        elif v != TXV_OK:
            raise RuntimeError("required-signer batch malformed at transaction %d" % t)
    return res


def resolve_transactions_verify(engine, txs: Sequence[SignedTransaction],
                                inputs_of: Callable[[SignedTransaction], Iterable[bytes]]):
    """ResolveTransactionsFlow's verification loop (ResolveTransactionsFlow.kt:83-99) as one batch:
    topologicalSort (:37-62, dependencies before dependers, deterministic for a given input order), then
    verifySignaturesExcept() of every transaction through verify_signatures_except_batch.  Returns
    (sorted transactions, the first failure in that order as (index, exception) or None) — the sequential
    loop would stop at that transaction, having verified the ones before it."""
    order = topological_sort(txs, inputs_of)
    res = verify_signatures_except_batch(engine, order)
    for i, e in enumerate(res):
        if e is not None:
            return order, (i, e)
    return order, None


def topological_sort(txs: Sequence[SignedTransaction], inputs_of) -> List[SignedTransaction]:
    """ResolveTransactionsFlow.topologicalSort (ResolveTransactionsFlow.kt:37-62)."""
    forward: Dict[bytes, List[SignedTransaction]] = {}
    for stx in txs:
        for txhash in inputs_of(stx):
            lst = forward.setdefault(bytes(txhash), [])
            if all(x is not stx for x in lst):       # LinkedHashSet
                lst.append(stx)
    visited: Set[bytes] = set()
    result: List[SignedTransaction] = []

    def visit(stx):          # the reference's recursive visit(), with an explicit stack
        if stx.id in visited:
            return
        visited.add(stx.id)
        stack = [(stx, iter(forward.get(stx.id, [])))]
        while stack:
            node, it = stack[-1]
            nxt = next(it, None)
            if nxt is None:
                stack.pop()
                result.append(node)
            elif nxt.id not in visited:
                visited.add(nxt.id)
                stack.append((nxt, iter(forward.get(nxt.id, []))))

    for stx in txs:
        visit(stx)
    result.reverse()
    if len(result) != len(txs):
        raise IllegalArgumentException("Failed requirement.")
    return result


# ---- WireTransaction ----
INPUTS_GROUP, OUTPUTS_GROUP, COMMANDS_GROUP, ATTACHMENTS_GROUP, NOTARY_GROUP, TIMEWINDOW_GROUP = range(6)


class TxBatch:
    """chip_tx_batch SoA layout."""

    def __init__(self, txs: Sequence["WireTransaction"]):
        salts, start, grp, internal, items = [], [0], [], [], []
        for tx in txs:
            tx.check_invariants()
            salts.append(tx.privacy_salt)
            for g, comps in sorted(tx.component_groups, key=lambda x: x[0]):
                for i, c in enumerate(comps):
                    grp.append(g)
                    internal.append(i)
                    items.append(c)
            start.append(len(grp))
        self.ntx = len(txs)
        self.salts = np.frombuffer(b"".join(salts), dtype=np.uint8).copy() if salts else np.zeros(0, np.uint8)
        self.tx_comp_start = np.array(start, dtype=np.uint64)
        self.comp_group = np.array(grp, dtype=np.uint32)
        self.comp_internal = np.array(internal, dtype=np.uint32)
        self.data, self.comp_off, self.comp_len = _pool(items)


class WireTransaction:
    """Component groups [(groupIndex, [serialized component bytes])] + PrivacySalt.  The required
    signers are carried as keys (the serialized commands are opaque to this layer)."""

    def __init__(self, component_groups: List[Tuple[int, List[bytes]]], privacy_salt: bytes,
                 command_signers: Iterable[bytes] = (), notary_key: Optional[bytes] = None):
        self.component_groups = component_groups
        self.privacy_salt = privacy_salt
        self.command_signers = list(command_signers)
        self.notary_key = notary_key

    def _group(self, g):
        for gi, comps in self.component_groups:
            if gi == g:
                return comps
        return []

    def check_invariants(self):
        """WireTransaction.kt:53-60 (the invariants the id depends on)."""
        idx = [g for g, _ in self.component_groups]
        if any(not comps for _, comps in self.component_groups):
            raise IllegalArgumentException("Empty component groups are not allowed")
        if len(set(idx)) != len(idx):
            raise IllegalArgumentException("Duplicated component groups detected")
        if any(g < 0 or g >= 64 for g in idx):
            raise IllegalArgumentException("component group ordinal outside [0, 64)")
        if not self._group(INPUTS_GROUP) and not self._group(OUTPUTS_GROUP):
            raise IllegalArgumentException("A transaction must contain at least one input or output state")
        if not self._group(COMMANDS_GROUP):
            raise IllegalArgumentException("A transaction must contain at least one command")
        if self._group(TIMEWINDOW_GROUP) and not self._group(NOTARY_GROUP):
            raise IllegalArgumentException("Transactions with time-windows must be notarised")
        if len(self.privacy_salt) != 32 or self.privacy_salt == bytes(32):
            raise IllegalArgumentException("Privacy salt should be 32 bytes and not all zeros")

    @property
    def required_signing_keys(self) -> Set[bytes]:
        """WireTransaction.kt:66-75."""
        keys = set(self.command_signers)
        if self.notary_key is not None and (self._group(INPUTS_GROUP) or self._group(TIMEWINDOW_GROUP)):
            keys.add(self.notary_key)
        return keys

    def id(self, engine) -> bytes:
        return WireTransaction.ids(engine, [self])[0]

    @staticmethod
    def ids(engine, txs: Sequence["WireTransaction"]) -> List[bytes]:
        """Batch WireTransaction.id (one chip_txid_batch call)."""
        if not txs:
            return []
        out = engine.txid_batch(TxBatch(txs))
        return [bytes(r) for r in np.asarray(out).reshape(len(txs), 32)]


# ---- notary uniqueness ----
@dataclass(frozen=True)
class StateRef:
    txhash: bytes
    index: int

    def key(self) -> bytes:
        return self.txhash + struct.pack("<I", self.index)


@dataclass(frozen=True)
class ConsumingTx:
    id: bytes
    input_index: int
    requesting_party: int


@dataclass
class Conflict:
    state_history: List[Tuple[StateRef, ConsumingTx]]


# notary_commit_log row (PersistentUniquenessProvider.kt:50-53): StateRef (32-B txhash + LE u32 index,
# the 36-B table key), consuming tx id, consuming input index, requesting party (interned id)
COMMIT_LOG_DTYPE = np.dtype([("ref", "u1", 36), ("tx", "u1", 32), ("idx", "<u4"), ("caller", "<u4")])


class CommitLog:
    """Append-only on-disk commit log of the notary (the role of the `notary_commit_log` table behind
    AppendOnlyPersistentMap, PersistentUniquenessProvider.kt:50-89): fixed 76-byte rows, appended in
    commit order after each batch; `load()` memory-maps the file for the table rebuild at open
    (AppendOnlyPersistentMap.allPersisted).  A torn final row (crash mid-append) is ignored.
    `append` returns only once the rows are durable (fsync, the role of the reference's database
    transaction commit); fsync=False trades that for speed in benchmarks and tests only."""

    def __init__(self, path: str, fsync: bool = True):
        self.path = path
        self.fsync = fsync
        self._f = open(path, "ab")

    def load(self) -> np.ndarray:
        import os
        n = os.path.getsize(self.path) // COMMIT_LOG_DTYPE.itemsize
        if n == 0:
            return np.zeros(0, dtype=COMMIT_LOG_DTYPE)
        return np.memmap(self.path, dtype=COMMIT_LOG_DTYPE, mode="r", shape=(n,))

    def append(self, rows: np.ndarray):
        if len(rows):
            import os
            self._f.seek(0, os.SEEK_END)
            size = self._f.tell()
            torn = size % COMMIT_LOG_DTYPE.itemsize
            if torn:                        # drop a torn row before appending whole ones
                self._f.truncate(size - torn)
            self._f.write(rows.tobytes())
            self._f.flush()
            if self.fsync:
                os.fsync(self._f.fileno())

    def close(self):
        if self._f:
            self._f.close()
            self._f = None


class PersistentUniquenessProvider:
    """UniquenessProvider backed by the GPU commit log (chip_uniq_*).  With `log_path`, committed rows
    are also appended to an on-disk CommitLog and the table is rebuilt from it at open, so a restarted
    notary rejects double spends of states committed before the restart."""

    def __init__(self, engine, capacity: int = 1 << 20, log_path: Optional[str] = None, fsync: bool = True):
        self.table = engine.uniq_open(capacity)
        self.log = None
        self._failed: Optional[BaseException] = None
        if log_path is not None:
            self.log = CommitLog(log_path, fsync)
            rows = self.log.load()
            if len(rows):
                self.table.rebuild(np.ascontiguousarray(rows["ref"]).reshape(-1),
                                   np.ascontiguousarray(rows["tx"]).reshape(-1),
                                   np.ascontiguousarray(rows["idx"]), np.ascontiguousarray(rows["caller"]))
            del rows

    def size(self) -> int:
        return self.table.size()

    def close(self):
        if self.log is not None:
            self.log.close()

    def _log_committed(self, requests, statuses):
        """Rows of the transactions this batch committed, in batch order; a StateRef repeated inside
        one transaction keeps its first index (AppendOnlyPersistentMap.set)."""
        rows = []
        for (states, tx_id, caller), st in zip(requests, statuses):
            if st != 0:
                continue
            seen = set()
            for i, sref in enumerate(states):
                k = sref.key()
                if k in seen:
                    continue
                seen.add(k)
                rows.append((np.frombuffer(k, np.uint8), np.frombuffer(tx_id, np.uint8), i, caller))
        self.log.append(np.array(rows, dtype=COMMIT_LOG_DTYPE))

    def commit_batch(self, requests: Sequence[Tuple[List[StateRef], bytes, int]]):
        """[(states, txId, callerIdentity)] applied in order -> [(status, Conflict)]; status 0 committed,
        1 re-notarisation of the same tx (commitInputStates accepts it), 2 conflict.  With a commit
        log, results are returned only after the committed rows are durable; if the append fails
        the provider fails stop (CommitLogFailure now and on every later call): the device table is
        then ahead of the log, and only a reopen — which rebuilds it from the log — may serve again.
        No result of the failed batch was reported, so its transactions were never acknowledged."""
        if self._failed is not None:
            raise CommitLogFailure("commit log append failed earlier; reopen the provider") from self._failed
        start = [0]
        refs, ids, callers = [], [], []
        for states, tx_id, caller in requests:
            refs += [s.key() for s in states]
            start.append(len(refs))
            ids.append(tx_id)
            callers.append(caller)
        st, recs = self.table.commit_batch(np.array(start, dtype=np.uint64),
                                           np.frombuffer(b"".join(refs) or bytes(36), dtype=np.uint8).copy(),
                                           np.frombuffer(b"".join(ids), dtype=np.uint8).copy(),
                                           np.array(callers, dtype=np.uint32))
        out = [(int(s), Conflict([])) for s in st]
        for tx, i, ci, cid, cc in recs:
            out[tx][1].state_history.append((requests[tx][0][i], ConsumingTx(cid, ci, cc)))
        if self.log is not None:
            try:
                self._log_committed(requests, [o[0] for o in out])
            except BaseException as e:
                self._failed = e
                raise CommitLogFailure("commit log append failed: %s" % e) from e
        return out

    def commit(self, states: List[StateRef], tx_id: bytes, caller_identity: int):
        """UniquenessProvider.commit: raises UniquenessException when an input is already consumed."""
        st, conflict = self.commit_batch([(states, tx_id, caller_identity)])[0]
        if st != 0:
            raise UniquenessException(conflict)


def commit_input_states(provider: PersistentUniquenessProvider, inputs: List[StateRef], tx_id: bytes,
                        caller: int):
    """TrustedAuthorityNotaryService.commitInputStates (NotaryService.kt:61-75)."""
    try:
        provider.commit(inputs, tx_id, caller)
    except UniquenessException as e:
        history = dict(e.error.state_history)
        conflicts = [ref for i, ref in enumerate(inputs)
                     if ref in history and history[ref] != ConsumingTx(tx_id, i, caller)]
        if conflicts:
            raise NotaryException(tx_id, e.error)
