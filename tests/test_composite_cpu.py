"""CompositeKey fulfilment and encoding (corda_amd.composite), following the reference's
CompositeKeyTests.kt scenarios (:44-216, :363-) and its use in getMissingSigners
(TransactionWithSignatures.kt:79-85) and CompositeSignature (CompositeSignature.kt:77-86).  Leaf keys
are Ed25519 SPKIs of the reference's deterministic test entropies; signatures go through the oracle
engine (CPU)."""
import pytest

import cordagen as G
from corda_amd import crypto as C
from corda_amd.composite import (ArithmeticException, CompositeKey, IllegalArgumentException, NodeAndWeight,
                                 contains_any, decode_public_key, is_fulfilled_by, keys_of)
from cash_workload import entropy_seed
from oracle_engine import OracleEngine

SEEDS = [entropy_seed(v) for v in (20, 30, 40, 50)]
ALICE, BOB, CHARLIE, DAVE = [G.spki_ed25519(G.ed25519_pub(s)) for s in SEEDS]


def B():
    return CompositeKey.Builder()


def test_single_key_fulfilled_by_itself():
    assert is_fulfilled_by(ALICE, ALICE)
    assert not is_fulfilled_by(ALICE, CHARLIE)


def test_alice_or_bob():
    k = B().add_keys(ALICE, BOB).build(threshold=1)
    assert k.is_fulfilled_by(ALICE) and k.is_fulfilled_by(BOB)
    assert k.is_fulfilled_by([ALICE, BOB])
    assert not k.is_fulfilled_by(CHARLIE)


def test_alice_and_bob_requires_both():
    k = B().add_keys(ALICE, BOB).build()
    assert k.threshold == 2
    assert not k.is_fulfilled_by([ALICE]) and not k.is_fulfilled_by([BOB])
    assert k.is_fulfilled_by([ALICE, BOB])


def test_nested_alice_and_bob_or_charlie():
    ab = B().add_keys(ALICE, BOB).build()
    k = B().add_keys(ab, CHARLIE).build(threshold=1)
    assert k.is_fulfilled_by([ALICE, BOB])
    assert k.is_fulfilled_by([CHARLIE])
    assert not k.is_fulfilled_by([ALICE])
    assert keys_of(k) == {ALICE, BOB, CHARLIE}
    assert contains_any(k, [BOB]) and not contains_any(k, [DAVE])
    # a composite key among the keys to check never fulfils (CompositeKey.kt:176)
    assert not k.is_fulfilled_by([CHARLIE, ab])


def test_der_round_trip_plain_and_weighted():
    ab = B().add_keys(ALICE, BOB).build()
    k = B().add_keys(ab, CHARLIE).build(threshold=1)
    assert CompositeKey.get_instance(k.encoded) == k
    assert decode_public_key(k.encoded) == k
    ab2 = B().add_key(ALICE, 2).add_key(BOB, 1).build(threshold=2)
    k2 = B().add_key(ab2, 3).add_key(CHARLIE, 2).build(threshold=3)
    d = CompositeKey.get_instance(k2.encoded)
    assert d == k2 and d.encoded == k2.encoded
    # SPKI shape: SEQUENCE { SEQUENCE { OID 2.25.30086077608615255153862931087626791002 }, BIT STRING }
    enc = k2.encoded
    i = enc.index(b"\x06", 2)
    oid = enc[i + 2:i + 2 + enc[i + 1]]
    arcs, v = [], 0
    for byte in oid:
        v = (v << 7) | (byte & 0x7F)
        if not byte & 0x80:
            arcs.append(v)
            v = 0
    assert [arcs[0] // 40, arcs[0] % 40] + arcs[1:] == [2, 25, 30086077608615255153862931087626791002]


def test_tree_canonical_form():
    assert B().add_keys(ALICE).build() == ALICE
    n1 = B().add_keys(ALICE, BOB).build(1)
    n2 = B().add_keys(ALICE, BOB).build(2)
    assert not n2.is_fulfilled_by(ALICE)
    t1 = B().add_key(n1, 13).add_key(n2, 27).build()
    t2 = B().add_key(n2, 27).add_key(n1, 13).build()
    assert t1 == t2 and hash(t1) == hash(t2) and t1.encoded == t2.encoded
    t3 = B().add_keys(n1, n2).build()
    t4 = B().add_keys(n2, n1).build()
    assert t3 == t4 and hash(t3) == hash(t4) and t3.encoded == t4.encoded
    t5 = B().add_key(n1, 3).add_key(n1, 14).build()
    t6 = B().add_key(n1, 14).add_key(n1, 3).build()
    assert t5 == t6
    assert B().add_keys(t1).build() == t1


def test_constraints():
    with pytest.raises(IllegalArgumentException):
        B().add_key(ALICE, 0)
    with pytest.raises(IllegalArgumentException):
        B().add_key(ALICE, -1)
    with pytest.raises(IllegalArgumentException):
        B().add_key(ALICE).build(0)
    with pytest.raises(IllegalArgumentException):
        B().add_key(ALICE).build(-1)
    with pytest.raises(IllegalArgumentException):
        B().add_key(ALICE, 2).add_key(BOB, 2).build(5)
    with pytest.raises(IllegalArgumentException):
        B().add_key(ALICE, 3).build(2)
    with pytest.raises(IllegalArgumentException):      # Int sum wraps negative -> threshold check
        B().add_key(ALICE, 2**31 - 1).add_key(BOB, 2**31 - 1).build()
    with pytest.raises(ArithmeticException):           # explicit threshold: addExact overflow
        B().add_key(ALICE, 2**31 - 1).add_key(BOB, 2**31 - 1).build(5)
    with pytest.raises(IllegalArgumentException):
        B().add_keys(ALICE, BOB, ALICE).build()
    with pytest.raises(IllegalArgumentException):
        B().add_keys(B().add_keys(ALICE, BOB).build(), B().add_keys(BOB, ALICE).build()).build()


def test_cycle_detection():
    k1 = B().add_keys(ALICE, BOB).build()
    k2 = B().add_keys(ALICE, k1).build()
    k3 = B().add_keys(ALICE, k2).build()
    k4 = B().add_keys(ALICE, k3).build()
    k5 = B().add_keys(ALICE, k4).build()
    k6 = B().add_keys(ALICE, k5, k2).build()
    for k in (k1, k2, k3, k4, k5, k6):
        k.check_validity()
    k3.children.append(NodeAndWeight(k5, 1))   # inject a cycle, as the reference does by reflection
    with pytest.raises(IllegalArgumentException):
        k5.check_validity()


def test_deterministic_children_sorting():
    keys = [G.spki_ed25519(G.ed25519_pub(entropy_seed(v))) for v in range(200, 210)]
    a = B().add_keys(*keys).build(3)
    b = B().add_keys(*reversed(keys)).build(3)
    assert [n for n, _ in a.children] == sorted(keys)
    assert a.encoded == b.encoded


@pytest.fixture(scope="module")
def eng():
    return OracleEngine()


def _sig(seed_i, key, tx_id, meta=C.SignatureMetadata(1, 4)):
    return C.TransactionSignature(G.ed25519_sign(SEEDS[seed_i], C.signable_data_bytes(tx_id, meta)), key, meta)


def test_signed_transaction_with_composite_required_key(eng):
    tx_id = bytes(range(32))
    two_of_three = B().add_keys(ALICE, BOB, CHARLIE).build(threshold=2)
    a, b, c = _sig(0, ALICE, tx_id), _sig(1, BOB, tx_id), _sig(2, CHARLIE, tx_id)
    for sigs, ok in (([a], False), ([b], False), ([a, b], True), ([a, c], True), ([b, c], True), ([a, b, c], True)):
        stx = C.SignedTransaction(tx_id, sigs, [two_of_three, DAVE])
        missing = stx.get_missing_signers()
        assert (two_of_three not in missing) == ok
        assert DAVE in missing
        stx.verify_signatures_except(eng, DAVE) if ok else None
        if not ok:
            with pytest.raises(C.SignaturesMissingException) as ei:
                stx.verify_signatures_except(eng, DAVE)
            assert set(ei.value.missing) == {two_of_three}
    # the batch entry point agrees with the sequential one
    stxs = [C.SignedTransaction(tx_id, s, [two_of_three]) for s in ([a], [a, b], [c], [b, c])]
    res = C.verify_signatures_except_batch(eng, stxs)
    assert [r is None for r in res] == [False, True, False, True]


def test_composite_signature_engine_verify(eng):
    """CompositeKeyTests.kt:156-174: the engine is fed the 32 id bytes (engine.update(SHA256(message)
    .bytes)); CompositeSignature wraps them as the tx id without hashing (SecureHash.SHA256(bytes),
    CompositeSignature.kt:81, SecureHash.kt:16-19)."""
    import hashlib
    tx_id = hashlib.sha256(b"composite clear data").digest()
    two_of_three = B().add_keys(ALICE, BOB, CHARLIE).build(threshold=2)
    a, b, c = _sig(0, ALICE, tx_id), _sig(1, BOB, tx_id), _sig(2, CHARLIE, tx_id)
    v = lambda sigs, clear=tx_id: C.composite_signature_verify(eng, two_of_three, sigs, clear)   # noqa: E731
    assert not v([a]) and not v([b]) and not v([c])
    assert v([a, b]) and v([a, c]) and v([b, c]) and v([a, b, c])
    broken_bob = C.TransactionSignature(a.bytes, BOB, C.SignatureMetadata(1, 4))
    assert not v([a, broken_bob])
    # composite given as its encoded SPKI bytes
    assert C.composite_signature_verify(eng, two_of_three.encoded, [a, c], tx_id)
    # the buffer is the id, not a message to hash: SHA256(id) as clear data fails every signature
    assert not v([a, b], hashlib.sha256(tx_id).digest())
    # not 32 bytes: SecureHash.SHA256's require(size == 32) -> IllegalArgumentException, but only
    # once the key is fulfilled (engineVerify checks fulfilment first)
    with pytest.raises(C.IllegalArgumentException):
        v([a, b], b"composite clear data")
    assert not v([a], b"composite clear data")


def test_is_valid_has_no_empty_checks(eng):
    """Crypto.isValid (Crypto.kt:615-625) has no empty-input checks, unlike doVerify (:528-529): an
    empty Ed25519 signature is the engine's SignatureException("signature length is wrong"), empty
    clear data is verified as the empty message."""
    import cordagen as G
    seed = SEEDS[0]
    sig_empty_msg = G.ed25519_sign(seed, b"")
    assert C.Crypto.is_valid(eng, ALICE, sig_empty_msg, b"")
    assert not C.Crypto.is_valid(eng, ALICE, sig_empty_msg, b"x")
    with pytest.raises(C.IllegalArgumentException):
        C.Crypto.do_verify(eng, ALICE, sig_empty_msg, b"")
    with pytest.raises(C.SignatureException, match="signature length is wrong"):
        C.Crypto.is_valid(eng, ALICE, b"", b"x")
    with pytest.raises(C.IllegalArgumentException):
        C.Crypto.do_verify(eng, ALICE, b"", b"x")
