"""cfg1 (BASELINE.json configs[0]): 10k finance Cash issue/move SignedTransactions,
verifySignaturesExcept(notary) on the CPU reference path — the host mirror (corda_amd.crypto) over
the oracle engine: tx ids, SignableData messages, first-failing-signature exceptions and the
missing-signer logic, sequential per transaction == one batched call."""
import pytest

from cash_workload import cash_workload, outcome, sign_all
from corda_amd import crypto as C
from oracle_engine import OracleEngine


@pytest.fixture(scope="module")
def cfg1():
    eng = OracleEngine()
    w = cash_workload(10_000)
    stxs, labels = sign_all(eng, *w)
    return eng, w, stxs, labels


def test_cfg1_required_signers(cfg1):
    _, (seeds, keys, notary, wtxs, plans, *_), _, _ = cfg1
    for wtx, signers in zip(wtxs[:200], plans[:200]):
        req = wtx.required_signing_keys
        has_inputs = any(g == C.INPUTS_GROUP for g, _ in wtx.component_groups)
        assert req == {keys[s] for s in signers} | ({notary} if has_inputs else set())


def test_cfg1_batch_equals_sequential_and_labels(cfg1):
    eng, (seeds, keys, notary, *_), stxs, labels = cfg1
    batch = C.verify_signatures_except_batch(eng, stxs, [notary])
    seq = []
    for stx in stxs:
        try:
            stx.verify_signatures_except(eng, notary)
            seq.append(None)
        except Exception as e:   # noqa: BLE001
            seq.append(e)
    got_b = [outcome(e) for e in batch]
    got_s = [outcome(e) for e in seq]
    assert got_b == got_s
    assert got_b == labels
    assert sum(x is not None for x in labels) > 50


def test_cfg1_notary_signature_required_without_exception(cfg1):
    eng, (seeds, keys, notary, *_), stxs, labels = cfg1
    moves = [s for s, l in zip(stxs, labels) if l is None and notary in s.required_signing_keys][:20]
    for stx in moves:
        with pytest.raises(C.SignaturesMissingException) as ei:
            stx.verify_required_signatures(eng)
        assert ei.value.missing == {notary}


def test_crypto_do_verify_exceptions(cfg1):
    eng, (seeds, keys, *_), stxs, _ = cfg1
    stx = stxs[0]
    s = stx.sigs[0]
    msg = C.signable_data_bytes(stx.id, s.signature_metadata)
    assert C.Crypto.do_verify(eng, s.by, s.bytes, msg)
    assert C.Crypto.is_valid(eng, s.by, s.bytes, msg)
    bad = bytes([s.bytes[0] ^ 1]) + s.bytes[1:]
    assert not C.Crypto.is_valid(eng, s.by, bad, msg)
    with pytest.raises(C.SignatureException, match="Signature Verification failed!"):
        C.Crypto.do_verify(eng, s.by, bad, msg)
    with pytest.raises(C.SignatureException, match="signature length is wrong"):
        C.Crypto.is_valid(eng, s.by, s.bytes[:63], msg)
    with pytest.raises(C.IllegalArgumentException, match="Signature data is empty!"):
        C.Crypto.do_verify(eng, s.by, b"", msg)
    with pytest.raises(C.IllegalArgumentException, match="Clear data is empty"):
        C.Crypto.do_verify(eng, s.by, s.bytes, b"")
    with pytest.raises(C.IllegalArgumentException):
        C.SignedTransaction(stx.id, [], set())
    assert C.find_signature_scheme(s.by) == C.EDDSA_ED25519_SHA512


def test_uniqueness_mirror_commit_input_states():
    """PersistentUniquenessProviderTests / NotaryServiceTests shapes through the mirror."""
    import hashlib
    eng = OracleEngine()
    p = C.PersistentUniquenessProvider(eng, 64)
    h = lambda s: hashlib.sha256(s.encode()).digest()   # noqa: E731
    a, b = C.StateRef(h("a"), 0), C.StateRef(h("b"), 1)
    p.commit([a], h("tx1"), 7)
    with pytest.raises(C.UniquenessException) as ei:
        p.commit([a, b], h("tx2"), 8)
    assert ei.value.error.state_history == [(a, C.ConsumingTx(h("tx1"), 0, 7))]
    C.commit_input_states(p, [a], h("tx1"), 7)            # re-notarisation of the same tx: accepted
    with pytest.raises(C.NotaryException):
        C.commit_input_states(p, [a], h("tx3"), 7)
    p.commit([b], h("tx4"), 9)                            # tx2 failed, so b is still free
    assert p.size() == 2
