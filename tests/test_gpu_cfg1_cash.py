"""GPU: the cfg1 Cash workload through the host mirror (corda_amd.crypto) on the HIP engine —
tx ids, batched verifySignaturesExcept(notary) and the notary mirror — equals the oracle engine."""
import hashlib

import pytest

from cash_workload import cash_workload, outcome, sign_all
from corda_amd import crypto as C
from oracle_engine import OracleEngine

pytestmark = pytest.mark.gpu


def test_cfg1_on_gpu_matches_oracle_engine(ctx):
    w = cash_workload(10_000)
    stxs_o, labels = sign_all(OracleEngine(), *w)
    wtxs = w[3]
    assert C.WireTransaction.ids(ctx, wtxs) == [s.id for s in stxs_o]
    notary = w[2]
    got = [outcome(e) for e in C.verify_signatures_except_batch(ctx, stxs_o, [notary])]
    assert got == labels
    # single-call API on a few transactions (each one engine call)
    for stx, lab in list(zip(stxs_o, labels))[:30]:
        try:
            stx.verify_signatures_except(ctx, notary)
            res = None
        except Exception as e:   # noqa: BLE001
            res = outcome(e)
        assert res == lab


def test_uniqueness_mirror_on_gpu(ctx):
    p = C.PersistentUniquenessProvider(ctx, 64)
    h = lambda s: hashlib.sha256(s.encode()).digest()   # noqa: E731
    a, b = C.StateRef(h("a"), 0), C.StateRef(h("b"), 1)
    p.commit([a], h("tx1"), 7)
    with pytest.raises(C.UniquenessException) as ei:
        p.commit([a, b], h("tx2"), 8)
    assert ei.value.error.state_history == [(a, C.ConsumingTx(h("tx1"), 0, 7))]
    C.commit_input_states(p, [a], h("tx1"), 7)
    with pytest.raises(C.NotaryException):
        C.commit_input_states(p, [a], h("tx3"), 7)
    p.commit([b], h("tx4"), 9)
    assert p.size() == 2


def test_composite_keys_on_gpu(ctx):
    """CompositeKey requirements (corda_amd.composite) with the signatures verified by the HIP engine:
    2-of-3 over Ed25519 leaves, getMissingSigners and CompositeSignature verify; same answers as the
    oracle engine."""
    import cordagen as G
    from cash_workload import entropy_seed
    from corda_amd.composite import CompositeKey
    seeds = [entropy_seed(v) for v in (20, 30, 40)]
    keys = [G.spki_ed25519(G.ed25519_pub(s)) for s in seeds]
    k = CompositeKey.Builder().add_keys(*keys).build(threshold=2)
    clear = b"composite on gpu"
    tx_id = hashlib.sha256(clear).digest()
    meta = C.SignatureMetadata(1, 4)
    sigs = [C.TransactionSignature(G.ed25519_sign(s, C.signable_data_bytes(tx_id, meta)), key, meta)
            for s, key in zip(seeds, keys)]
    broken = C.TransactionSignature(sigs[0].bytes, keys[1], meta)
    cases = [[sigs[0]], [sigs[0], sigs[1]], [sigs[1], sigs[2]], [sigs[0], broken], sigs]
    oracle = OracleEngine()
    for cs in cases:
        assert (C.composite_signature_verify(ctx, k, cs, tx_id)
                == C.composite_signature_verify(oracle, k, cs, tx_id))
    assert C.composite_signature_verify(ctx, k, sigs, tx_id)
    # Crypto.isValid semantics on the device: empty clear data is an ordinary message
    s0 = G.ed25519_sign(seeds[0], b"")
    assert C.Crypto.is_valid(ctx, keys[0], s0, b"") and not C.Crypto.is_valid(ctx, keys[0], s0, b"\x00")
    with pytest.raises(C.SignatureException):
        C.Crypto.is_valid(ctx, keys[0], b"", b"\x00")
    stxs = [C.SignedTransaction(tx_id, cs, [k]) for cs in cases]
    got = [outcome(e) for e in C.verify_signatures_except_batch(ctx, stxs)]
    ref = [outcome(e) for e in C.verify_signatures_except_batch(oracle, stxs)]
    assert got == ref
    assert [g is None for g in got] == [False, True, True, False, True]
