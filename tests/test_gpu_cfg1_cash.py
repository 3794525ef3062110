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
