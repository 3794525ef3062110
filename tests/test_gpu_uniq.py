"""GPU parity: notary uniqueness (K4) vs the oracle restatement of PersistentUniquenessProvider.commit
+ TrustedAuthorityNotaryService.commitInputStates, and the reference's own scenarios."""
import hashlib

import numpy as np
import pytest

import cordagen as G
import golden_cases

pytestmark = pytest.mark.gpu

COMMITTED, IDEMPOTENT, CONFLICT = 0, 1, 2


def h(s):
    return hashlib.sha256(s.encode()).digest()


def run_both(ctx, oracle, pre, batches, cap=1 << 12):
    t = ctx.uniq_open(cap)
    o = oracle.Uniq(cap)
    if pre is not None:
        t.rebuild(*pre)
        o.preload(*pre)
    outs = []
    for b in batches:
        g = t.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
        r = o.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
        outs.append((g, r))
    assert t.size() == o.size()
    t.close()
    return outs


def test_uniq_golden_scenarios(ctx, oracle):
    for case in golden_cases.uniq_cases():
        batches = [G.uniq_batch_from_lists([(bytes.fromhex(tx), [bytes.fromhex(s) for s in ins], c)
                                            for tx, ins, c in bt]) for bt in case["batches"]]
        outs = run_both(ctx, oracle, None, batches)
        for (g, r), want in zip(outs, case["expected"]):
            assert g[0].tolist() == want, case["label"]
            assert g[0].tolist() == r[0].tolist(), case["label"]
            assert g[1] == r[1], case["label"]


def test_uniq_random_cfg5_shape_matches_oracle(ctx, oracle):
    pre, b = G.uniq_workload(20000, 30000, seed=7, pre_hit=0.02, dbl=0.02, resubmit=0.01)
    (g, r), = run_both(ctx, oracle, pre, [b], cap=1 << 16)
    assert np.array_equal(g[0], r[0])
    assert g[1] == r[1]
    assert (g[0] == CONFLICT).sum() > 0 and (g[0] == IDEMPOTENT).sum() > 0


def test_uniq_multi_batch_and_growth(ctx, oracle):
    batches = []
    pre, b0 = G.uniq_workload(5000, 1000, seed=1, pre_hit=0.05, dbl=0.05)
    batches.append(b0)
    for s in range(2, 5):   # later batches re-spend earlier batches' inputs
        _, bs = G.uniq_workload(5000, 0, seed=s, pre_hit=0.0, dbl=0.03)
        k = 2000
        bs.refs[:36 * k] = b0.refs[:36 * k]
        batches.append(bs)
    outs = run_both(ctx, oracle, pre, batches, cap=1024)   # forces rehash growth
    for g, r in outs:
        assert np.array_equal(g[0], r[0])
        assert g[1] == r[1]
