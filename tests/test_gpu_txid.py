"""GPU parity: WireTransaction.id recomputation (K3) vs the committed hashlib vectors and the oracle."""
import numpy as np
import pytest

import cordagen as G
import golden_cases

pytestmark = pytest.mark.gpu


def test_txid_golden(ctx):
    tb, ids = golden_cases.tx_batch_from_cases(golden_cases.txid_cases())
    got = ctx.txid_batch(tb)
    for i, want in enumerate(ids):
        assert got[i].tobytes() == want, golden_cases.txid_cases()[i]["label"]


def test_txid_cfg4_shape_matches_oracle(ctx, oracle):
    tb = G.tx_batch(3000, seed=21)
    got = ctx.txid_batch(tb)
    ref = oracle.txid_batch(tb, threads=8)
    assert np.array_equal(got, ref)
    # ids are distinct (salts differ) and never all-zero
    assert len({r.tobytes() for r in got}) == len(got)


def test_txid_mixed_shapes_matches_oracle(ctx, oracle):
    rng = np.random.Generator(np.random.PCG64(5))
    txs = []
    for t in range(500):
        groups = []
        for g in sorted(rng.choice(8, size=int(rng.integers(1, 7)), replace=False)):
            comps = [rng.bytes(int(rng.integers(0, 300))) for _ in range(int(rng.integers(1, 6)))]
            groups.append((int(g), comps))
        txs.append((rng.bytes(32), groups))
    tb = G.tx_batch_from_lists(txs)
    assert np.array_equal(ctx.txid_batch(tb), oracle.txid_batch(tb))
