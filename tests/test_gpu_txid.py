"""GPU parity: WireTransaction.id recomputation (K3) vs the committed hashlib vectors and the oracle."""
import numpy as np
import pytest

import cordagen as G
import golden_cases
from corda_amd import native

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


def test_txid_fast_path_edges_match_oracle(ctx, oracle):
    """Both k_txid schedules against the oracle: the register / LDS tree path (groups ascending, <= 16
    components, ordinals < 16) at its limits — 1, 2, 15, 16 components per group, ordinal 15, every power-of-two
    boundary of the top tree — and the HBM-slab fallback just past them (17 components, ordinal 16, 20, 63,
    groups out of ordinal order)."""
    rng = np.random.Generator(np.random.PCG64(11))
    txs = []
    shapes = [[(0, 1)], [(0, 2)], [(3, 15)], [(1, 16)], [(15, 1)], [(0, 1), (1, 1)], [(0, 3), (2, 5), (7, 16)],
              [(0, 17)], [(16, 1)], [(20, 2)], [(63, 1)], [(2, 2), (0, 1)], [(0, 1), (4, 1), (8, 1), (9, 3)]]
    for shape in shapes * 6:
        groups = [(g, [rng.bytes(int(rng.integers(0, 200))) for _ in range(k)]) for g, k in shape]
        txs.append((rng.bytes(32), groups))
    for _ in range(300):
        gs = sorted(rng.choice(18, size=int(rng.integers(1, 9)), replace=False))
        groups = [(int(g), [rng.bytes(int(rng.integers(0, 120))) for _ in range(int(rng.integers(1, 19)))]) for g in gs]
        txs.append((rng.bytes(32), groups))
    tb = G.tx_batch_from_lists(txs)
    assert np.array_equal(ctx.txid_batch(tb), oracle.txid_batch(tb))


def _permute_txs(tb, p):
    """The same transactions in order p, their components still at their old pool offsets (so every chunk's byte
    range spans the pool)."""
    s = tb.tx_comp_start.astype(np.int64)
    idx = np.concatenate([np.arange(s[t], s[t + 1]) for t in p]).astype(np.int64)
    out = G.TxBatch()
    out.ntx = tb.ntx
    out.salts = tb.salts.reshape(-1, 32)[p].reshape(-1).copy()
    out.tx_comp_start = np.concatenate([[0], np.cumsum(s[1:][p] - s[:-1][p])]).astype(np.uint64)
    out.comp_group, out.comp_internal = tb.comp_group[idx].copy(), tb.comp_internal[idx].copy()
    out.comp_off, out.comp_len, out.data = tb.comp_off[idx].copy(), tb.comp_len[idx].copy(), tb.data
    return out


@pytest.mark.parametrize("permute", [False, True])
def test_txid_host_chunks_equal_one_chunk(ctx, oracle, monkeypatch, permute):
    """chip_txid_batch in transaction chunks (chunk j+1's arrays and bytes over PCIe beside chunk j's hashing):
    ids equal the one-chunk call and the oracle, also with the transactions in shuffled pool order; a component
    outside the pool or a start going backwards inside a later chunk is refused like the one-chunk call refuses it."""
    tb = G.tx_batch(2000, seed=33)
    if permute:
        tb = _permute_txs(tb, np.random.Generator(np.random.PCG64(3)).permutation(tb.ntx))
    ref = oracle.txid_batch(tb, threads=8)
    monkeypatch.setenv("CHIP_TXID_CHUNKS", "1")
    assert np.array_equal(ctx.txid_batch(tb), ref)
    for k in (2, 3, 7):
        monkeypatch.setenv("CHIP_TXID_CHUNKS", str(k))
        assert np.array_equal(ctx.txid_batch(tb), ref), k
    monkeypatch.setenv("CHIP_TXID_CHUNKS", "4")
    bad = _permute_txs(tb, np.arange(tb.ntx))
    bad.comp_off = bad.comp_off.copy()
    bad.comp_off[-3] = len(tb.data) - 2
    with pytest.raises(native.ChipError) as e:
        ctx.txid_batch(bad)
    assert "outside" in str(e.value)
    bad = _permute_txs(tb, np.arange(tb.ntx))
    bad.tx_comp_start = bad.tx_comp_start.copy()
    bad.tx_comp_start[1700] = bad.tx_comp_start[1698]
    bad.tx_comp_start[1699] = bad.tx_comp_start[1701]
    with pytest.raises(native.ChipError) as e:
        ctx.txid_batch(bad)
    assert "monotone" in str(e.value)
    assert np.array_equal(ctx.txid_batch(tb), ref)   # the context is still usable
