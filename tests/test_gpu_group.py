"""GPU: device groups (chip_group_*, corda_amd/csrc/group.hip) — one process driving several member contexts, as a
Corda node's single JVM drives the GPUs of its host.  On the one-GPU box the device list is [0, 0] (and [0, 0, 0]):
two / three contexts on the same GPU, each on its own host thread and streams, which is the same code path as
[0, 1, ...] on a multi-GPU node.  Every split entry must give the oracle's result and the single-context result:
statuses, bitmaps (member ranges that do not start on a 64-signature word), ids, verdicts, first-failing-signature
args (which index the WHOLE batch's signature list), missing flags, FilteredTransaction reasons, and the uniqueness
statuses, conflict records and table size of a cfg5-shaped notary batch over key-space shards."""
import os

import numpy as np
import pytest

import cordagen as G
import oracle_bind as O
from corda_amd import native

pytestmark = pytest.mark.gpu


def _group(devices):
    os.environ["CHIP_GROUP_MIN_SHARE"] = "1"   # split even test-sized batches over every member
    try:
        return native.Group(devices)
    finally:
        del os.environ["CHIP_GROUP_MIN_SHARE"]


@pytest.fixture(scope="module")
def group2():
    g = _group([0, 0])
    yield g
    g.close()


@pytest.fixture(scope="module")
def group3():
    g = _group([0, 0, 0])
    yield g
    g.close()


def concat_sig_batches(a, b):
    """One chip_sig_batch holding a's signatures then b's (pools appended, b's indices shifted)."""
    c = G.SigBatch()
    c.key_idx = np.concatenate([a.key_idx, b.key_idx + len(a.key_off)]).astype(np.uint32)
    c.msg_idx = np.concatenate([a.msg_idx, b.msg_idx + len(a.msg_off)]).astype(np.uint32)
    c.sig_data = np.concatenate([a.sig_data, b.sig_data])
    c.sig_off = np.concatenate([a.sig_off, b.sig_off + np.uint64(len(a.sig_data))]).astype(np.uint64)
    c.sig_len = np.concatenate([a.sig_len, b.sig_len]).astype(np.uint32)
    c.key_data = np.concatenate([a.key_data, b.key_data])
    c.key_off = np.concatenate([a.key_off, b.key_off + np.uint64(len(a.key_data))]).astype(np.uint64)
    c.key_len = np.concatenate([a.key_len, b.key_len]).astype(np.uint32)
    c.msg_data = np.concatenate([a.msg_data, b.msg_data])
    c.msg_off = np.concatenate([a.msg_off, b.msg_off + np.uint64(len(a.msg_data))]).astype(np.uint64)
    c.msg_len = np.concatenate([a.msg_len, b.msg_len]).astype(np.uint32)
    c.expected = np.concatenate([a.expected, b.expected])
    return c


@pytest.mark.parametrize("members", [2, 3])
def test_group_ed25519_and_mixed_ecdsa(group2, group3, ctx, oracle, members):
    g = group2 if members == 2 else group3
    b = concat_sig_batches(G.ed25519_batch(6002, n_keys=32, corrupt=0.25, seed=101),
                           G.ecdsa_batch(4000, n_keys=32, corrupt=0.3, seed=102))
    cut = native.plan_sigs(b.msg_idx, members, 1)
    assert np.all(np.diff(cut.astype(np.int64)) > 0) and any(int(c) % 64 for c in cut[1:-1])
    st, bm = g.verify_batch(b)
    ref = oracle.verify_batch(b, threads=8)
    bad = np.nonzero(st != ref)[0]
    assert len(bad) == 0, [(int(i), int(st[i]), int(ref[i])) for i in bad[:20]]
    assert np.array_equal(st, b.expected)
    st1, bm1 = ctx.verify_batch(b)
    assert np.array_equal(st, st1) and np.array_equal(bm, bm1)
    sv, bv = g.verify_batch(b, is_valid=True)                      # Crypto.isValid semantics, split the same way
    sv1, bv1 = ctx.verify_batch(b, is_valid=True)
    assert np.array_equal(sv, sv1) and np.array_equal(bv, bv1)


def test_group_tx_ids_and_empty_members(group3, oracle):
    tb = G.tx_batch(5000, seed=31)
    assert np.array_equal(group3.txid_batch(tb), oracle.txid_batch(tb, threads=8))
    tiny = G.tx_batch(2, seed=32)                                   # 2 transactions, 3 members: one empty
    assert np.array_equal(group3.txid_batch(tiny), oracle.txid_batch(tiny, threads=8))


def test_group_fused_verify_signatures_except(group2, ctx):
    """cfg4 shape (ids -> SignableData -> signatures -> required signers) over two members: ids, statuses, verdicts,
    args (global signature indices) and missing flags equal the single context's, and the labels."""
    ntx = 6000
    tb, tm, sb, ids, msgs = G.cfg4_workload(ntx, n_keys=64, corrupt=0.02, seed=0x5EED0901, threads=8)
    q = G.cfg4_required(sb, ntx, 64, seed=0x5EED0902)
    got = group2.verify_signed_tx_batch(tb, tm, sb, q)
    want = ctx.verify_signed_tx_batch(tb, tm, sb, q)
    for a, w in zip(got, want):
        assert np.array_equal(a, w)
    assert np.array_equal(got[0], ids)
    assert np.array_equal(got[2], q.expected_verdict) and np.array_equal(got[3], q.expected_arg)
    assert int((got[2] == native.TXV_SIGNATURE).sum()) > 10 and int(got[3][ntx // 2:].max()) > ntx
    # a signature naming a transaction outside its range: the whole batch goes to one member (one-context result)
    sb.tx_idx = sb.tx_idx.copy()
    sb.tx_idx[7] = ntx - 1
    got = group2.verify_signed_tx_batch(tb, tm, sb, q)
    want = ctx.verify_signed_tx_batch(tb, tm, sb, q)
    for a, w in zip(got, want):
        assert np.array_equal(a, w)
    assert got[2][3] == native.TXV_MALFORMED


def test_group_from_bytes(group2, ctx):
    """SignedTransaction bytes (parse, requiredSigningKeys, ids, signatures) over two members: statuses, verdicts,
    args and ids equal the single context's and the labels; a damaged blob in the second member's range."""
    ntx = 5000
    tb, tm, sb, ids_ref, verdict, arg = G.cfg4_workload_commands(ntx, n_keys=32, corrupt=0.02, seed=0x5EED0904,
                                                                 threads=8)
    data, off, ln = G.stx_uniform(tb, sb, 2)
    st, v, a, ids = group2.stx_verify(data, off, ln, tm, [[1, 4]], want_ids=True)
    assert not st.any()
    assert np.array_equal(ids, ids_ref) and np.array_equal(v, verdict) and np.array_equal(a, arg)
    assert int((v == native.TXV_SIGNATURE).sum()) > 10
    ln2 = ln.copy()
    ln2[ntx - 10] = 100                                             # truncated: KryoException
    st, v, a, ids = group2.stx_verify(data, off, ln2, tm, [[1, 4]], want_ids=True)
    st1, v1, a1, ids1 = ctx.stx_verify(data, off, ln2, tm, [[1, 4]], want_ids=True)
    assert st[ntx - 10] == 1 and np.array_equal(st, st1)
    ok = st == 0
    assert np.array_equal(v[ok], v1[ok]) and np.array_equal(a[ok], a1[ok]) and np.array_equal(ids[ok], ids1[ok])


def test_group_filtered_transactions(group2, ctx):
    from ftx_build import FtxBatch, notary_workload
    ftxs, want = notary_workload(4000, seed=0x5EED0017, flow=True)
    b = FtxBatch(ftxs)
    st, rs = group2.ftx_verify_batch(b)
    ost, ors = O.ftx_verify_batch(b)
    assert np.array_equal(st, ost) and np.array_equal(rs, ors)
    assert list(zip(st.tolist(), rs.tolist())) == want


@pytest.mark.parametrize("members", [2, 3])
def test_group_notary_commit(group2, group3, ctx, oracle, members):
    """cfg5 shape over key-space shards: pre-committed rows rebuilt into their owners, two batches (the second
    re-spends the first's inputs): statuses, Conflict.stateHistory records in (tx, input_index) order and the
    table size equal the single-table oracle; every member holds only states it owns."""
    g = group2 if members == 2 else group3
    pre, b = G.uniq_workload(20000, 30000, seed=41, pre_hit=0.02, dbl=0.03, resubmit=0.01)
    _, b2 = G.uniq_workload(8000, 0, seed=42, pre_hit=0.0, dbl=0.03)
    b2.refs[:36 * 4000] = b.refs[:36 * 4000]
    t = g.uniq_open(1 << 16)
    o = oracle.Uniq(1 << 16)
    one = ctx.uniq_open(1 << 16)                                  # the single context: same rounds
    t.rebuild(*pre)
    o.preload(*pre)
    one.rebuild(*pre)
    assert t.size() == o.size()
    for batch in (b, b2):
        st, recs = t.commit_batch(batch.tx_ref_start, batch.refs, batch.tx_ids, batch.callers)
        ws, wr = o.commit_batch(batch.tx_ref_start, batch.refs, batch.tx_ids, batch.callers)
        assert np.array_equal(st, ws)
        assert recs == wr
        assert (st == 2).sum() > 0 and (st == 1).sum() > 0
        s = t.last_stats()
        one.commit_batch(batch.tx_ref_start, batch.refs, batch.tx_ids, batch.callers)
        assert s["rounds"] == one.last_rounds() >= 2
        # each member staged only its slice of the batch from the host (ABI 10)
        whole = 8 * (len(batch.tx_ref_start)) + len(batch.refs) + 36 * (len(batch.tx_ref_start) - 1)
        assert s["members_used"] == members
        assert abs(s["h2d_bytes_total"] - whole) <= 8 * members
        assert s["h2d_bytes_max"] < whole / members * 1.25
    assert t.size() == o.size()
    one.close()
    # capacity: the full count comes back with CHIP_E_CAPACITY
    _, b3 = G.uniq_workload(3000, 0, seed=43, pre_hit=0.0, dbl=0.0)
    b3.refs[:] = b.refs[:len(b3.refs)]
    with pytest.raises(native.ChipError) as e:
        t.commit_batch(b3.tx_ref_start, b3.refs, b3.tx_ids, b3.callers, cap=1)
    assert e.value.code == -4
    t.close()


def test_group_of_one_is_the_single_context(ctx, oracle):
    """A group of one member: the notary commit is the single-context host entry (statuses, records, rounds), and a
    verify batch runs whole on the member (members_used 1)."""
    g = native.Group([0])
    try:
        pre, b = G.uniq_workload(20000, 30000, seed=44, pre_hit=0.02, dbl=0.03, resubmit=0.01)
        t, o, one = g.uniq_open(1 << 16), oracle.Uniq(1 << 16), ctx.uniq_open(1 << 16)
        t.rebuild(*pre)
        o.preload(*pre)
        one.rebuild(*pre)
        st, raw, n = t.commit_batch_raw(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
        st1, raw1, n1 = one.commit_batch_raw(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
        ws, wr = o.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
        assert np.array_equal(st, ws) and np.array_equal(st, st1)
        assert n == n1 == len(wr) and np.array_equal(raw, raw1)
        s = t.last_stats()
        assert s["members_used"] == 1 and s["rounds"] == one.last_rounds() >= 2
        t.close()
        one.close()
        vb = G.ed25519_batch(20000, n_keys=32, corrupt=0.2, seed=103)
        st, bm = g.verify_batch(vb)
        assert np.array_equal(st, vb.expected)
        assert g.last_stats()["members_used"] == 1
    finally:
        g.close()


def test_group_concurrent_verify_and_commit(group2, oracle):
    """Two host threads on one group, one verifying signature batches and one committing notary batches: the group
    serialises the calls (one member-thread pool), so every result equals the oracle's."""
    import threading
    pre, b = G.uniq_workload(6000, 8000, seed=45, pre_hit=0.02, dbl=0.03, resubmit=0.01)
    vb = G.ed25519_batch(6000, n_keys=16, corrupt=0.2, seed=104)
    t = group2.uniq_open(1 << 15)
    t.rebuild(*pre)
    errors = []

    def verify():
        try:
            for _ in range(6):
                st, _bm = group2.verify_batch(vb)
                if not np.array_equal(st, vb.expected):
                    errors.append("verify statuses")
        except Exception as e:   # noqa: BLE001
            errors.append(repr(e))

    results = []

    def commit():
        try:
            for _ in range(3):
                results.append(t.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers))
        except Exception as e:   # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=verify), threading.Thread(target=commit)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not errors, errors
    o = oracle.Uniq(1 << 15)
    o.preload(*pre)
    for st, recs in results:                  # the same batch three times: commit, then re-submissions
        ws, wr = o.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
        assert np.array_equal(st, ws) and recs == wr
    t.close()
