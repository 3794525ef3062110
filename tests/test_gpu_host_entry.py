"""GPU: chip_verify_batch's argument checks (now on the device, before any verify kernel) and its status
counters.  An out-of-range key / message index or an (offset, length) outside its pool is CHIP_E_ARG and
nothing is verified; a valid call afterwards is unaffected and chip_stats counts its statuses."""
import copy

import numpy as np
import pytest

import cordagen as G
from corda_amd import native

pytestmark = pytest.mark.gpu


def test_bad_arguments_rejected_then_valid_call(ctx):
    b = G.ed25519_batch(512, n_keys=8, corrupt=0.25, seed=77)
    cases = []
    x = copy.copy(b)
    x.key_idx = b.key_idx.copy()
    x.key_idx[3] = len(b.key_off) + 5
    cases.append((x, "key_idx"))
    x = copy.copy(b)
    x.msg_idx = b.msg_idx.copy()
    x.msg_idx[-1] = len(b.msg_off)
    cases.append((x, "msg_idx"))
    x = copy.copy(b)
    x.sig_off = b.sig_off.copy()
    x.sig_off[100] = len(b.sig_data) - 10
    cases.append((x, "sig pool"))
    x = copy.copy(b)
    x.key_len = b.key_len.copy()
    x.key_len[0] = 10 ** 6
    cases.append((x, "key pool"))
    x = copy.copy(b)
    x.msg_off = b.msg_off.copy()
    x.msg_off[0] = 2 ** 64 - 4                       # offset + length wraps around
    cases.append((x, "msg pool"))
    for bad, what in cases:
        with pytest.raises(native.ChipError) as e:
            ctx.verify_batch(bad)
        assert "range" in str(e.value) or "outside" in str(e.value), what
    ctx.reset_stats()
    st, _bm = ctx.verify_batch(b)
    assert np.array_equal(st, b.expected)
    s = ctx.stats()
    assert [int(s.status_count[k]) for k in range(8)] == list(np.bincount(st, minlength=8))


def _permuted(b, seed):
    """The same signatures in a shuffled order: sig offsets and message indices no longer ascend, so
    every chunk's pool ranges overlap the others' (the copied intervals grow on both sides)."""
    p = np.random.Generator(np.random.PCG64(seed)).permutation(len(b.key_idx))
    x = copy.copy(b)
    for f in ("key_idx", "msg_idx", "sig_off", "sig_len", "expected"):
        setattr(x, f, np.ascontiguousarray(getattr(b, f)[p]))
    return x


def _chunked(ctx, b, chunks, monkeypatch):
    monkeypatch.setenv("CHIP_HOST_CHUNKS", str(chunks))
    return ctx.verify_batch(b)


@pytest.mark.parametrize("permute", [False, True])
def test_host_chunk_pipeline_equals_one_chunk(ctx, monkeypatch, permute):
    """chip_verify_batch in chunks (H2D of chunk j+1 beside the kernels of chunk j; key tables built by
    the first chunk and reused): statuses and bitmap equal the one-chunk call and the labels, on a batch
    that takes the eager per-key comb tables (80k signatures over 64 keys)."""
    b = G.ed25519_batch(80000, n_keys=64, corrupt=0.1, seed=0x5EED0501)
    if permute:
        b = _permuted(b, 5)
    st1, bm1 = _chunked(ctx, b, 1, monkeypatch)
    assert np.array_equal(st1, b.expected)
    for k in (3, 7):
        st, bm = _chunked(ctx, b, k, monkeypatch)
        assert np.array_equal(st, st1), k
        assert np.array_equal(bm, bm1), k


def test_host_chunk_pipeline_ecdsa_tables_reused(ctx, monkeypatch):
    """ECDSA (P-256 + secp256k1) in 4 chunks: the per-key comb tables of the first chunk serve the rest."""
    b = G.ecdsa_batch(72000, n_keys=32, corrupt=0.1, seed=0x5EED0502)
    st1, bm1 = _chunked(ctx, b, 1, monkeypatch)
    assert np.array_equal(st1, b.expected)
    st, bm = _chunked(ctx, b, 4, monkeypatch)
    assert np.array_equal(st, st1)
    assert np.array_equal(bm, bm1)


def test_host_chunk_pipeline_rejects_bad_index_in_a_later_chunk(ctx, monkeypatch):
    """A bad index in the last chunk is found by that chunk's device check: CHIP_E_ARG, and the next
    call is unaffected."""
    b = G.ed25519_batch(20000, n_keys=16, corrupt=0.1, seed=0x5EED0503)
    x = copy.copy(b)
    x.msg_idx = b.msg_idx.copy()
    x.msg_idx[-3] = len(b.msg_off) + 1
    with pytest.raises(native.ChipError) as e:
        _chunked(ctx, x, 5, monkeypatch)
    assert "range" in str(e.value)
    st, _ = _chunked(ctx, b, 5, monkeypatch)
    assert np.array_equal(st, b.expected)


@pytest.mark.parametrize("field", ["key_off", "key_len"])
def test_host_chunk_pipeline_rejects_key_outside_pool_before_key_prep(ctx, monkeypatch, field):
    """In the chunked host entry the key prep and the table chains start on the keys alone: a key range
    outside the key pool is CHIP_E_ARG before any kernel reads through it (no device fault), and the next
    call is unaffected."""
    b = G.ed25519_batch(20000, n_keys=16, corrupt=0.1, seed=0x5EED0504)
    x = copy.copy(b)
    arr = getattr(b, field).copy()
    if field == "key_off":
        arr[5] = len(b.key_data) + (1 << 30)
    else:
        arr[5] = 1 << 31
    setattr(x, field, arr)
    with pytest.raises(native.ChipError) as e:
        _chunked(ctx, x, 4, monkeypatch)
    assert "key pool" in str(e.value)
    st, _ = _chunked(ctx, b, 4, monkeypatch)
    assert np.array_equal(st, b.expected)


def test_other_host_entries_check_arguments_on_the_device(ctx):
    """The tx-id, fused, FilteredTransaction, chip_stx_verify and uniqueness host entries check their
    arrays on the device after staging (no host walk): each bad argument is CHIP_E_ARG with its message,
    and the same call with good arguments afterwards is correct."""
    import sys
    sys.path.insert(0, __import__("os").path.dirname(__file__))
    from ftx_build import FtxBatch, notary_workload

    def bad(fn, *a, want):
        with pytest.raises(native.ChipError) as e:
            fn(*a)
        assert want in str(e.value), (want, str(e.value))

    tb, tm, sb, ids, _msgs = G.cfg4_workload(300, n_keys=8, corrupt=0.05, seed=0x5EED0504, threads=8)
    # tx ids: a non-monotone start array, a component outside the pool
    x = copy.copy(tb)
    x.tx_comp_start = tb.tx_comp_start.copy()
    x.tx_comp_start[5], x.tx_comp_start[6] = x.tx_comp_start[6], x.tx_comp_start[5] - 1
    bad(ctx.txid_batch, x, want="tx_comp_start")
    x = copy.copy(tb)
    x.comp_off = tb.comp_off.copy()
    x.comp_off[-1] = len(tb.data)
    bad(ctx.txid_batch, x, want="component outside")
    assert np.array_equal(ctx.txid_batch(tb), ids)
    # fused: key index, signature range, template range
    y = copy.copy(sb)
    y.key_idx = sb.key_idx.copy()
    y.key_idx[7] = 10 ** 6
    bad(ctx.verify_tx_batch, tb, tm, y, want="key_idx")
    y = copy.copy(sb)
    y.sig_off = sb.sig_off.copy()
    y.sig_off[-1] = len(sb.sig_data)
    bad(ctx.verify_tx_batch, tb, tm, y, want="signature outside")
    z = copy.copy(tm)
    z.id_at = tm.id_at.copy()
    z.id_at[0] = int(tm.len[0]) + 1
    bad(ctx.verify_tx_batch, tb, z, sb, want="template")
    z = copy.copy(tm)
    z.max_len = int(tm.len.max()) - 1                # a template longer than the message slots
    bad(ctx.verify_tx_batch, tb, z, sb, want="template")
    gids, st, _ = ctx.verify_tx_batch(tb, tm, sb)
    assert np.array_equal(gids, ids) and np.array_equal(st, sb.expected)
    # FilteredTransaction: a component outside the pool
    ftxs, want = notary_workload(200, seed=4)
    fb = FtxBatch(ftxs)
    f2 = copy.copy(fb)
    f2.comp_off = fb.comp_off.copy()
    f2.comp_off[0] = len(fb.comp_data) + 3
    bad(ctx.ftx_verify_batch, f2, want="component outside")
    st, rs = ctx.ftx_verify_batch(fb)
    assert list(zip(st.tolist(), rs.tolist())) == want
    # chip_stx_verify: a blob outside the pool
    tb2, tm2, sb2, ids2, verdict, arg = G.cfg4_workload_commands(200, n_keys=8, seed=0x5EED0505, threads=8)
    data, off, ln = G.stx_uniform(tb2, sb2, 2)
    o2 = off.copy()
    o2[3] = len(data)
    bad(ctx.stx_verify, data, o2, ln, tm2, [[1, 4]], want="blob outside")
    z2 = copy.copy(tm2)
    z2.max_len = int(tm2.len.max()) - 1
    bad(ctx.stx_verify, data, off, ln, z2, [[1, 4]], want="template")
    st, v, a, _ = ctx.stx_verify(data, off, ln, tm2, [[1, 4]])
    assert not st.any() and np.array_equal(v, verdict)
    # uniqueness: tx_ref_start not starting at 0
    pre, ub = G.uniq_workload(500, 100, seed=31)
    t = ctx.uniq_open(4096)
    s2 = ub.tx_ref_start.copy()
    s2[0] = 1
    bad(t.commit_batch, s2, ub.refs, ub.tx_ids, ub.callers, want="tx_ref_start")
    st, _recs = t.commit_batch(ub.tx_ref_start, ub.refs, ub.tx_ids, ub.callers)
    assert (st == 0).sum() > 400
    t.close()


@pytest.mark.parametrize("chunks", [1, 4])
def test_pageable_input_through_the_staging_ring(ctx, monkeypatch, chunks):
    """Pageable host input (numpy arrays) through the context's pinned staging ring (CHIP_STAGING_RING=1: 4 MB
    pieces, parallel memcpy, DMA from the ring): statuses and bitmaps equal HIP's own pageable path (the default),
    the page-locked path and the labels, in one chunk and in four, also with the signatures permuted (every chunk
    copies a piece of the pools on both sides of what earlier chunks copied)."""
    import corda_amd
    monkeypatch.setenv("CHIP_STAGING_RING", "1")
    ring = corda_amd.Context(0)
    monkeypatch.delenv("CHIP_STAGING_RING")
    try:
        b = G.ed25519_batch(150000, n_keys=64, corrupt=0.1, seed=0x5EED0511)
        assert b.sig_data.nbytes > (4 << 20) and b.msg_data.nbytes > (4 << 20)
        monkeypatch.setenv("CHIP_HOST_CHUNKS", str(chunks))
        for x in (b, _permuted(b, 11)):
            st, bm = ring.verify_batch(x)
            assert np.array_equal(st, x.expected)
            st0, bm0 = ctx.verify_batch(x)
            assert np.array_equal(st, st0) and np.array_equal(bm, bm0)
        pb = copy.copy(b)
        for f in ("key_idx", "msg_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len",
                  "msg_data", "msg_off", "msg_len"):
            setattr(pb, f, ctx.pinned_copy(getattr(b, f)))
        stp, bmp = ctx.verify_batch(pb)
        assert np.array_equal(stp, b.expected)
        ctx.free_pinned()
    finally:
        ring.close()
