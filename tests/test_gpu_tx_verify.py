"""GPU parity: fused transaction verification (chip_verify_tx_batch) — WireTransaction.id recomputed
on the device, SignableData messages built on the device from the ids, every required signer
verified — vs the oracle run on host-built messages (cfg4 shape)."""
import numpy as np
import pytest

import cordagen as G

pytestmark = pytest.mark.gpu


def test_fused_cfg4_matches_oracle(ctx, oracle):
    tb, tm, sb, ids, msgs = G.cfg4_workload(3000, n_keys=64, corrupt=0.05, threads=8)
    gids, st, bm = ctx.verify_tx_batch(tb, tm, sb)
    assert np.array_equal(gids, oracle.txid_batch(tb, threads=8))
    assert np.array_equal(gids, ids)
    ref = oracle.verify_batch(G.signer_sig_batch(sb, msgs), threads=8)
    assert np.array_equal(st, ref)
    assert np.array_equal(st, sb.expected)
    assert (st == 1).sum() > 0


def test_fused_device_entry(ctx, oracle):
    import torch
    tb, tm, sb, ids, msgs = G.cfg4_workload(1500, n_keys=16, corrupt=0.05, seed=77, threads=8)
    dev = torch.device("cuda", 0)

    def up(obj, fields):
        class D:
            pass
        d = D()
        for f in fields:
            a = getattr(obj, f)
            if a.dtype == np.uint64:
                a = a.view(np.int64)
            elif a.dtype == np.uint32:
                a = a.view(np.int32)
            setattr(d, f, torch.from_numpy(np.ascontiguousarray(a)).to(dev))
        return d
    dt = up(tb, ["salts", "tx_comp_start", "comp_group", "comp_internal", "data", "comp_off", "comp_len"])
    dt.ntx = tb.ntx
    dm = up(tm, ["data", "off", "len", "id_at"])
    dm.max_len = tm.max_len
    ds = up(sb, ["tx_idx", "tmpl_idx", "key_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len"])
    gids = torch.empty(tb.ntx * 32, dtype=torch.uint8, device=dev)
    st = torch.empty(sb.n, dtype=torch.uint8, device=dev)
    bm = torch.empty((sb.n + 63) // 64, dtype=torch.int64, device=dev)
    ctx.verify_tx_batch_device(dt, dm, ds, gids, st, bm)
    torch.cuda.synchronize()
    assert np.array_equal(gids.cpu().numpy().reshape(-1, 32), ids)
    assert np.array_equal(st.cpu().numpy(), sb.expected)


def test_fused_templates_and_bad_indices(ctx, oracle):
    """Two SignableData templates (platformVersion 1 and 2), a template whose id sits at offset 0,
    and signatures with an out-of-range tx / template index (-> UNSUPPORTED, JCA fallback)."""
    tb, tm, sb, ids, msgs = G.cfg4_workload(400, n_keys=8, corrupt=0.0, seed=5, threads=8)
    t1, a1 = G.signable_template(4, platform_version=1)
    t2, a2 = G.signable_template(4, platform_version=2, total=120)
    t3, a3 = b"\x07" * 40, 0
    tm = G.templates_from_list([(t1, a1), (t2, a2), (t3, a3)])
    n = sb.n
    tmpl_idx = (np.arange(n) % 3).astype(np.uint32)
    # re-sign each signature over its own template's message
    seeds = [G.key_seed(i) for i in range(8)] + [G.NOTARY_SEED]
    sigs = np.zeros((n, 64), dtype=np.uint8)
    host_msgs = []
    for i in range(n):
        tb_, at_ = [(t1, a1), (t2, a2), (t3, a3)][tmpl_idx[i]]
        m = tb_[:at_] + ids[sb.tx_idx[i]].tobytes() + tb_[at_:]
        host_msgs.append(m)
        sigs[i] = np.frombuffer(G.ed25519_sign(seeds[sb.key_idx[i]], m), dtype=np.uint8)
    sb.sig_data = sigs.reshape(-1)
    sb.tmpl_idx = tmpl_idx
    sb.tx_idx = sb.tx_idx.copy()
    sb.tx_idx[5] = tb.ntx + 3          # tx out of range
    sb.tmpl_idx[9] = 3                 # template out of range
    gids, st, _ = ctx.verify_tx_batch(tb, tm, sb)
    want = np.zeros(n, dtype=np.uint8)
    want[5] = want[9] = 5
    assert np.array_equal(gids, ids)
    assert st.tolist() == want.tolist()
    # the oracle agrees on the in-range signatures
    b = G.SigBatch()
    b.key_idx, b.sig_data, b.sig_off, b.sig_len = sb.key_idx, sb.sig_data, sb.sig_off, sb.sig_len
    b.key_data, b.key_off, b.key_len = sb.key_data, sb.key_off, sb.key_len
    b.msg_data, b.msg_off, b.msg_len = G.pools_from_list(host_msgs)
    b.msg_idx = np.arange(n, dtype=np.uint32)
    ref = oracle.verify_batch(b)
    keep = np.ones(n, bool)
    keep[[5, 9]] = False
    assert np.array_equal(st[keep], ref[keep])
