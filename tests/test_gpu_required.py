"""GPU parity: required-signer check on the device (k_required_signers via chip_required_signers*,
chip_verify_signed_tx_batch*) vs the oracle restatement (oracle/required_ref.c): verdicts, first
failing signature, missing-key flags — seeded random batches with nested CompositeKey trees, a key
pool with byte-identical duplicates, CHIP_REQ_NO_SIGNER leaves, allowedToBeMissing flags and every
MALFORMED class; the fused cfg4 pipeline (ids -> messages -> signatures -> required signers) against
generator labels and the oracle; the Python mirror's batch verifySignaturesExcept with composites."""
import hashlib

import numpy as np
import pytest

import cordagen as G
import req_build as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,malformed", [(11, False), (12, True), (13, True)])
def test_required_signers_matches_oracle(ctx, oracle, seed, malformed):
    q, b, st, _ = R.make(ntx=5000, seed=seed, malformed=malformed)
    v, a, m = ctx.required_signers(q, b, st)
    ov, oa, om = oracle.required_signers(q, b, st)
    assert np.array_equal(v, ov)
    assert np.array_equal(a, oa)
    assert np.array_equal(m, om)
    assert len(np.unique(v)) >= (4 if malformed else 3)


def test_required_signers_device_entry(ctx, oracle):
    import torch
    dev = torch.device("cuda", 0)
    q, b, st, _ = R.make(ntx=3000, seed=21, dup_keys=16)

    def t(a):
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        elif a.dtype == np.uint32:
            a = a.view(np.int32)
        return torch.from_numpy(a).to(dev)

    class D:
        pass
    dq, db = D(), D()
    dq.ntx = q.ntx
    for f in ("sig_start", "req_start", "node_start", "allowed", "node_val", "node_nkids", "node_weight"):
        setattr(dq, f, t(getattr(q, f)))
    for f in ("key_idx", "msg_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len", "msg_data",
              "msg_off", "msg_len"):
        setattr(db, f, t(getattr(b, f)))
    dst = t(st)
    verdict = torch.empty(q.ntx, dtype=torch.uint8, device=dev)
    arg = torch.empty(q.ntx, dtype=torch.int32, device=dev)
    missing = torch.empty(len(q.node_start) - 1, dtype=torch.uint8, device=dev)
    ctx.required_signers_device(dq, db, dst, verdict, arg, missing)
    torch.cuda.synchronize()
    ov, oa, om = oracle.required_signers(q, b, st)
    assert np.array_equal(verdict.cpu().numpy(), ov)
    assert np.array_equal(arg.cpu().numpy().view(np.uint32), oa)
    assert np.array_equal(missing.cpu().numpy(), om)


def test_fused_signed_tx_cfg4(ctx, oracle):
    """chip_verify_signed_tx_batch on the cfg4 shape: ids, statuses, verdicts and missing flags equal
    the generator labels and the oracle (run on host-built messages)."""
    tb, tm, sb, ids, msgs = G.cfg4_workload(4000, n_keys=64, corrupt=0.03, seed=31, threads=8)
    q = G.cfg4_required(sb, tb.ntx, 64, p_composite=0.1, p_missing=0.05)
    gids, st, v, a, m = ctx.verify_signed_tx_batch(tb, tm, sb, q)
    assert np.array_equal(gids, ids)
    assert np.array_equal(st, sb.expected)
    assert np.array_equal(v, q.expected_verdict)
    assert np.array_equal(a, q.expected_arg)
    plain = G.signer_sig_batch(sb, msgs)
    ov, oa, om = oracle.required_signers(q, plain, oracle.verify_batch(plain, threads=8), tx_idx=sb.tx_idx)
    assert np.array_equal(v, ov) and np.array_equal(a, oa) and np.array_equal(m, om)
    assert set(np.unique(v).tolist()) == {0, 1, 2}


def test_fused_signed_tx_foreign_signature(ctx, oracle):
    """A signature inside tx t's range that carries another transaction's tx_idx: t is MALFORMED
    (the signature itself is verified against the other transaction's message)."""
    tb, tm, sb, ids, msgs = G.cfg4_workload(600, n_keys=16, corrupt=0.0, seed=41, threads=8)
    q = G.cfg4_required(sb, tb.ntx, 16)
    sb.tx_idx = sb.tx_idx.copy()
    sb.tx_idx[2 * 7] = 8
    gids, st, v, a, m = ctx.verify_signed_tx_batch(tb, tm, sb, q)
    assert v[7] == 3 and st[14] == 1
    plain = G.signer_sig_batch(sb, msgs)
    plain.msg_idx = sb.tx_idx.astype(np.uint32)
    ov, oa, om = oracle.required_signers(q, plain, oracle.verify_batch(plain, threads=8), tx_idx=sb.tx_idx)
    assert np.array_equal(v, ov) and np.array_equal(a, oa)


def test_fused_signed_tx_device_entry(ctx):
    import torch
    dev = torch.device("cuda", 0)
    tb, tm, sb, ids, msgs = G.cfg4_workload(2000, n_keys=32, corrupt=0.02, seed=51, threads=8)
    q = G.cfg4_required(sb, tb.ntx, 32, p_composite=0.05, p_missing=0.05)

    def up(obj, fields):
        class D:
            pass
        d = D()
        for f in fields:
            x = np.ascontiguousarray(getattr(obj, f))
            if x.dtype == np.uint64:
                x = x.view(np.int64)
            elif x.dtype == np.uint32:
                x = x.view(np.int32)
            setattr(d, f, torch.from_numpy(x).to(dev))
        return d
    dt = up(tb, ["salts", "tx_comp_start", "comp_group", "comp_internal", "data", "comp_off", "comp_len"])
    dt.ntx = tb.ntx
    dm = up(tm, ["data", "off", "len", "id_at"])
    dm.max_len = tm.max_len
    ds = up(sb, ["tx_idx", "tmpl_idx", "key_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len"])
    dq = up(q, ["sig_start", "req_start", "node_start", "node_val", "node_nkids", "node_weight"])
    dq.ntx = q.ntx
    gids = torch.empty(tb.ntx * 32, dtype=torch.uint8, device=dev)
    st = torch.empty(sb.n, dtype=torch.uint8, device=dev)
    v = torch.empty(tb.ntx, dtype=torch.uint8, device=dev)
    a = torch.empty(tb.ntx, dtype=torch.int32, device=dev)
    ctx.verify_signed_tx_batch_device(dt, dm, ds, dq, gids, st, v, a)
    torch.cuda.synchronize()
    assert np.array_equal(gids.cpu().numpy().reshape(-1, 32), ids)
    assert np.array_equal(v.cpu().numpy(), q.expected_verdict)
    assert np.array_equal(a.cpu().numpy().view(np.uint32), q.expected_arg)


def test_python_mirror_batch_with_composites_on_gpu(ctx):
    """verify_signatures_except_batch through the HIP engine == the sequential reference-semantics
    path through the oracle engine (CompositeKey trees, allowedToBeMissing)."""
    from corda_amd import crypto as C
    from corda_amd.composite import CompositeKey
    from oracle_engine import OracleEngine
    seeds = [hashlib.sha256(b"greq-%d" % i).digest() for i in range(6)]
    keys = [G.spki_ed25519(G.ed25519_pub(s)) for s in seeds]
    rng = np.random.Generator(np.random.PCG64(5))
    meta = C.SignatureMetadata(1, 4)
    stxs = []
    for t in range(120):
        tid = hashlib.sha256(b"g%d" % t).digest()
        who = rng.choice(6, size=int(rng.integers(1, 4)), replace=False)
        sigs = []
        for i in who:
            s = bytearray(G.ed25519_sign(seeds[int(i)], C.signable_data_bytes(tid, meta)))
            if rng.random() < 0.05:
                s[0] ^= 1
            sigs.append(C.TransactionSignature(bytes(s), keys[int(i)], meta))
        ks = rng.choice(6, size=3, replace=False)
        ck = CompositeKey.Builder().add_key(keys[int(ks[0])], 2).add_key(keys[int(ks[1])]).add_key(
            keys[int(ks[2])]).build(int(rng.integers(1, 4)))
        stxs.append(C.SignedTransaction(tid, sigs, {ck, keys[int(rng.integers(0, 6))]}))
    got = C.verify_signatures_except_batch(ctx, stxs, [keys[5]])
    eng = OracleEngine()
    for stx, g in zip(stxs, got):
        try:
            stx.verify_signatures_except(eng, keys[5])
            want = None
        except Exception as e:   # noqa: BLE001
            want = e
        assert type(g) is type(want)
        if want is not None:
            assert str(g) == str(want)
