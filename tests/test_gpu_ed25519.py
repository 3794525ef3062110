"""GPU parity: Ed25519 verification through the C-ABI vs the CPU restatement (oracle).

Bit-exact on status bytes (CHIP_* codes) and the VALID bitmap, on seeded synthetic batches
with every corruption class of cfg2 plus hand-built edge cases."""
import hashlib

import numpy as np
import pytest

import cordagen as G

pytestmark = pytest.mark.gpu


def bitmap_of(status):
    n = len(status)
    words = np.zeros((n + 63) // 64, dtype=np.uint64)
    for i in np.nonzero(status == 0)[0]:
        words[i // 64] |= np.uint64(1) << np.uint64(i % 64)
    return words


MODES = ["default", "comb", "straus", "ungated"]


@pytest.mark.parametrize("mode", MODES)
def test_ed25519_batch_matches_oracle(ctx_modes, oracle, mode):
    ctx = ctx_modes[mode]
    b = G.ed25519_batch(3000, n_keys=64, corrupt=0.4, seed=11)
    st, bm = ctx.verify_batch(b)
    ref = oracle.verify_batch(b, threads=8)
    bad = np.nonzero(st != ref)[0]
    assert len(bad) == 0, [(int(i), int(b.kind[i]), int(st[i]), int(ref[i])) for i in bad[:20]]
    assert np.array_equal(st, b.expected)
    assert np.array_equal(bm, bitmap_of(ref))


@pytest.mark.parametrize("mode", MODES)
def test_ed25519_edge_cases(ctx_modes, oracle, mode):
    import golden_cases
    ctx = ctx_modes[mode]
    b = golden_cases.ed25519_edge_batch()
    st, _ = ctx.verify_batch(b)
    ref = oracle.verify_batch(b)
    assert st.tolist() == ref.tolist()
    assert st.tolist() == b.expected.tolist()


@pytest.mark.parametrize("mode", ["comb", "straus"])
@pytest.mark.parametrize("msg_len", [1, 55, 56, 63, 64, 111, 112, 127, 128, 200, 1000])
def test_ed25519_message_lengths(ctx_modes, oracle, msg_len, mode):
    ctx = ctx_modes[mode]
    # SHA-512 block boundaries (64 + |M| + 17 crossing 128-byte multiples)
    seed = hashlib.sha256(b"len%d" % msg_len).digest()
    a = G.ed25519_pub(seed)
    msgs, sigs = [], []
    for j in range(64):
        m = hashlib.sha512(b"m%d" % j).digest() * (msg_len // 64 + 1)
        m = m[:msg_len]
        msgs.append(m)
        s = bytearray(G.ed25519_sign(seed, m))
        if j % 3 == 1:
            s[5] ^= 4
        sigs.append(bytes(s))
    b = G.SigBatch()
    b.key_data, b.key_off, b.key_len = G.pools_from_list([G.spki_ed25519(a)])
    b.msg_data, b.msg_off, b.msg_len = G.pools_from_list(msgs)
    b.sig_data, b.sig_off, b.sig_len = G.pools_from_list(sigs)
    b.key_idx = np.zeros(64, dtype=np.uint32)
    b.msg_idx = np.arange(64, dtype=np.uint32)
    st, _ = ctx.verify_batch(b)
    ref = oracle.verify_batch(b)
    assert st.tolist() == ref.tolist()
    assert st.tolist() == [1 if j % 3 == 1 else 0 for j in range(64)]


def test_ed25519_mixed_policy_large(ctx_modes):
    """200k signatures with a skewed key distribution (hot keys on the comb, singletons on Straus in
    the default policy): every schedule gives the labels' status bytes."""
    b = G.ed25519_batch(200_000, n_keys=20_000, corrupt=0.1, seed=77)
    outs = {m: ctx_modes[m].verify_batch(b)[0] for m in MODES}
    for m in MODES:
        assert np.array_equal(outs[m], b.expected), m


def test_ed25519_comb_stats(ctx_modes):
    """The default policy (size gate off) routes repeated keys through the comb kernels (native path
    observable)."""
    from corda_amd import native
    c = ctx_modes["ungated"]
    c.reset_stats()
    b = G.ed25519_batch(4096, n_keys=16, corrupt=0.1, seed=5)
    st, _ = c.verify_batch(b)
    assert np.array_equal(st, b.expected)
    s = c.stats()
    assert s.kernel_launches[native.K_ED_COMB] >= 1
    assert s.kernel_launches[native.K_ED_FINISH] >= 1


def test_cfg2_shape_quarter_million_matches_oracle(ctx, oracle):
    """The headline schedule at a quarter of cfg2: 250,000 signatures over 4,096 keys on the device entry (eager
    per-key comb tables, challenge hash and [S]B started with the batch while the key prep and the tables run on
    the second stream) — every status byte equal to the oracle's and the labels, every corruption class present."""
    import torch
    b = G.ed25519_batch(250_000, n_keys=4096, corrupt=0.10, seed=0x5EED0602)
    dev = torch.device("cuda", 0)

    class D:
        pass
    d = D()
    for f in ("key_idx", "msg_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len", "msg_data",
              "msg_off", "msg_len"):
        a = getattr(b, f)
        a = a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32) if a.dtype == np.uint32 else a
        setattr(d, f, torch.from_numpy(np.ascontiguousarray(a)).to(dev))
    d.schemes_hint = 1 << 4
    st = torch.empty(b.n, dtype=torch.uint8, device=dev)
    bm = torch.empty((b.n + 63) // 64, dtype=torch.int64, device=dev)
    ctx.verify_batch_device(d, st, bm)
    torch.cuda.synchronize()
    got = st.cpu().numpy()
    ref = oracle.verify_batch(b, threads=16)
    bad = np.nonzero(got != ref)[0]
    assert len(bad) == 0, [(int(i), int(got[i]), int(ref[i]), int(b.kind[i])) for i in bad[:20]]
    assert np.array_equal(got, b.expected)
    assert len(set(b.kind.tolist())) == len(G.ED_KINDS)
    assert np.array_equal(bm.cpu().numpy().view(np.uint64), bitmap_of(got))


def _device_batch(b, dev):
    import torch

    class D:
        pass
    d = D()
    for f in ("key_idx", "msg_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len", "msg_data",
              "msg_off", "msg_len"):
        a = getattr(b, f)
        a = a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32) if a.dtype == np.uint32 else a
        setattr(d, f, torch.from_numpy(np.ascontiguousarray(a)).to(dev))
    return d


@pytest.mark.parametrize("env", [{}, {"CHIP_ED_STRAUS_EARLY": "0"}, {"CHIP_ED_STRAUS_SPLIT": "0"}],
                         ids=["split_early", "split", "fused"])
def test_cold_keys_device_entry_matches_oracle(oracle, env):
    """Cold keys (every signature its own key) on the device entry: the split Straus path (hash + [S]B comb,
    k_ed25519_verify_a, batched finish), with its hash and [S]B started beside the key prep (default) or after
    classify, and the fused k_ed25519_verify — every status byte equal to the oracle's and the labels; a second
    batch through the same context (reused rows and R' buffers) too."""
    import os
    import torch
    import corda_amd
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c = corda_amd.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    dev = torch.device("cuda", 0)
    try:
        for n, seed in ((40_000, 0x5EED0610), (9_000, 0x5EED0611)):
            b = G.ed25519_batch(n, n_keys=n, corrupt=0.2, seed=seed)
            d = _device_batch(b, dev)
            d.schemes_hint = 1 << 4
            st = torch.empty(b.n, dtype=torch.uint8, device=dev)
            bm = torch.empty((b.n + 63) // 64, dtype=torch.int64, device=dev)
            c.verify_batch_device(d, st, bm)
            torch.cuda.synchronize()
            got = st.cpu().numpy()
            ref = oracle.verify_batch(b, threads=16)
            bad = np.nonzero(got != ref)[0]
            assert len(bad) == 0, [(int(i), int(got[i]), int(ref[i]), int(b.kind[i])) for i in bad[:20]]
            assert np.array_equal(got, b.expected)
            assert np.array_equal(bm.cpu().numpy().view(np.uint64), bitmap_of(got))
    finally:
        c.close()
