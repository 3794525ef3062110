"""Required-signer check (chip_required_signers contract) on the CPU: the oracle restatement
(oracle/required_ref.c) against
  * the host mirror of the Kotlin semantics (corda_amd.composite / SignedTransaction, per transaction:
    checkSignaturesAreValid, getMissingSigners with CompositeKey thresholds, minus allowedToBeMissing,
    TransactionWithSignatures.kt:44-50,62-66,79-85, CompositeKey.kt:175-185), and
  * an independent pure-Python evaluation of the flattened layout (incl. the MALFORMED rules),
plus ResolveTransactionsFlow.topologicalSort (ResolveTransactionsFlow.kt:37-62)."""
import hashlib

import numpy as np
import pytest

import cordagen as G
import oracle_bind as O
import req_build as R
from corda_amd import crypto as C
from corda_amd.composite import CompositeKey
from oracle_engine import OracleEngine

B = CompositeKey.Builder
OK, SIG, MISS, BAD = range(4)


def py_eval(q, b, status, tx_idx=None):
    """Flattened-layout restatement: recursive isFulfilledBy from each root."""
    nk_pool = len(b.key_off)
    keys = [bytes(b.key_data[int(o):int(o) + int(n)]) for o, n in zip(b.key_off, b.key_len)]
    nreq = len(q.node_start) - 1
    verdict, arg, missing = [], [], np.zeros(nreq, np.uint8)
    for t in range(q.ntx):
        s0, s1, r0, r1 = (int(x) for x in (q.sig_start[t], q.sig_start[t + 1], q.req_start[t], q.req_start[t + 1]))
        if s0 > s1 or s1 > len(b.key_idx) or not (r0 <= r1 <= nreq):
            verdict.append(BAD), arg.append(0)
            continue
        if any((tx_idx is not None and tx_idx[j] != t) or b.key_idx[j] >= nk_pool for j in range(s0, s1)):
            verdict.append(BAD), arg.append(0)
            continue
        bad_sig = [j for j in range(s0, s1) if status[j] != 0]
        if bad_sig:
            verdict.append(SIG), arg.append(bad_sig[0])
            continue
        signer_keys = {keys[int(b.key_idx[j])] for j in range(s0, s1)}
        needed, malformed, miss = 0, False, {}
        for r in range(r0, r1):
            a, e = int(q.node_start[r]), int(q.node_start[r + 1])
            # pending-subtree limit of the engine
            sp, ok = 0, a < e <= len(q.node_val)
            for j in range(a, e if ok else a):
                sp -= int(q.node_nkids[j])
                if sp < 0 or sp >= C.REQ_MAX_PENDING:
                    ok = False
                    break
                sp += 1
            if not ok or sp != 1:
                malformed = True
                break

            def ful(j):
                n = int(q.node_nkids[j])
                if n == 0:
                    k = int(q.node_val[j])
                    if k == R.NO_SIGNER:
                        return False, j
                    if k >= nk_pool:
                        raise ValueError
                    return keys[k] in signer_keys, j
                total, c = 0, j
                for _ in range(n):
                    f, first = ful(c - 1)
                    total += int(q.node_weight[c - 1]) if f else 0
                    c = first
                return total >= int(q.node_val[j]), c
            try:
                f, _ = ful(e - 1)
            except ValueError:
                malformed = True
                break
            m = (not f) and not (len(q.allowed) and q.allowed[r])
            miss[r] = m
            needed += m
        if malformed:
            verdict.append(BAD), arg.append(0)
            continue
        for r, m in miss.items():
            missing[r] = m
        verdict.append(MISS if needed else OK), arg.append(needed)
    return np.array(verdict, np.uint8), np.array(arg, np.uint32), missing


@pytest.mark.parametrize("seed,malformed", [(1, False), (2, False), (3, True), (4, True)])
def test_oracle_matches_flattened_restatement(seed, malformed):
    q, b, st, tx_idx = R.make(ntx=1500, seed=seed, malformed=malformed)
    for ti in (None, tx_idx):
        v, a, m = O.required_signers(q, b, st, tx_idx=ti)
        pv, pa, pm = py_eval(q, b, st, ti)
        assert np.array_equal(v, pv)
        assert np.array_equal(a, pa)
        assert np.array_equal(m, pm)
    assert {int(x) for x in np.unique(v)} >= ({OK, SIG, MISS, BAD} if malformed else {OK, SIG, MISS})


def test_pending_limit_and_no_signer():
    """A CompositeKey node with CHIP_REQ_MAX_PENDING children is accepted, one more pending subtree is
    MALFORMED; a CHIP_REQ_NO_SIGNER leaf is never fulfilled."""
    q, b, st, _ = R.make(ntx=1, seed=9, max_sigs=2, max_req=0)
    st[:] = 0
    k = int(b.key_idx[0]) if len(b.key_idx) else 0
    for width, want in ((C.REQ_MAX_PENDING, OK), (C.REQ_MAX_PENDING + 1, BAD)):
        q.node_val = np.array([k] + [R.NO_SIGNER] * (width - 1) + [1], np.uint32)
        q.node_nkids = np.array([0] * width + [width], np.uint32)
        q.node_weight = np.ones(width + 1, np.uint32)
        q.node_start = np.array([0, width + 1], np.uint64)
        q.req_start = np.array([0, 1], np.uint64)
        q.allowed = np.zeros(1, np.uint8)
        has_sig = int(q.sig_start[1]) > 0
        v, a, m = O.required_signers(q, b, st)
        assert int(v[0]) == (want if has_sig or want == BAD else MISS)
        assert np.array_equal(v, py_eval(q, b, st)[0])
    q.node_val = np.array([R.NO_SIGNER], np.uint32)
    q.node_nkids = np.zeros(1, np.uint32)
    q.node_weight = np.ones(1, np.uint32)
    q.node_start = np.array([0, 1], np.uint64)
    v, a, m = O.required_signers(q, b, st)
    assert (int(v[0]), int(a[0]), int(m[0])) == (MISS, 1, 1)


# ---- against the host mirror of the Kotlin semantics ----
SEEDS = [hashlib.sha256(b"req-%d" % i).digest() for i in range(8)]
KEYS = [G.spki_ed25519(G.ed25519_pub(s)) for s in SEEDS]


def _sig(i, tx_id, bad=False):
    m = C.signable_data_bytes(tx_id, C.SignatureMetadata(1, 4))
    s = bytearray(G.ed25519_sign(SEEDS[i], m))
    if bad:
        s[3] ^= 1
    return C.TransactionSignature(bytes(s), KEYS[i], C.SignatureMetadata(1, 4))


def _random_key(rng, depth):
    if depth and rng.random() < 0.6:
        kids = rng.choice(len(KEYS), size=int(rng.integers(2, 5)), replace=False)
        b = B()
        total = 0
        for k in kids:
            sub = _random_key(rng, depth - 1) if rng.random() < 0.3 else KEYS[int(k)]
            w = int(rng.integers(1, 4))
            total += w
            b.add_key(sub, w)
        try:
            return b.build(int(rng.integers(1, total + 1)))
        except Exception:     # duplicated child nodes: use a plain key
            return KEYS[int(kids[0])]
    return KEYS[int(rng.integers(0, len(KEYS)))]


@pytest.fixture(scope="module")
def eng():
    return OracleEngine()


def test_batch_equals_sequential_with_composites(eng):
    rng = np.random.Generator(np.random.PCG64(77))
    stxs, allowed = [], [KEYS[7]]
    for t in range(150):
        tx_id = hashlib.sha256(b"tx%d" % t).digest()
        signers = rng.choice(len(KEYS), size=int(rng.integers(1, 5)), replace=False)
        sigs = [_sig(int(i), tx_id, bad=rng.random() < 0.04) for i in signers]
        req = {_random_key(rng, 2) for _ in range(int(rng.integers(1, 4)))}
        if rng.random() < 0.2:
            req.add(KEYS[7])
        stxs.append(C.SignedTransaction(tx_id, sigs, req))
    batch = C.verify_signatures_except_batch(eng, stxs, allowed)
    outcomes = {"none": 0, "sig": 0, "missing": 0}
    for stx, got in zip(stxs, batch):
        try:
            stx.verify_signatures_except(eng, *allowed)
            want = None
        except Exception as e:   # noqa: BLE001
            want = e
        assert type(got) is type(want)
        if isinstance(want, C.SignaturesMissingException):
            assert got.missing == want.missing
            outcomes["missing"] += 1
        elif want is None:
            outcomes["none"] += 1
        else:
            outcomes["sig"] += 1
            assert str(got) == str(want)
    assert min(outcomes.values()) > 3


def test_invalid_composite_raises_only_after_signatures(eng):
    """isFulfilledBy validates the CompositeKey first (CompositeKey.kt:192-198) — but only once every
    signature passed checkSignaturesAreValid."""
    tx_id = hashlib.sha256(b"inv").digest()
    ck = B().add_keys(KEYS[0], KEYS[1]).build(2)
    ck.children = ck.children + [ck.children[0]]          # duplicated child: checkValidity fails
    good = C.SignedTransaction(tx_id, [_sig(0, tx_id)], [ck])
    badsig = C.SignedTransaction(tx_id, [_sig(0, tx_id, bad=True)], [ck])
    r = C.verify_signatures_except_batch(eng, [good, badsig])
    assert isinstance(r[0], C.IllegalArgumentException)
    assert isinstance(r[1], C.SignatureException)


class _Stx:
    def __init__(self, name, inputs):
        self.id = hashlib.sha256(name.encode()).digest()
        self.name = name
        self.inputs = [hashlib.sha256(i.encode()).digest() for i in inputs]


def test_topological_sort():
    """ResolveTransactionsFlowTest-style graph: dependencies before dependers, deterministic for one
    input order, duplicate ids rejected."""
    a, b = _Stx("a", []), _Stx("b", ["a"])
    c, d = _Stx("c", ["a", "b"]), _Stx("d", ["c", "zz"])
    for order in ([d, c, b, a], [a, b, c, d], [c, a, d, b]):
        res = C.topological_sort(order, lambda s: s.inputs)
        pos = {s.name: i for i, s in enumerate(res)}
        assert pos["a"] < pos["b"] < pos["c"] < pos["d"]
        assert res == C.topological_sort(order, lambda s: s.inputs)
    with pytest.raises(C.IllegalArgumentException):
        C.topological_sort([a, _Stx("a", [])], lambda s: s.inputs)


def test_resolve_transactions_verify(eng):
    tx_ids = [hashlib.sha256(b"r%d" % i).digest() for i in range(4)]

    class S(C.SignedTransaction):
        pass
    stxs = []
    for i, tid in enumerate(tx_ids):
        s = C.SignedTransaction(tid, [_sig(i, tid, bad=(i == 2))], [KEYS[i]])
        s.inputs = [tx_ids[i - 1]] if i else []
        stxs.append(s)
    order, first = C.resolve_transactions_verify(eng, list(reversed(stxs)), lambda s: s.inputs)
    assert [s.id for s in order] == tx_ids
    assert first[0] == 2 and isinstance(first[1], C.SignatureException)
