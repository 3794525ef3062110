"""GPU: CHIP_FLAG_KEY_CACHE keeps the key state (decoded keys, per-key tables, comb tables) across batches and
reuses it only when the batch's key pool is the same, compared on the device key by key.  Every batch below is
checked against the oracle: a wrong reuse (tables of other keys) would change statuses."""
import copy
import os

import numpy as np
import pytest

import cordagen as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kctx():
    import corda_amd
    from corda_amd import native
    os.environ["CHIP_COMB_MIN_TOTAL"] = "0"   # test-sized batches take the eager comb schedules
    try:
        c = corda_amd.Context(0, flags=native.FLAG_KEY_CACHE)
    finally:
        del os.environ["CHIP_COMB_MIN_TOTAL"]
    yield c
    c.close()


def _keys(b):
    return [bytes(b.key_data[int(o):int(o) + int(n)]) for o, n in zip(b.key_off, b.key_len)]


def _with_keys(b, keys, key_idx):
    out = copy.copy(b)
    out.key_data, out.key_off, out.key_len = G.pools_from_list(keys)
    out.key_idx = np.ascontiguousarray(key_idx, dtype=np.uint32)
    return out


def permuted(b, p):
    """The same signatures with key j of the pool = old key p[j] (key_idx remapped)."""
    keys = _keys(b)
    pos = np.argsort(p)
    return _with_keys(b, [keys[k] for k in p], pos[b.key_idx])


def check(ctx, oracle, b):
    st, bm = ctx.verify_batch(b)
    ref = oracle.verify_batch(b, threads=8)
    bad = np.nonzero(st != ref)[0]
    assert len(bad) == 0, [(int(i), int(st[i]), int(ref[i])) for i in bad[:10]]
    return st


def test_key_cache_ed25519_pool_changes(kctx, oracle):
    b = G.ed25519_batch(4000, n_keys=32, corrupt=0.3, seed=5)
    st = check(kctx, oracle, b)
    assert np.array_equal(st, b.expected)
    check(kctx, oracle, b)                                   # same pool: reused
    p = np.random.Generator(np.random.PCG64(1)).permutation(len(b.key_off))
    check(kctx, oracle, permuted(b, p))                      # same keys, other order: rebuilt
    check(kctx, oracle, b)
    keys = _keys(b)
    keys[7] = keys[7][:-1] + bytes([keys[7][-1] ^ 1])        # one key's last byte
    check(kctx, oracle, _with_keys(b, keys, b.key_idx))
    check(kctx, oracle, b)
    small = G.ed25519_batch(2000, n_keys=16, corrupt=0.3, seed=6)   # another key count
    check(kctx, oracle, small)
    check(kctx, oracle, b)
    check(kctx, oracle, b)


def test_key_cache_ecdsa_and_mixed(kctx, oracle):
    e = G.ecdsa_batch(3000, n_keys=16, corrupt=0.3, seed=9)
    check(kctx, oracle, e)
    check(kctx, oracle, e)
    p = np.random.Generator(np.random.PCG64(2)).permutation(len(e.key_off))
    check(kctx, oracle, permuted(e, p))
    check(kctx, oracle, e)
    b = G.ed25519_batch(4000, n_keys=32, corrupt=0.3, seed=5)
    check(kctx, oracle, b)
    check(kctx, oracle, e)
    check(kctx, oracle, e)


def test_key_cache_state_dropped_after_a_failed_batch(oracle):
    """A batch that fails after k_key_cache copied its pool (here: CHIP_TEST_FAIL_KEYSTATE forces CHIP_E_NOMEM
    before the key preps / table builds are enqueued, as a failed allocation would) must not leave the cache
    describing that pool: the same pool again is rebuilt (no reuse check: key_cache_checks does not move) and its
    statuses equal the oracle's; the call after that may reuse the rebuilt state."""
    import corda_amd
    from corda_amd import native
    os.environ["CHIP_COMB_MIN_TOTAL"] = "0"
    os.environ["CHIP_TEST_FAIL_KEYSTATE"] = "2"      # the second key-cache batch fails
    try:
        c = corda_amd.Context(0, flags=native.FLAG_KEY_CACHE)
    finally:
        del os.environ["CHIP_COMB_MIN_TOTAL"]
        del os.environ["CHIP_TEST_FAIL_KEYSTATE"]
    try:
        p = G.ed25519_batch(4000, n_keys=32, corrupt=0.3, seed=11)
        q = G.ed25519_batch(4000, n_keys=32, corrupt=0.3, seed=12)   # same key count, other keys
        check(c, oracle, p)
        with pytest.raises(native.ChipError) as e:
            c.verify_batch(q)
        assert e.value.code == -3
        before = c.stats().key_cache_checks
        st = check(c, oracle, q)                      # rebuilt: the failed call's pool copy is not trusted
        assert np.array_equal(st, q.expected)
        assert c.stats().key_cache_checks == before
        check(c, oracle, q)                           # now a reuse candidate again
        assert c.stats().key_cache_checks == before + 1
        check(c, oracle, p)
    finally:
        c.close()
