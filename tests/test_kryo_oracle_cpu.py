"""CPU: the oracle's restatement of the Kryo front end (oracle/kryo_ref.c, written as a de-chunking
recursive-descent reader) against the host mirror (corda_amd/kryo.py + keys.py) on every test blob and
on thousands of damaged ones; the -m gpu tests then compare the device with the oracle.

PARITY UNPINNED for the bytes (no JVM output exists in the reference or here): what is pinned is that two
independent restatements of the reference's serializers / init checks / CompositeKey rules agree, and that
each documented rule (registry ids, canonical StateRef inputs, key decoding, composite canonical form)
gives the status the reference's semantics call for."""
import collections

import numpy as np
import pytest

import oracle_bind as O
import stx_build as S
from corda_amd import composite as CK
from corda_amd import keys as KS
from corda_amd import kryo as K

REG = K.DEFAULT_REGISTRY


def _same_parse(orc, mir):
    assert orc[0] == mir[0]
    if mir[0] == K.STX_OK:
        assert orc[2] == [(g, list(c)) for g, c in mir[1]]
        assert orc[3] == mir[2]
        assert orc[4] == list(mir[3])


def test_oracle_equals_mirror_on_cases():
    blobs = S.cases(seed=7, n_valid=300)
    orc = O.stx_parse(blobs, REG)
    for i, b in enumerate(blobs):
        _same_parse(orc[i], K.stx_parse(b))
    assert {o[0] for o in orc} == {0, 1, 2, 3, 4}


def test_oracle_equals_mirror_required_keys():
    blobs = S.cases_required(seed=13, n=400)
    want, _kid = S.expected_required(blobs)
    orc = O.stx_parse(blobs, REG, want_required=True)
    for (pst, fst, g, salt, sigs, trees), (wst, wtrees) in zip(orc, want):
        assert fst == wst
        if wst == K.STX_OK:
            assert trees == wtrees
    c = collections.Counter(o[1] for o in orc)
    assert c[K.STX_OK] > 300 and c[K.STX_UNSUPPORTED] >= 30
    # composite trees (nested included) are decoded, not sent to the JVM
    assert sum(1 for o in orc if o[1] == 0 and any(len(t) > 1 for t in o[5])) >= 30
    assert any(o[1] == 0 and any(sum(1 for n in t if n[2]) > 1 for t in o[5]) for o in orc)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_oracle_equals_mirror_on_damaged_blobs(seed):
    """4 x 25,000 mutants (1-3 bit flips, byte changes, deletions, insertions, truncations) of 120 base
    blobs each: the oracle and the mirror agree on every parse status, required-signer status and result."""
    base = S.cases(seed=7 + seed, n_valid=40)[:40] + S.cases_required(seed=13 + seed, n=80)
    blobs = S.mutants(base, seed=seed, n=25_000)
    orc = O.stx_parse(blobs, REG, want_required=True)
    mir = [K.stx_parse(b) for b in blobs]
    want, _ = S.expected_required(blobs)
    for o, m, (wst, wtrees) in zip(orc, mir, want):
        _same_parse(o, m)
        assert o[1] == wst
        if wst == K.STX_OK:
            assert o[5] == wtrees
    assert {0, 1, 4} <= {o[0] for o in orc}


def test_registry_is_a_parameter():
    """The oracle takes the registry like the device: blobs written with other ids parse under those ids
    and fail closed under the defaults."""
    ids = K.registration_ids(K.REGISTRATION_ORDER[:20] + [("x.Extra", "")] + K.REGISTRATION_ORDER[20:])
    other = K.Registry(ids)
    rng = np.random.default_rng(4)
    keys = S.key_pool(rng)
    blobs = []
    for _ in range(20):
        groups, salt, sigs, kinds, skind = S.random_valid(rng, keys)
        sigs = [K.Sig(s.sig, s.key, s.platform_version, s.scheme_number_id,
                      other.eddsa_public_key if len(s.key) == 44 else other.bcec_public_key) for s in sigs]
        blobs.append(K.signed_transaction(K.wire_transaction(groups, salt, other.privacy_salt, kinds), sigs, skind))
    assert [o[0] for o in O.stx_parse(blobs, other)] == [K.stx_parse(b, other)[0] for b in blobs] == [0] * 20
    assert [o[0] for o in O.stx_parse(blobs, REG)] == [K.stx_parse(b, REG)[0] for b in blobs] == [4] * 20


def test_key_rules():
    rng = np.random.default_rng(8)
    ed, r1, k1 = S.ed_key(rng), S.ec_key(rng, 3), S.ec_key(rng, 2)
    for k in (ed, r1, k1, S.ec_key(rng, 3, compressed=True)):
        assert KS.plain_key_ok(k)
    assert KS.plain_key_canonical(ed) and KS.plain_key_canonical(r1)
    assert not KS.plain_key_canonical(S.ec_key(rng, 3, compressed=True))
    assert not KS.plain_key_ok(S.bad_ed_key(rng)) and not KS.plain_key_ok(S.bad_ec_key(rng))
    # Ed25519: y >= p decodes (i2p takes y mod p) but is not the canonical encoding
    y = (2**255 - 19) + 1                        # y = 1 mod p: the identity
    a = y.to_bytes(32, "little")
    assert KS.ed25519_point_ok(a) and not KS.ed25519_canonical(a)
    assert not KS.ed25519_canonical(bytes([1] + [0] * 30 + [0x80]))   # x = 0 with the sign bit set
    # the same rules in the oracle's primitives
    for k in (ed, r1, k1, S.bad_ed_key(rng), S.bad_ec_key(rng)):
        scheme, raw = KS.spki_scheme(k)
        if scheme == KS.ED25519:
            assert (O.ed25519_decode_key(raw) is not None) == KS.plain_key_ok(k)
        else:
            assert (O.ecdsa_decode_key(scheme, raw) is not None) == KS.plain_key_ok(k)


def test_composite_rules():
    rng = np.random.default_rng(9)
    p = [S.ed_key(rng) for _ in range(6)] + [S.ec_key(rng, 3)]
    c = S.composite([(p[0], 1), (p[1], 2), (p[6], 1)], 2)
    tree = KS.composite_tree(c)
    assert [n[2] for n in tree] == [0, 0, 0, 3] and tree[-1][1] == 2
    assert sorted(n[3] for n in tree[:3]) == [1, 1, 2]
    nested = S.composite([(S.composite([(p[2], 1), (p[3], 1)], 1), 3), (p[4], 1)], 3)
    assert [n[2] for n in KS.composite_tree(nested)] == [0, 0, 0, 2, 2] or \
        [n[2] for n in KS.composite_tree(nested)] == [0, 0, 2, 0, 2]
    # the host CompositeKey (composite.py) and the tree agree on fulfilment for every signer subset
    key = CK.as_key(nested)
    for mask in range(1 << 3):
        signers = [p[2 + i] for i in range(3) if mask >> i & 1]
        t = KS.composite_tree(nested)
        assert _eval(t, set(signers)) == key.is_fulfilled_by(signers)
    bad = [S.composite_raw([(p[1], 1), (p[0], 1)] if p[1] > p[0] else [(p[0], 1), (p[1], 1)], 1),   # unsorted
           S.composite_raw([(p[0], 1), (p[1], 1)], 3),
           S.composite_raw([(p[0], 1), (p[0], 1)], 1),
           S.composite_raw([(p[0], 1)], 1),
           S.composite_raw([(p[0], 0), (p[1], 1)], 1),
           S.composite_raw([(p[0], 2**31 - 1), (p[1], 2**31 - 1)], 1)]
    for b in bad:
        with pytest.raises(KS.KeyUnsupported):
            KS.composite_tree(b)
    deep = p[0]
    for i in range(9):                           # 8 levels of composites decode, the 9th does not
        if i == 8:
            assert len(KS.composite_tree(deep)) == 17
        deep = S.composite([(deep, 1), (p[1 + i % 5], 1)], 1)
    with pytest.raises(KS.KeyUnsupported):
        KS.composite_tree(deep)


def _eval(tree, signers):
    """Post-order evaluation of a composite tree (k_required_signers' rule)."""
    stack = []
    for leaf, thr, nk, w in tree:
        if nk == 0:
            stack.append((leaf in signers, w))
        else:
            kids = stack[-nk:]
            del stack[-nk:]
            stack.append((sum(kw for ok, kw in kids if ok) >= thr, w))
    return stack[-1][0]
