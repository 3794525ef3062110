"""CPU: the Kryo SignedTransaction / WireTransaction restatement (corda_amd/kryo.py) — the host mirror of
the device front end (chip_stx_parse_device) and the writer of its test and bench inputs.

PARITY UNPINNED: no JVM output exists here.  These tests pin the restatement's own rules: write -> read
round trips for every list class and chunk-spanning component, the OutputChunked placement rules
(1024-byte chunks, a primitive never straddles a chunk, nested fields flush the enclosing chunk), the
status each failure class gets, and the uniform-batch filler against the per-transaction writer."""
import numpy as np
import pytest

import cordagen as G
import stx_build as S
from corda_amd import kryo as K


def test_round_trip_of_random_transactions():
    rng = np.random.default_rng(11)
    pool = S.key_pool(rng)
    for _ in range(150):
        groups, salt, sigs, kinds, skind = S.random_valid(rng, pool)
        b = S.blob(groups, salt, sigs, kinds, skind)
        st, g, s, sg = K.stx_parse(b)
        assert st == K.STX_OK
        assert g == [(gi, list(c)) for gi, c in groups]
        assert s == salt
        assert sg == [x.tuple() for x in sigs]


def test_status_classes():
    blobs = S.cases(seed=7, n_valid=20)
    st = [K.stx_parse(b)[0] for b in blobs]
    assert st[:20] == [K.STX_OK] * 20
    tail = st[20:]
    k, i = S.N_KRYO, S.N_KRYO + S.N_NO_SIGS
    assert tail[:k] == [K.STX_KRYO] * k                   # truncations, damaged headers, truncated txBits
    assert tail[k:i] == [K.STX_NO_SIGS]
    assert tail[i:i + S.N_INVARIANT] == [K.STX_INVARIANT] * S.N_INVARIANT   # each deserialisation check
    assert tail[i + S.N_INVARIANT:] == [K.STX_UNSUPPORTED] * (len(tail) - i - S.N_INVARIANT)
    assert len(tail) - i - S.N_INVARIANT >= 15            # outside the grammar, incl. 7 rejected class ids


def test_registry_restates_the_registration_order():
    """DefaultKryoCustomizer.kt:77-80 pins 10-13; every later id is the position of a new class in the
    registration order; PublicKeySerializer's classes are the key slots' accepted ids."""
    ids = K.registration_ids()
    reg = K.DEFAULT_REGISTRY
    assert (reg.arrays_aslist, reg.signed_tx, reg.wire_tx, reg.serialized_bytes) == (10, 11, 12, 13)
    assert sorted(ids.values()) == list(range(10, 10 + len(ids)))
    assert reg.public_key == [ids[c] for c in K.PUBLIC_KEY_CLASSES]
    assert ids["net.i2p.crypto.eddsa.EdDSAPublicKey"] == ids["sun.security.ec.ECPublicKeyImpl"] + 1
    assert reg.privacy_salt == ids["net.corda.core.contracts.PrivacySalt"] > max(reg.public_key)
    # a re-registered class keeps its id (Kryo.register on a known class replaces the serializer only)
    again = K.registration_ids(K.REGISTRATION_ORDER + [("java.util.BitSet", "")])
    assert again == ids
    # a deployment's own ids (e.g. one more Guava class) shift every later id; the Registry follows
    shifted = K.Registry(K.registration_ids(K.REGISTRATION_ORDER[:20] + [("x.Extra", "")] + K.REGISTRATION_ORDER[20:]))
    assert shifted.privacy_salt == reg.privacy_salt + 1 and shifted.public_key == [k + 1 for k in reg.public_key]


def test_rejected_class_ids_fail_closed():
    """A class id other than the registry's in the PrivacySalt slot or a key slot: a different serializer
    on the JVM, so the front end hands the transaction to the JVM path."""
    rng = np.random.default_rng(3)
    keys = S.key_pool(rng)
    groups, salt, sigs, _, _ = S.random_valid(rng, keys)
    assert K.stx_parse(S.blob(groups, salt, sigs))[0] == K.STX_OK
    ids = K.registration_ids()
    for sid in (K.DEFAULT_REGISTRY.eddsa_public_key, 14, ids["java.util.BitSet"], K.DEFAULT_REGISTRY.privacy_salt + 1):
        assert K.stx_parse(S.blob(groups, salt, sigs, salt_id=sid))[0] == K.STX_UNSUPPORTED
    for kid in K.DEFAULT_REGISTRY.public_key:
        assert K.stx_parse(S.blob(groups, salt, [K.Sig(sigs[0].sig, sigs[0].key, 1, 4, kid)]))[0] == K.STX_OK
    for kid in (K.DEFAULT_REGISTRY.privacy_salt, ids["net.i2p.crypto.eddsa.EdDSAPrivateKey"], 13, 14):
        assert K.stx_parse(S.blob(groups, salt, [K.Sig(sigs[0].sig, sigs[0].key, 1, 4, kid)]))[0] == K.STX_UNSUPPORTED
    other = K.Registry(K.registration_ids(K.REGISTRATION_ORDER[:20] + [("x.Extra", "")] + K.REGISTRATION_ORDER[20:]))
    assert K.stx_parse(S.blob(groups, salt, sigs), other)[0] == K.STX_UNSUPPORTED


def test_state_ref_inputs_are_canonical():
    rng = np.random.default_rng(5)
    for idx in (0, 1, 63, 64, 8191, 2**31 - 1, -1, -2**31):
        h = rng.bytes(32)
        b = K.state_ref(h, idx)
        assert K.state_ref_of(b) == (h, idx)
    assert K.state_ref_of(S.overlong_stateref(rng)) is None
    good = K.state_ref(rng.bytes(32), 2)
    assert K.state_ref_of(good + b"\0") is None and K.state_ref_of(good[:-1]) is None
    assert K.state_ref_of(rng.bytes(176)) is None


@pytest.mark.parametrize("groups,msg", [
    ([(1, [b"a"]), (2, [])], "Empty component groups are not allowed"),
    ([(1, [b"a"]), (1, [b"b"]), (2, [b"c"])], "Duplicated component groups detected"),
    ([(0, [b"a"]), (1, [b"b"]), (2, [b"c"])], "The notary must be specified explicitly for any transaction that has inputs"),
    ([(0, [b"a", b"a"]), (2, [b"c"]), (4, [b"n"])], "Duplicate input states detected"),
    ([(2, [b"c"]), (4, [b"n"])], "A transaction must contain at least one input or output state"),
    ([(1, [b"o"]), (4, [b"n"])], "A transaction must contain at least one command"),
    ([(1, [b"o"]), (2, [b"c"]), (5, [b"t"])], "Transactions with time-windows must be notarised"),
    ([(0, [b"a"]), (1, [b"o"]), (2, [b"c"]), (4, [b"n"]), (5, [b"t"])], None),
    ([(1, [b"o"]), (2, [b"c"]), (4, [b"n", b"m"])], "Invalid Transaction. More than 1 notary party detected."),
    ([(1, [b"o"]), (2, [b"c"]), (4, [b"n"]), (5, [b"t", b"u"])], "Invalid Transaction. More than 1 time-window detected."),
    ([(1, [b"o"]), (2, []), (4, [b"n", b"m"])], "Invalid Transaction. More than 1 notary party detected."),
])
def test_wire_transaction_invariants(groups, msg):
    assert K.wire_invariant_error(groups) == msg


def test_chunk_placement():
    # a 1500-byte component: ComponentGroup.components is one chunked field; the first chunk is full
    w = K.wire_transaction([(1, [bytes(1500)]), (2, [b"c"])], bytes(32))
    assert b"\x80\x08" in w                                  # varint(1024)
    groups, salt = K.parse_wire_transaction(w)
    assert groups[0][1][0] == bytes(1500)
    # a varint never straddles a chunk: 1023 payload bytes then a 2-byte varint -> flush at 1023
    o = K.Out()
    c = K.Out(o)
    c.write_bytes(bytes(1023))
    c.write_varint(300)
    c.end_chunks()
    assert o.getvalue() == b"\xff\x07" + bytes(1023) + b"\x02\xac\x02\x00"
    # nested CompatibleFieldSerializer: every inner chunk flushes the enclosing field's chunk
    s = K.signed_transaction(K.wire_transaction([(1, [b"o"]), (2, [b"c"])], bytes(32)),
                             [K.Sig(bytes(64), bytes(44), 1, 4, 31)])
    assert b"\x01\x02\x03\x00\x01\x08\x01\x00\x00" in s       # ...01 02 | 00 01 08 | 00 | end


def test_uniform_filler_equals_writer():
    tb, tm, sb, ids, _v, _a = G.cfg4_workload_commands(24, n_keys=8, seed=0x5EED0204, threads=4)
    data, off, ln = G.stx_uniform(tb, sb, 2)
    for t in range(24):
        b = data[int(off[t]):int(off[t]) + int(ln[t])].tobytes()
        assert b == G.stx_signed_tx(tb, sb, t, range(2 * t, 2 * t + 2))
        st, groups, salt, sigs = K.stx_parse(b)
        assert st == K.STX_OK and salt == tb.salts[32 * t:32 * t + 32].tobytes()
        assert [len(c) for _, cs in groups for c in cs][:2] == [176, 176]
        assert all(K.state_ref_of(c) for gi, cs in groups if gi == 0 for c in cs)


def test_device_name_tables_match_the_restatement():
    """The class / field names and lengths the device grammar compares against (kryo.hip constant tables)
    are the restatement's (kryo.py)."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "corda_amd", "csrc", "kryo.hip")).read()

    def table(arr, lens):
        body = src[src.index("__constant__ char %s" % arr):]
        names = re.findall(r'"([^"]*)"', body[:body.index("};")])
        lb = src[src.index("__constant__ uint8_t %s" % lens):]
        return names, [int(x) for x in lb[lb.index("{") + 1:lb.index("}")].split(",")]

    names, lens = table("k_names", "k_name_len")
    assert names == [K.ARRAY_LIST, K.SINGLETON_LIST, K.TRANSACTION_SIGNATURE, K.COMPONENT_GROUP, K.COMMAND, K.PARTY]
    assert lens == [len(x) for x in names]
    fields, flens = table("k_fields", "k_field_len")
    assert fields == K.TXSIG_FIELDS + K.META_FIELDS + K.GROUP_FIELDS + K.COMMAND_FIELDS + K.PARTY_FIELDS
    assert flens == [len(x) for x in fields]
