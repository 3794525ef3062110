"""SignedTransaction blobs for the Kryo front-end tests (chip_stx_parse_device vs corda_amd/kryo.py).

Every case is built with the kryo.py writer (the Kryo 4.0.0 restatement, parity unpinned) and labelled
with the status the host mirror kryo.stx_parse gives; the cases cover each status class the device
reports: valid transactions of random shapes (chunk-spanning components, unknown group ordinals 20 /
63, every list class, several key classes and metadata values), truncations and header damage
(KryoException), empty signature lists, each WireTransaction.init invariant, and well-formed bytes
outside the device grammar (class names for keys, object back-references, group index 64, > 64 inputs,
renamed fields)."""
import numpy as np

from corda_amd import kryo as K

ED_KEY = 44
EC_KEYS = (91, 88)
METAS = [(1, 4), (1, 3), (1, 2), (2, 4)]


def _key(rng, n):
    return bytes([0x30]) + rng.bytes(n - 1)


def random_valid(rng, key_pool):
    """(groups, salt, sigs, list kinds) of one structurally valid transaction."""
    groups = []
    if rng.random() < 0.8:
        groups.append((0, [rng.bytes(int(rng.integers(36, 120))) for _ in range(int(rng.integers(1, 4)))]))
    if rng.random() < 0.8 or not groups:
        groups.append((1, [rng.bytes(int(rng.integers(0, 1600))) for _ in range(int(rng.integers(1, 4)))]))
    groups.append((2, [rng.bytes(int(rng.integers(20, 300))) for _ in range(int(rng.integers(1, 3)))]))
    if rng.random() < 0.5:
        groups.append((3, [rng.bytes(34) for _ in range(int(rng.integers(1, 3)))]))
    if groups[0][0] == 0 or rng.random() < 0.5:
        groups.append((4, [rng.bytes(int(rng.integers(60, 400)))]))
        if rng.random() < 0.5:
            groups.append((5, [rng.bytes(40)]))
    if rng.random() < 0.15:
        groups.append((int(rng.choice([20, 63])), [rng.bytes(int(rng.integers(1, 50)))]))
    order = list(range(len(groups)))
    if rng.random() < 0.2:
        rng.shuffle(order)                       # group order is the writer's list order
    groups = [groups[i] for i in order]
    sigs = []
    for _ in range(int(rng.integers(1, 5))):
        key = key_pool[int(rng.integers(0, len(key_pool)))]
        sl = 64 if len(key) == ED_KEY else int(rng.integers(70, 73))
        pv, sch = METAS[int(rng.integers(0, len(METAS)))]
        sigs.append(K.Sig(rng.bytes(sl), key, pv, sch, int(rng.integers(14, 60))))
    kinds = {}
    r = rng.random()
    if r < 0.2:
        kinds[-1] = ("aslist", K.COMPONENT_GROUP)
    for gi, comps in groups:
        if rng.random() < 0.2:
            kinds[gi] = ("aslist", K.REG_SERIALIZED_BYTES)
        elif rng.random() < 0.2:
            kinds[gi] = "array"
    if len(sigs) == 1:
        skind = "single" if rng.random() < 0.7 else "array"
    else:
        skind = ("aslist", K.TRANSACTION_SIGNATURE) if rng.random() < 0.3 else "array"
    return groups, rng.bytes(32), sigs, kinds, skind


def blob(groups, salt, sigs, kinds=None, skind="auto"):
    return K.signed_transaction(K.wire_transaction(groups, salt, K.DEFAULT_IDS["privacy_salt"], kinds), sigs, skind)


def _replace_once(b: bytes, old: bytes, new: bytes) -> bytes:
    i = b.index(old)
    return b[:i] + new + b[i + len(old):]


def cases(seed: int = 7, n_valid: int = 200):
    """-> list of blobs (bytes); labels come from K.stx_parse."""
    rng = np.random.default_rng(seed)
    key_pool = [_key(rng, ED_KEY) for _ in range(12)] + [_key(rng, n) for n in EC_KEYS for _ in range(3)]
    out = []
    valid = [random_valid(rng, key_pool) for _ in range(n_valid)]
    out += [blob(*v) for v in valid]
    g0, s0, sg0, _, _ = valid[0]
    ok = blob(g0, s0, sg0)
    # KryoException: truncations of the outer bytes and of txBits, damaged headers
    for cut in (3, 8, 12, 40, len(ok) // 3, len(ok) // 2, len(ok) - 40, len(ok) - 1):
        out.append(ok[:cut])
    out.append(b"cordb" + ok[5:])
    w = K.wire_transaction(g0, s0)
    out.append(K.signed_transaction(b"corda\x00\x00\x02" + w[8:], sg0))
    out.append(K.signed_transaction(w[:len(w) // 2], sg0))
    out.append(K.signed_transaction(w[:-1], sg0))
    # SignedTransaction.init: no signatures
    out.append(K.signed_transaction(w, [], "array"))
    # WireTransaction.init invariants
    c = lambda n=40: rng.bytes(n)
    inv = [
        [(1, [c()]), (2, []), (4, [c()])],                                   # empty group
        [(1, [c()]), (2, [c()]), (1, [c()])],                                # duplicated group
        [(0, [c()]), (1, [c()]), (2, [c()])],                                # inputs without notary
        [(2, [c()]), (4, [c()])],                                            # no input or output
        [(1, [c()]), (4, [c()])],                                            # no command
        [(1, [c()]), (2, [c()]), (5, [c()])],                                # time-window without notary
        [(0, [b"x" * 36, b"y" * 36, b"x" * 36]), (1, [c()]), (2, [c()]), (4, [c()])],   # duplicate inputs
    ]
    out += [blob(g, c(32), sg0) for g in inv]
    # outside the device grammar (UNSUPPORTED: the JVM path decides)
    out.append(blob([(0, [c(36 + i % 3) for i in range(65)]), (2, [c()]), (4, [c()])], c(32), sg0))   # > 64 inputs
    out.append(blob([(1, [c()]), (2, [c()]), (64, [c()])], c(32), sg0))                                # group 64
    out.append(blob(g0, s0, [K.Sig(sg0[0].sig, sg0[0].key, 1, 4, "net.i2p.crypto.eddsa.EdDSAPublicKey")]))  # by name
    out.append(_replace_once(ok, b"\x0f\x01", b"\x0f\x02"))                 # txBits as a back-reference
    out.append(ok.replace(b"TransactionSignature.b\xf9", b"TransactionSignature.x\xf9", 1))   # renamed field
    out.append(ok.replace(b"java.util.ArrayLis\xf4", b"java.util.LinkedLis\xf4", 1)
               if b"java.util.ArrayLis\xf4" in ok else ok.replace(b"java.util.Collections$SingletonLis\xf4",
                                                                     b"java.util.Collections$SingletonSe\xf4", 1))
    return out


def cases_required(seed: int = 13, n: int = 240):
    """SignedTransactions whose command / notary components are real Kryo Command / Party objects:
    requiredSigningKeys = commands' signers (several commands, repeated and non-signing keys, every list
    class) + the notary when there are inputs or a time-window; plus a CompositeKey signer, a malformed
    command and a command of another class (-> UNSUPPORTED)."""
    from corda_amd import composite as CK
    rng = np.random.default_rng(seed)
    pool = [_key(rng, ED_KEY) for _ in range(10)] + [_key(rng, 91), _key(rng, 88)]
    comp = CK.CompositeKey.Builder().add_keys(pool[0], pool[1]).build(1).encoded \
        if hasattr(CK.CompositeKey, "Builder") else None
    out = []
    for i in range(n):
        signers_of_cmds = [[pool[int(rng.integers(0, len(pool)))] for _ in range(int(rng.integers(1, 4)))]
                           for _ in range(int(rng.integers(1, 3)))]
        notary_key = pool[int(rng.integers(0, len(pool)))]
        kind = rng.random()
        groups = []
        has_in = rng.random() < 0.6
        if has_in:
            groups.append((0, [rng.bytes(40) + bytes([j]) for j in range(int(rng.integers(1, 3)))]))
        groups.append((1, [rng.bytes(int(rng.integers(20, 900)))]))
        cmds = []
        for ss in signers_of_cmds:
            lk = "auto" if len(ss) == 1 else ("aslist", 31) if rng.random() < 0.3 else "array"
            cmds.append(K.command(ss, list_kind=lk if lk[0] != "aslist" else ("aslist", K.DEFAULT_IDS["eddsa_public_key"])))
        if kind < 0.03 and comp is not None:
            cmds.append(K.command([comp]))                                 # CompositeKey signer
        elif kind < 0.06:
            cmds.append(K.command(signers_of_cmds[0])[:40])                 # truncated inside the signers
        elif kind < 0.08:
            cmds[0] = cmds[0].replace(b"net.corda.core.contracts.Comman\xe4", b"net.corda.core.contracts.Commanx\xe4", 1)
        groups.append((2, cmds))
        if has_in or rng.random() < 0.5:
            groups.append((4, [K.party(notary_key)]))
            if rng.random() < 0.3:
                groups.append((5, [rng.bytes(40)]))
        if i % 97 == 5:                                                     # > 64 signer entries
            cmds.append(K.command([pool[j % len(pool)] for j in range(70)], list_kind="array"))
        req_all = [k for ss in signers_of_cmds for k in ss] + [notary_key]
        sig_keys = [req_all[int(rng.integers(0, len(req_all)))] for _ in range(int(rng.integers(1, 4)))]
        sigs = [K.Sig(rng.bytes(64) if len(k) == ED_KEY else rng.bytes(71), k, 1, 4, 31) for k in sig_keys]
        out.append(blob(groups, rng.bytes(32), sigs))
    return out


def expected_required(blobs):
    """Host mirror of chip_stx_parse_device(..., CHIP_STX_REQUIRED): per blob (status, [required key
    bytes]) and the signer key numbering (first occurrence over the signatures of the transactions the
    parse passes accepted, before the required-key stage)."""
    from corda_amd import composite as CK
    parsed = [K.stx_parse(b) for b in blobs]
    kid = {}
    for st, g, salt, sigs in parsed:
        if st == K.STX_OK:
            for sig, key, pv, sch in sigs:
                kid.setdefault(key, len(kid))
    out = []
    for st, g, salt, sigs in parsed:
        if st != K.STX_OK:
            out.append((st, None))
            continue
        try:
            req = K.required_signing_keys(g)
            present = {gi for gi, _ in g}
            entries = sum(len(K.command_signers(c)) for gi, cs in g if gi == K.GROUP_COMMANDS for c in cs) + \
                (1 if K.GROUP_NOTARY in present and (K.GROUP_INPUTS in present or K.GROUP_TIMEWINDOW in present) else 0)
        except K.KryoException:
            out.append((K.STX_UNSUPPORTED, None))
            continue
        if entries > 64:                         # the device's duplicate check covers <= 64 signer entries
            out.append((K.STX_UNSUPPORTED, None))
            continue
        if any(k not in kid and CK._spki_oid(k) == CK._COMPOSITE_OID_TLV for k in req):
            out.append((K.STX_UNSUPPORTED, None))
            continue
        out.append((K.STX_OK, req))
    return out, kid
