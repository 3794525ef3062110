"""GPU: the Kryo front end (chip_stx_parse_device, kryo.hip) against the oracle (oracle/kryo_ref.c, an
independent de-chunking restatement) and the host mirror (corda_amd/kryo.py).

PARITY UNPINNED for the bytes themselves (no JVM output exists here: kryo.py restates Kryo 4.0.0); what
these tests pin is that the device parse of every SignedTransaction equals the oracle's — statuses
for each failure class, components (group, internal index, bytes), salts, signatures, signer keys,
metadata -> template mapping, the first-occurrence key numbering — and that verifying a batch from its
bytes gives the same ids, signature statuses and required-signer verdicts as the structured batch."""
import numpy as np
import pytest
import torch

import cordagen as G
import oracle_bind as O
import stx_build as S
from corda_amd import kryo as K
from corda_amd import native

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
METAS = np.array(S.METAS[:3], dtype=np.int32)     # (2, 4) maps to no template


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def parse(ctx, blobs):
    data, off, ln = G.stx_blobs_from_lists(blobs)
    if len(data) == 0:
        data = np.zeros(1, np.uint8)
    dd, doff, dlen = _dev(data), _dev(off), _dev(ln)
    st = torch.zeros(len(blobs), dtype=torch.uint8, device=DEV)
    p = ctx.stx_parse_device(dd, doff, dlen, len(data), METAS, st)
    torch.cuda.synchronize()
    return p, st.cpu().numpy(), (dd, doff, dlen)


def host(ctx, p, n):
    t, s = p.txs, p.sigs
    r = {"cstart": ctx.copy_to_host(t.tx_comp_start, n + 1, np.uint64),
         "sstart": ctx.copy_to_host(p.sig_start, n + 1, np.uint64),
         "salts": ctx.copy_to_host(t.salts, 32 * n, np.uint8).reshape(n, 32),
         "group": ctx.copy_to_host(t.comp_group, t.ncomp, np.uint32),
         "internal": ctx.copy_to_host(t.comp_internal, t.ncomp, np.uint32),
         "coff": ctx.copy_to_host(t.comp_off, t.ncomp, np.uint64),
         "clen": ctx.copy_to_host(t.comp_len, t.ncomp, np.uint32),
         "pool": ctx.copy_to_host(t.data, t.data_bytes, np.uint8),
         "tx_idx": ctx.copy_to_host(s.tx_idx, s.n, np.uint32),
         "tmpl": ctx.copy_to_host(s.tmpl_idx, s.n, np.uint32),
         "kidx": ctx.copy_to_host(s.key_idx, s.n, np.uint32),
         "soff": ctx.copy_to_host(s.sig_off, s.n, np.uint64),
         "slen": ctx.copy_to_host(s.sig_len, s.n, np.uint32),
         "koff": ctx.copy_to_host(s.key_off, s.n_keys, np.uint64),
         "klen": ctx.copy_to_host(s.key_len, s.n_keys, np.uint32)}
    return r


def test_parse_equals_host_mirror(ctx):
    blobs = S.cases(seed=7, n_valid=300)
    p, st, _keep = parse(ctx, blobs)
    n = len(blobs)
    want = [K.stx_parse(b) for b in blobs]
    assert list(st) == [w[0] for w in want]
    assert set(st) == {0, 1, 2, 3, 4}                   # every status class is exercised
    h = host(ctx, p, n)
    pool = h["pool"]
    keys_seen = {}
    for t, (status, groups, salt, sigs) in enumerate(want):
        c0, c1 = int(h["cstart"][t]), int(h["cstart"][t + 1])
        s0, s1 = int(h["sstart"][t]), int(h["sstart"][t + 1])
        if status != K.STX_OK:
            dup_only = status == K.STX_INVARIANT and K.wire_invariant_error(
                K.parse_wire_transaction(K.parse_signed_transaction(blobs[t])[0])[0], check_duplicates=False) is None
            assert dup_only or (c0 == c1 and s0 == s1), t
            continue
        comps = [(gi, i, c) for gi, cs in groups for i, c in enumerate(cs)]
        assert c1 - c0 == len(comps), t
        for k, (gi, i, c) in enumerate(comps):
            o, ln = int(h["coff"][c0 + k]), int(h["clen"][c0 + k])
            assert (int(h["group"][c0 + k]), int(h["internal"][c0 + k])) == (gi, i), (t, k)
            assert pool[o:o + ln].tobytes() == c, (t, k)
        assert h["salts"][t].tobytes() == salt
        assert s1 - s0 == len(sigs), t
        for j, (sig, key, pv, sch) in enumerate(sigs):
            i = s0 + j
            o, ln = int(h["soff"][i]), int(h["slen"][i])
            assert pool[o:o + ln].tobytes() == sig, (t, j)
            assert int(h["tx_idx"][i]) == t
            m = [k for k in range(len(METAS)) if tuple(METAS[k]) == (pv, sch)]
            assert int(h["tmpl"][i]) == (m[0] if m else 0xFFFFFFFF)
            kid = keys_seen.setdefault(key, len(keys_seen))          # first-occurrence numbering
            assert int(h["kidx"][i]) == kid, (t, j)
            ko, kl = int(h["koff"][kid]), int(h["klen"][kid])
            assert pool[ko:ko + kl].tobytes() == key
    assert p.sigs.n_keys == len(keys_seen)


def test_empty_and_single_blob(ctx):
    p, st, _ = parse(ctx, [])
    assert p.txs.ntx == 0 and p.sigs.n == 0
    blobs = S.cases(seed=3, n_valid=1)[:1]
    p, st, _ = parse(ctx, blobs)
    assert list(st) == [K.stx_parse(blobs[0])[0]] == [0]


def test_verify_from_bytes_equals_structured_path(ctx):
    """cfg4-shaped batch: ids, signature statuses and required-signer verdicts from the parsed bytes
    equal those of the structured batch (chip_verify_signed_tx_batch_device on host-built arrays)."""
    ntx = 2000
    # inputs must be canonical StateRefs for the front end: the Command / Party variant of the cfg4 shape
    tb, tm, sb, ids_ref, _v, _a = G.cfg4_workload_commands(ntx, n_keys=64, seed=0x5EED0104, threads=8)
    q = G.cfg4_required(sb, ntx, 64, seed=0x5EED0106)
    data, off, ln = G.stx_uniform(tb, sb, 2)
    dd, doff, dlen = _dev(data), _dev(off), _dev(ln)
    st = torch.zeros(ntx, dtype=torch.uint8, device=DEV)
    p = ctx.stx_parse_device(dd, doff, dlen, len(data), np.array([[1, 4]], np.int32), st)
    assert int((st != 0).sum()) == 0
    q2 = G.required_for_parsed(q, sb)
    # structured reference
    ids, status, verdict, arg, missing = ctx.verify_signed_tx_batch(tb, tm, sb, q)
    dev = {k: _dev(getattr(q2, k)) for k in ("sig_start", "req_start", "node_start", "allowed", "node_val",
                                               "node_nkids", "node_weight") if getattr(q2, k) is not None}
    dq2 = G.ReqBatch()
    dq2.ntx = ntx
    for k in ("sig_start", "req_start", "node_start", "allowed", "node_val", "node_nkids", "node_weight"):
        setattr(dq2, k, dev.get(k))
    dq2.nreq, dq2.n_nodes = len(q.node_start) - 1, len(q.node_val)
    dtm = G.Templates()
    dtm.data, dtm.off, dtm.len, dtm.id_at, dtm.max_len = _dev(tm.data), _dev(tm.off), _dev(tm.len), _dev(tm.id_at), tm.max_len
    d_ids = torch.zeros(ntx * 32, dtype=torch.uint8, device=DEV)
    d_status = torch.zeros(sb.n, dtype=torch.uint8, device=DEV)
    d_verdict = torch.zeros(ntx, dtype=torch.uint8, device=DEV)
    d_arg = torch.zeros(ntx, dtype=torch.int32, device=DEV)
    d_missing = torch.zeros(max(dq2.nreq, 1), dtype=torch.uint8, device=DEV)
    ctx.verify_signed_tx_parsed_device(p, dtm, dq2, d_ids, d_status, d_verdict, d_arg, d_missing)
    torch.cuda.synchronize()
    assert np.array_equal(d_ids.cpu().numpy().reshape(ntx, 32), ids)
    assert np.array_equal(ids, ids_ref)
    assert np.array_equal(d_status.cpu().numpy(), status)
    assert np.array_equal(d_verdict.cpu().numpy(), verdict)
    assert np.array_equal(d_arg.cpu().numpy().view(np.uint32), arg)
    assert np.array_equal(d_missing.cpu().numpy()[:dq2.nreq], missing)
    assert int((status == 0).sum()) > 0 and int((verdict != 0).sum()) > 0



def device_records(ctx, blobs, required=False, metas=METAS, in_place=False):
    """chip_stx_parse_device over `blobs` -> one record per blob in the shape of oracle_bind.stx_parse:
    (status, groups, salt, [(sig, key, template index)], required key trees).  A leaf of a tree is its key's
    bytes when the device gave it a signer-pool index (else None: CHIP_REQ_NO_SIGNER)."""
    data, off, ln = G.stx_blobs_from_lists(blobs)
    if len(data) == 0:
        data = np.zeros(1, np.uint8)
    cap = 0
    if in_place:   # room for the de-chunked runs behind the blobs: parsed in place (data_capacity)
        cap = 2 * len(data) + 4096
        dd = torch.zeros(cap, dtype=torch.uint8, device=DEV)
        dd[:len(data)].copy_(torch.from_numpy(np.ascontiguousarray(data)))
    else:
        dd = _dev(data)
    doff, dlen = _dev(off), _dev(ln)
    st = torch.zeros(max(len(blobs), 1), dtype=torch.uint8, device=DEV)
    p = ctx.stx_parse_device(dd, doff, dlen, len(data), metas, st[:len(blobs)], required=required,
                             data_capacity=cap)
    torch.cuda.synchronize()
    n = len(blobs)
    st = st.cpu().numpy()[:n]
    h = host(ctx, p, n)
    pool = h["pool"]
    keys = [pool[int(h["koff"][k]):int(h["koff"][k]) + int(h["klen"][k])].tobytes() for k in range(p.sigs.n_keys)]
    q = p.req
    if required:
        rstart = ctx.copy_to_host(q.req_start, n + 1, np.uint64)
        nstart = ctx.copy_to_host(q.node_start, q.nreq + 1, np.uint64)
        val = ctx.copy_to_host(q.node_val, q.n_nodes, np.uint32)
        nk = ctx.copy_to_host(q.node_nkids, q.n_nodes, np.uint32)
        w = ctx.copy_to_host(q.node_weight, q.n_nodes, np.uint32)
    out = []
    for t in range(n):
        if st[t] != K.STX_OK:
            out.append((int(st[t]), None, None, None, None))
            continue
        c0, c1 = int(h["cstart"][t]), int(h["cstart"][t + 1])
        groups = []
        for k in range(c0, c1):
            o, l = int(h["coff"][k]), int(h["clen"][k])
            c = pool[o:o + l].tobytes()
            if int(h["internal"][k]) == 0:
                groups.append((int(h["group"][k]), [c]))
            else:
                groups[-1][1].append(c)
        s0, s1 = int(h["sstart"][t]), int(h["sstart"][t + 1])
        sigs = []
        for i in range(s0, s1):
            o, l = int(h["soff"][i]), int(h["slen"][i])
            assert int(h["tx_idx"][i]) == t
            sigs.append((pool[o:o + l].tobytes(), keys[int(h["kidx"][i])], int(h["tmpl"][i])))
        trees = None
        if required:
            trees = []
            for r in range(int(rstart[t]), int(rstart[t + 1])):
                tree = []
                for j in range(int(nstart[r]), int(nstart[r + 1])):
                    if nk[j] == 0:
                        tree.append((None if val[j] == G.REQ_NO_SIGNER else keys[int(val[j])], 0, 0, int(w[j])))
                    else:
                        tree.append((None, int(val[j]), int(nk[j]), int(w[j])))
                trees.append(tree)
        out.append((int(st[t]), groups, h["salts"][t].tobytes(), sigs, trees))
    return out, keys


def assert_device_equals_oracle(ctx, blobs, required, reg=K.DEFAULT_REGISTRY, in_place=False):
    """Device records == oracle/kryo_ref.c records for every blob (statuses, components, salts, signatures with
    their template mapping, required-key trees with leaves resolved against the device's signer key pool)."""
    dev, keys = device_records(ctx, blobs, required, in_place=in_place)
    orc = O.stx_parse(blobs, reg, want_required=required)
    pool_keys = set(keys)
    metas = [tuple(m) for m in METAS]
    for t, (d, o) in enumerate(zip(dev, orc)):
        pst, fst, groups, salt, sigs, trees = o
        want = fst if required else pst
        assert d[0] == want, (t, d[0], want)
        if want != K.STX_OK:
            continue
        assert d[1] == groups, t
        assert d[2] == salt, t
        exp_sigs = [(s, k, metas.index((pv, sch)) if (pv, sch) in metas else 0xFFFFFFFF) for s, k, pv, sch in sigs]
        assert d[3] == exp_sigs, t
        if required:
            exp = [[((leaf if leaf in pool_keys else None) if nk == 0 else None, thr, nk, w) for leaf, thr, nk, w in tree]
                   for tree in trees]
            assert d[4] == exp, t
    return dev, orc


def test_required_keys_derived_on_device(ctx):
    """CHIP_STX_REQUIRED: requiredSigningKeys read from the Command / notary Party components on the device
    equal the oracle's (and the host mirror's): per transaction the distinct keys in first-appearance order,
    plain keys as leaves of the signer key pool (or NO_SIGNER), CompositeKeys as their post-order trees;
    UNSUPPORTED for an invalid / non-canonical composite, an undecodable key, a damaged command, an empty
    signers list, > 64 signer entries."""
    blobs = S.cases_required(seed=13, n=300) + S.cases(seed=5, n_valid=40)
    dev, orc = assert_device_equals_oracle(ctx, blobs, required=True)
    want, _ = S.expected_required(blobs)
    assert [d[0] for d in dev] == [w[0] for w in want]
    got = np.array([d[0] for d in dev])
    assert int((got == K.STX_UNSUPPORTED).sum()) >= 20 and int((got == K.STX_OK).sum()) > 250
    assert sum(1 for d in dev if d[0] == 0 and any(len(t) > 1 for t in d[4])) >= 20   # composite trees on device


@pytest.mark.parametrize("required,in_place", [(False, False), (True, False), (True, True)])
def test_device_equals_oracle_on_cases(ctx, required, in_place):
    """in_place: the blobs parsed where they lie (data_capacity), the de-chunked runs written behind them."""
    blobs = S.cases(seed=7, n_valid=200) + S.cases_required(seed=21, n=200)
    dev, _ = assert_device_equals_oracle(ctx, blobs, required, in_place=in_place)
    assert {d[0] for d in dev} == {0, 1, 2, 3, 4}


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_device_equals_oracle_on_damaged_blobs(ctx, seed):
    """Fuzzed blobs (bit flips, byte changes, insertions, deletions, truncations of valid ones), 4 x 12,500
    mutants: the device's status and outputs equal the oracle's for every one, with and without the
    required-key stage (100k device parses in all)."""
    base = S.cases(seed=7 + seed, n_valid=40)[:40] + S.cases_required(seed=13 + seed, n=80)
    blobs = S.mutants(base, seed=seed, n=12_500)
    for required in (False, True):
        assert_device_equals_oracle(ctx, blobs, required)


def dup_input_blobs(seed, n=400):
    """Transactions with 6-40 canonical StateRef inputs (the input group's list field spans several 1024-byte
    chunks, so inputs straddle chunk boundaries and are de-chunked by k_stx_dechunk); every even one has a
    duplicated input at random positions, every odd one distinct inputs."""
    rng = np.random.default_rng(seed)
    keys = S.key_pool(rng)
    out = []
    for i in range(n):
        nin = int(rng.integers(6, 41))
        ins = [S.stateref(rng) for _ in range(nin)]
        if i % 2 == 0:
            a, b = sorted(int(x) for x in rng.choice(nin, 2, replace=False))
            ins[b] = ins[a]
        key = keys[int(rng.integers(0, len(keys)))]
        sig = K.Sig(rng.bytes(64 if len(key) == S.ED_KEY else 71), key, 1, 4, S.REG.key_class_for(key))
        groups = [(0, ins), (1, [rng.bytes(int(rng.integers(20, 700)))]), (2, [K.command([key])]), (4, [K.party(key)])]
        out.append(S.blob(groups, rng.bytes(32), [sig]))
    return out


@pytest.mark.parametrize("required", [False, True])
def test_duplicate_inputs_across_chunk_boundaries(required):
    """checkNoDuplicateInputs (WireTransaction.kt:53-60) over inputs that cross a chunk boundary of the group list
    (pass 2 only records such a run as a copy descriptor, so the comparison must wait for
    k_stx_dechunk): on a fresh context, and again after a batch of other blobs has left its bytes in the pool,
    every duplicate is INVARIANT and every distinct list OK, equal to the oracle and the host mirror."""
    import corda_amd
    c = corda_amd.Context(0)
    try:
        for seed in (0xD0B, 0xD0C):
            blobs = dup_input_blobs(seed)
            dev, _ = assert_device_equals_oracle(c, blobs, required)
            want = [K.stx_parse(b)[0] for b in blobs]
            assert [d[0] for d in dev] == want
            assert want[0::2] == [K.STX_INVARIANT] * (len(blobs) // 2)
            assert want[1::2] == [K.STX_OK] * (len(blobs) // 2)
    finally:
        c.close()


def row_overflow_blobs(seed, n=300):
    """Transactions around the fused walk's row limits (KRYO_LM_C = 16 components, KRYO_LM_S = 4 signatures,
    KRYO_XD = 8 chunk-spanning runs per blob): 1-9 signatures, 2-30 components, 0-12 outputs of 1100-2600 bytes
    (each spans a 1024-byte chunk), signatures and keys of later entries crossing chunk boundaries too."""
    rng = np.random.default_rng(seed)
    keys = S.key_pool(rng)
    out = []
    for i in range(n):
        nin = int(rng.integers(0, 14))
        groups = []
        if nin:
            groups.append((0, [S.stateref(rng) for _ in range(nin)]))
        nbig = int(rng.integers(0, 13)) if i % 3 else int(rng.integers(9, 13))
        outs = [rng.bytes(int(rng.integers(1100, 2600))) for _ in range(nbig)] + \
               [rng.bytes(int(rng.integers(1, 200))) for _ in range(int(rng.integers(0 if nbig else 1, 8)))]
        groups.append((1, outs))
        sigs = []
        for _ in range(int(rng.integers(1, 10)) if i % 4 else int(rng.integers(5, 10))):
            key = keys[int(rng.integers(0, len(keys)))]
            sigs.append(K.Sig(rng.bytes(64 if len(key) == S.ED_KEY else 71), key, 1, 4, S.REG.key_class_for(key)))
        groups.append((2, [K.command([s.key for s in sigs[:3]])]))
        if nin or rng.random() < 0.5:
            groups.append((4, [K.party(sigs[0].key)]))
        out.append(S.blob(groups, rng.bytes(32), sigs))
    return out


@pytest.mark.parametrize("fused", ["2", "1", "0"])
def test_row_overflow_blobs(monkeypatch, fused):
    """Blobs past the fused pass 1's rows (more components, signatures or chunk-spanning runs than it records) are
    re-walked by pass 2; the records of both kinds of blob equal the oracle's, with the fused walk (default) and the
    two-walk front end (CHIP_KRYO_FUSED=0), with and without the required-key stage."""
    import corda_amd
    monkeypatch.setenv("CHIP_KRYO_FUSED", fused)
    c = corda_amd.Context(0)
    try:
        blobs = row_overflow_blobs(0x0F1 + int(fused))
        for required in (False, True):
            dev, _ = assert_device_equals_oracle(c, blobs, required)
            ok = [d for d in dev if d[0] == K.STX_OK]
            assert len(ok) > 250
            assert sum(1 for d in ok if len(d[3]) > 4) > 50 and sum(1 for d in ok if sum(len(g[1]) for g in d[1]) > 16) > 20
    finally:
        c.close()


def test_registry_is_applied(ctx):
    """chip_set_kryo_registry: blobs written with another deployment's ids parse under that registry and fail
    closed (UNSUPPORTED) under the defaults, on the device as in the oracle."""
    ids = K.registration_ids(K.REGISTRATION_ORDER[:20] + [("x.Extra", "")] + K.REGISTRATION_ORDER[20:])
    other = K.Registry(ids)
    rng = np.random.default_rng(4)
    keys = S.key_pool(rng)
    blobs = []
    for _ in range(30):
        groups, salt, sigs, kinds, skind = S.random_valid(rng, keys)
        sigs = [K.Sig(s.sig, s.key, s.platform_version, s.scheme_number_id,
                      other.eddsa_public_key if len(s.key) == 44 else other.bcec_public_key) for s in sigs]
        blobs.append(K.signed_transaction(K.wire_transaction(groups, salt, other.privacy_salt, kinds), sigs, skind))
    assert [d[0] for d in device_records(ctx, blobs)[0]] == [4] * 30
    ctx.set_kryo_registry(other)
    try:
        assert tuple(ctx.kryo_registry().public_key)[:6] == tuple(other.public_key)[:6]
        assert_device_equals_oracle(ctx, blobs, required=False, reg=other)
        assert [d[0] for d in device_records(ctx, blobs)[0]] == [0] * 30
    finally:
        ctx.set_kryo_registry(K.DEFAULT_REGISTRY)
    assert ctx.kryo_registry().privacy_salt == K.DEFAULT_REGISTRY.privacy_salt


def test_verify_from_bytes_with_derived_required_keys(ctx):
    """cfg4 with real Command / Party components: the whole verifySignaturesExcept from the bytes alone
    (ids, SignableData messages, signatures, requiredSigningKeys on the device) gives the labelled
    verdicts: OK, SignatureException at the first corrupted signature, SignaturesMissingException
    when the command names a party that did not sign."""
    ntx = 3000
    tb, tm, sb, ids_ref, verdict, arg = G.cfg4_workload_commands(ntx, n_keys=64, seed=0x5EED0304, threads=8)
    data, off, ln = G.stx_uniform(tb, sb, 2)
    dd, doff, dlen = _dev(data), _dev(off), _dev(ln)
    st = torch.zeros(ntx, dtype=torch.uint8, device=DEV)
    p = ctx.stx_parse_device(dd, doff, dlen, len(data), np.array([[1, 4]], np.int32), st, required=True)
    assert int((st != 0).sum()) == 0
    dtm = G.Templates()
    dtm.data, dtm.off, dtm.len, dtm.id_at, dtm.max_len = _dev(tm.data), _dev(tm.off), _dev(tm.len), _dev(tm.id_at), tm.max_len
    d_ids = torch.zeros(ntx * 32, dtype=torch.uint8, device=DEV)
    d_status = torch.zeros(sb.n, dtype=torch.uint8, device=DEV)
    d_verdict = torch.zeros(ntx, dtype=torch.uint8, device=DEV)
    d_arg = torch.zeros(ntx, dtype=torch.int32, device=DEV)
    d_missing = torch.zeros(max(p.req.nreq, 1), dtype=torch.uint8, device=DEV)
    ctx.verify_signed_tx_parsed_device(p, dtm, None, d_ids, d_status, d_verdict, d_arg, d_missing)
    torch.cuda.synchronize()
    assert np.array_equal(d_ids.cpu().numpy().reshape(ntx, 32), ids_ref)
    assert np.array_equal(d_status.cpu().numpy(), sb.expected)
    assert np.array_equal(d_verdict.cpu().numpy(), verdict)
    assert np.array_equal(d_arg.cpu().numpy().view(np.uint32), arg)
    assert set(np.unique(verdict)) == {0, 1, 2}


def test_host_entry_from_bytes(ctx):
    """chip_stx_verify (what the JNI binding calls): host blobs in, per-tx status / verdict / arg / ids out."""
    ntx = 1500
    tb, tm, sb, ids_ref, verdict, arg = G.cfg4_workload_commands(ntx, n_keys=32, seed=0x5EED0404, threads=8)
    data, off, ln = G.stx_uniform(tb, sb, 2)
    st, v, a, ids = ctx.stx_verify(data, off, ln, tm, [[1, 4]], want_ids=True)
    assert not st.any()
    assert np.array_equal(ids, ids_ref) and np.array_equal(v, verdict) and np.array_equal(a, arg)
    # a damaged blob and an empty batch
    blobs = [data[int(off[t]):int(off[t]) + int(ln[t])].tobytes() for t in range(3)]
    blobs[1] = blobs[1][:100]
    d2, o2, l2 = G.stx_blobs_from_lists(blobs)
    st, v, a, _ = ctx.stx_verify(d2, o2, l2, tm, [[1, 4]])
    assert list(st) == [0, K.STX_KRYO, 0] and v[0] == verdict[0] and v[2] == verdict[2]
    st, v, a, _ = ctx.stx_verify(np.zeros(1, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32), tm, [[1, 4]])
    assert len(st) == 0


@pytest.mark.parametrize("permute", [False, True])
def test_host_entry_chunks_equal_one_chunk(ctx, monkeypatch, permute):
    """chip_stx_verify in transaction chunks (chunk j+1's blobs over PCIe beside chunk j's parse and verify):
    status, verdict, arg and ids equal the one-chunk call and the labels, also with the blobs in shuffled
    pool order (every chunk's byte range then overlaps the others', the copied interval grows both ways);
    a blob outside the pool in a later chunk is CHIP_E_ARG."""
    from corda_amd import native
    ntx = 6000
    tb, tm, sb, ids_ref, verdict, arg = G.cfg4_workload_commands(ntx, n_keys=32, seed=0x5EED0704, threads=8)
    data, off, ln = G.stx_uniform(tb, sb, 2)
    if permute:
        p = np.random.Generator(np.random.PCG64(7)).permutation(ntx)
        # a SIGNATURE verdict's arg indexes the batch's signature list, which the permutation reorders
        cnt = np.bincount(sb.tx_idx, minlength=ntx).astype(np.int64)
        base = np.concatenate([[0], np.cumsum(cnt)])[:-1]
        pbase = np.concatenate([[0], np.cumsum(cnt[p])])[:-1]
        sig = verdict[p] == native.TXV_SIGNATURE
        arg = arg[p].astype(np.int64)
        arg[sig] += pbase[sig] - base[p][sig]
        off, ln, ids_ref, verdict, arg = off[p].copy(), ln[p].copy(), ids_ref[p], verdict[p], arg.astype(np.uint32)
    monkeypatch.setenv("CHIP_STX_CHUNKS", "1")
    st1, v1, a1, i1 = ctx.stx_verify(data, off, ln, tm, [[1, 4]], want_ids=True)
    assert not st1.any() and np.array_equal(i1, ids_ref) and np.array_equal(v1, verdict) and np.array_equal(a1, arg)
    for k in (3, 5):
        monkeypatch.setenv("CHIP_STX_CHUNKS", str(k))
        st, v, a, ids = ctx.stx_verify(data, off, ln, tm, [[1, 4]], want_ids=True)
        assert np.array_equal(st, st1) and np.array_equal(v, v1) and np.array_equal(a, a1) and np.array_equal(ids, i1), k
    bad = off.copy()
    bad[-2] = len(data) - 3
    monkeypatch.setenv("CHIP_STX_CHUNKS", "4")
    with pytest.raises(native.ChipError) as e:
        ctx.stx_verify(data, bad, ln, tm, [[1, 4]])
    assert "outside" in str(e.value)
    st, v, a, _ = ctx.stx_verify(data, off, ln, tm, [[1, 4]])
    assert np.array_equal(v, v1)


def test_two_buffer_sets_alternate(ctx):
    """The outputs of a parse stay valid across the next parse (two buffer sets): batch A is parsed,
    then batch B (on another stream), and A's parsed batch still verifies to A's labels."""
    ta = G.cfg4_workload_commands(700, n_keys=16, seed=0x5EED0504, threads=8)
    tb_ = G.cfg4_workload_commands(900, n_keys=16, seed=0x5EED0604, threads=8)
    parsed = []
    keep = []
    other = torch.cuda.Stream(DEV)
    for i, (tbx, tmx, sbx, idsx, vx, ax) in enumerate((ta, tb_)):
        data, off, ln = G.stx_uniform(tbx, sbx, 2)
        dd, doff, dlen = _dev(data), _dev(off), _dev(ln)
        st = torch.zeros(tbx.ntx, dtype=torch.uint8, device=DEV)
        p = ctx.stx_parse_device(dd, doff, dlen, len(data), np.array([[1, 4]], np.int32), st, required=True,
                                 stream=other.cuda_stream if i else None)
        parsed.append(p)
        keep.append((dd, doff, dlen, st))
    tbx, tmx, sbx, idsx, vx, ax = ta
    p = parsed[0]
    dtm = G.Templates()
    dtm.data, dtm.off, dtm.len, dtm.id_at, dtm.max_len = _dev(tmx.data), _dev(tmx.off), _dev(tmx.len), _dev(tmx.id_at), tmx.max_len
    d_ids = torch.zeros(tbx.ntx * 32, dtype=torch.uint8, device=DEV)
    d_status = torch.zeros(sbx.n, dtype=torch.uint8, device=DEV)
    d_verdict = torch.zeros(tbx.ntx, dtype=torch.uint8, device=DEV)
    d_arg = torch.zeros(tbx.ntx, dtype=torch.int32, device=DEV)
    d_missing = torch.zeros(max(p.req.nreq, 1), dtype=torch.uint8, device=DEV)
    ctx.verify_signed_tx_parsed_device(p, dtm, None, d_ids, d_status, d_verdict, d_arg, d_missing)
    torch.cuda.synchronize()
    assert np.array_equal(d_ids.cpu().numpy().reshape(-1, 32), idsx)
    assert np.array_equal(d_verdict.cpu().numpy(), vx) and np.array_equal(d_arg.cpu().numpy().view(np.uint32), ax)
