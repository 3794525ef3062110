"""Seeded chip_req_batch workloads for the required-signer tests (test infrastructure).

A batch of `ntx` transactions over a key pool of `n_keys` SPKIs (optionally with byte-identical
duplicate entries, i.e. a pool that is not de-duplicated), each transaction with a few signatures
(random statuses, mostly VALID) and a few required keys: plain keys, CHIP_REQ_NO_SIGNER leaves, and
CompositeKey trees (nested, weighted, random thresholds) flattened in post-order.  `malformed=True`
adds transactions whose ranges / trees / key indices are invalid."""
import numpy as np

NO_SIGNER = 0xFFFFFFFF


class Obj:
    pass


def _tree(rng, n_keys, depth, val, nk, w, weight):
    """Append one random key tree in post-order; returns nothing (arrays grow in place)."""
    if depth > 0 and rng.random() < 0.5:
        kids = int(rng.integers(2, 5))
        total = 0
        for _ in range(kids):
            cw = int(rng.integers(1, 4))
            total += cw
            _tree(rng, n_keys, depth - 1, val, nk, w, cw)
        val.append(int(rng.integers(1, total + 1)))
        nk.append(kids)
    else:
        val.append(NO_SIGNER if rng.random() < 0.05 else int(rng.integers(0, n_keys)))
        nk.append(0)
    w.append(weight)


def make(ntx=2000, n_keys=64, dup_keys=8, seed=1, max_sigs=4, max_req=3, depth=3, p_bad_sig=0.03,
         malformed=False, with_tx_idx=False):
    rng = np.random.Generator(np.random.PCG64(seed))
    # key pool: n_keys distinct 44-byte Ed25519-shaped SPKIs + dup_keys byte-identical copies
    prefix = bytes.fromhex("302a300506032b6570032100")
    base = [prefix + rng.bytes(32) for _ in range(n_keys)]
    pool = base + [base[int(rng.integers(0, n_keys))] for _ in range(dup_keys)]
    nk_all = len(pool)
    key_len = np.full(nk_all, 44, dtype=np.uint32)
    key_off = np.arange(nk_all, dtype=np.uint64) * 44
    key_data = np.frombuffer(b"".join(pool), dtype=np.uint8).copy()
    sig_start, req_start, node_start = [0], [0], [0]
    key_idx, tx_idx, val, nk, w, allowed = [], [], [], [], [], []
    for t in range(ntx):
        ns = int(rng.integers(0, max_sigs + 1))
        for _ in range(ns):
            key_idx.append(int(rng.integers(0, nk_all)))
            tx_idx.append(t)
        sig_start.append(len(key_idx))
        nr = int(rng.integers(0, max_req + 1))
        for _ in range(nr):
            _tree(rng, nk_all, depth, val, nk, w, 1)
            node_start.append(len(val))
            allowed.append(1 if rng.random() < 0.1 else 0)
        req_start.append(len(allowed))
    n = len(key_idx)
    status = np.where(rng.random(n) < p_bad_sig, rng.integers(1, 7, size=n), 0).astype(np.uint8)
    q = Obj()
    q.ntx = ntx
    q.sig_start = np.array(sig_start, dtype=np.uint64)
    q.req_start = np.array(req_start, dtype=np.uint64)
    q.node_start = np.array(node_start, dtype=np.uint64)
    q.allowed = np.array(allowed or [0], dtype=np.uint8)[:len(allowed)] if allowed else np.zeros(0, np.uint8)
    q.node_val = np.array(val, dtype=np.uint32)
    q.node_nkids = np.array(nk, dtype=np.uint32)
    q.node_weight = np.array(w, dtype=np.uint32)
    b = Obj()
    b.key_idx = np.array(key_idx or [0], dtype=np.uint32)[:n] if n else np.zeros(0, np.uint32)
    b.msg_idx = np.zeros(n, dtype=np.uint32)
    b.sig_data = np.zeros(max(n, 1) * 64, dtype=np.uint8)
    b.sig_off = np.arange(n, dtype=np.uint64) * 64
    b.sig_len = np.full(n, 64, dtype=np.uint32)
    b.key_data, b.key_off, b.key_len = key_data, key_off, key_len
    b.msg_data = np.zeros(16, dtype=np.uint8)
    b.msg_off = np.zeros(1, dtype=np.uint64)
    b.msg_len = np.zeros(1, dtype=np.uint32)
    tx_idx = np.array(tx_idx, dtype=np.uint32)
    if malformed:
        _corrupt(rng, q, b, tx_idx, nk_all)
    return q, b, status, tx_idx


def _corrupt(rng, q, b, tx_idx, nk_all):
    """Invalidate a few transactions in every way the contract names."""
    ntx = q.ntx
    picks = rng.choice(ntx, size=min(ntx, 60), replace=False)
    for i, t in enumerate(picks):
        kind = i % 6
        r0, r1 = int(q.req_start[t]), int(q.req_start[t + 1])
        s0, s1 = int(q.sig_start[t]), int(q.sig_start[t + 1])
        if kind == 0 and r1 > r0:                       # leaf key index past the pool
            a, bb = int(q.node_start[r0]), int(q.node_start[r0 + 1])
            leaves = [j for j in range(a, bb) if q.node_nkids[j] == 0]
            q.node_val[leaves[0]] = nk_all + 5
        elif kind == 1 and r1 > r0:                      # composite claiming more children than precede it
            a, bb = int(q.node_start[r0]), int(q.node_start[r0 + 1])
            q.node_nkids[bb - 1] = (bb - a) + 1
        elif kind == 2 and r1 > r0:                      # two trees in one required-key range
            a, bb = int(q.node_start[r0]), int(q.node_start[r0 + 1])
            if bb - a >= 3 and q.node_nkids[bb - 1] > 0:
                q.node_nkids[bb - 1] -= 1 if q.node_nkids[bb - 1] > 1 else 0
        elif kind == 3 and s1 > s0:                      # signature owned by another transaction
            tx_idx[s0] = (t + 1) % ntx
        elif kind == 4 and s1 > s0:                      # signature key index past the pool
            b.key_idx[s0] = nk_all + 1
        elif kind == 5 and r1 > r0:                      # empty node range
            pass
