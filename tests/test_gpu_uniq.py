"""GPU parity: notary uniqueness (K4) vs the oracle restatement of PersistentUniquenessProvider.commit
+ TrustedAuthorityNotaryService.commitInputStates, and the reference's own scenarios."""
import ctypes
import hashlib

import numpy as np
import pytest

import cordagen as G
import golden_cases

pytestmark = pytest.mark.gpu

COMMITTED, IDEMPOTENT, CONFLICT = 0, 1, 2


@pytest.fixture(autouse=True, params=["0", "1"], ids=["claim", "intern"])
def lookup_mode(request, monkeypatch):
    """Every test under both lookups (read at chip_uniq_open): the claim CAS on the table line (CHIP_UNIQ_INTERN=0)
    and the read-only walk + batch intern table with the slot claimed at insert (CHIP_UNIQ_INTERN=1)."""
    monkeypatch.setenv("CHIP_UNIQ_INTERN", request.param)
    return request.param


def h(s):
    return hashlib.sha256(s.encode()).digest()


def run_both(ctx, oracle, pre, batches, cap=1 << 12):
    t = ctx.uniq_open(cap)
    o = oracle.Uniq(cap)
    if pre is not None:
        t.rebuild(*pre)
        o.preload(*pre)
    outs = []
    for b in batches:
        g = t.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
        r = o.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
        outs.append((g, r))
    assert t.size() == o.size()
    t.close()
    return outs


def test_uniq_golden_scenarios(ctx, oracle):
    for case in golden_cases.uniq_cases():
        batches = [G.uniq_batch_from_lists([(bytes.fromhex(tx), [bytes.fromhex(s) for s in ins], c)
                                            for tx, ins, c in bt]) for bt in case["batches"]]
        outs = run_both(ctx, oracle, None, batches)
        for (g, r), want in zip(outs, case["expected"]):
            assert g[0].tolist() == want, case["label"]
            assert g[0].tolist() == r[0].tolist(), case["label"]
            assert g[1] == r[1], case["label"]


def test_uniq_random_cfg5_shape_matches_oracle(ctx, oracle):
    pre, b = G.uniq_workload(20000, 30000, seed=7, pre_hit=0.02, dbl=0.02, resubmit=0.01)
    (g, r), = run_both(ctx, oracle, pre, [b], cap=1 << 16)
    assert np.array_equal(g[0], r[0])
    assert g[1] == r[1]
    assert (g[0] == CONFLICT).sum() > 0 and (g[0] == IDEMPOTENT).sum() > 0


def test_uniq_multi_batch_and_growth(ctx, oracle):
    batches = []
    pre, b0 = G.uniq_workload(5000, 1000, seed=1, pre_hit=0.05, dbl=0.05)
    batches.append(b0)
    for s in range(2, 5):   # later batches re-spend earlier batches' inputs
        _, bs = G.uniq_workload(5000, 0, seed=s, pre_hit=0.0, dbl=0.03)
        k = 2000
        bs.refs[:36 * k] = b0.refs[:36 * k]
        batches.append(bs)
    outs = run_both(ctx, oracle, pre, batches, cap=1024)   # forces rehash growth
    for g, r in outs:
        assert np.array_equal(g[0], r[0])
        assert g[1] == r[1]


def test_uniq_failed_inputs_then_consumed(ctx, oracle):
    """Inputs of failed txs are claimed in the batch but never consumed: their slots stay empty or are
    written back dead (when another key's probe walked past the claim).  Later batches consume those
    states, and new keys probe through the dead slots, at a load factor kept near 1/2: statuses,
    records and the live size equal the oracle after every batch."""
    pre, b0 = G.uniq_workload(6000, 3000, seed=21, pre_hit=0.3, dbl=0.05, resubmit=0.01)
    batches = [b0]
    for s in range(22, 26):
        _, bs = G.uniq_workload(6000, 0, seed=s, pre_hit=0.0, dbl=0.05)
        k = 3000
        bs.refs[:36 * k] = b0.refs[36 * (s - 22) * 500:36 * ((s - 22) * 500 + k)]
        batches.append(bs)
    outs = run_both(ctx, oracle, pre, batches, cap=1 << 13)
    for g, r in outs:
        assert np.array_equal(g[0], r[0])
        assert g[1] == r[1]
    assert (outs[0][0][0] == CONFLICT).sum() > 1000


def test_uniq_device_entry_matches_host_entry(ctx, oracle):
    """chip_uniq_commit_batch_device (inputs resident in HBM) == the host entry == the oracle."""
    import torch
    from corda_amd import native
    pre, b = G.uniq_workload(30000, 40000, seed=9, pre_hit=0.02, dbl=0.02, resubmit=0.01)
    dev = torch.device("cuda", 0)
    t = ctx.uniq_open(1 << 17)
    t.rebuild(*pre)
    o = oracle.Uniq(1 << 17)
    o.preload(*pre)
    nref = int(b.tx_ref_start[-1])
    d_start = torch.from_numpy(b.tx_ref_start.view(np.int64)).to(dev)
    d_refs = torch.from_numpy(b.refs).to(dev)
    d_ids = torch.from_numpy(b.tx_ids).to(dev)
    d_call = torch.from_numpy(b.callers.view(np.int32)).to(dev)
    d_st = torch.empty(b.ntx, dtype=torch.uint8, device=dev)
    cap = nref + 1
    rec = ctypes.sizeof(native.ChipConflict)
    d_out = torch.empty(cap * rec, dtype=torch.uint8, device=dev)
    n = t.commit_batch_device(d_start, nref, d_refs, d_ids, d_call, d_st, d_out, cap)
    torch.cuda.synchronize()
    recs = native.records_from_bytes(d_out[:min(n, cap) * rec].cpu().numpy().tobytes())
    ws, wr = o.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
    assert np.array_equal(d_st.cpu().numpy(), ws)
    assert recs == wr and n == len(wr)
    assert t.size() == o.size()
    t.close()


@pytest.mark.parametrize("world", [2, 3])
def test_uniq_sharded_gpu_shards_match_oracle(ctx, oracle, world):
    """The multi-GPU protocol with `world` GPU shard tables (chip_uniq_shard_* kernels) on one
    device; the all-reduce MAX is an element-wise max here.  Two batches, pre-committed rows routed
    to their owners: statuses, records and table sizes equal the single-process oracle."""
    from corda_amd import distributed as D
    from corda_amd import native
    pre, b = G.uniq_workload(20000, 30000, seed=12, pre_hit=0.02, dbl=0.03, resubmit=0.01)
    _, b2 = G.uniq_workload(8000, 0, seed=13, pre_hit=0.0, dbl=0.03)
    b2.refs[:36 * 4000] = b.refs[:36 * 4000]
    tables = [ctx.uniq_open(1 << 14) for _ in range(world)]
    refs, tx, idx, caller = pre
    for r, rows in enumerate(D.route_rows(refs, world)):
        tables[r].rebuild(refs.reshape(-1, 36)[rows].reshape(-1).copy(), tx.reshape(-1, 32)[rows].reshape(-1).copy(),
                          idx[rows].copy(), caller[rows].copy())
    engines = [native.UniqShardEngine(t) for t in tables]
    o = oracle.Uniq(1 << 14)
    o.preload(*pre)
    for batch in (b, b2):
        st, recs, rounds = D.commit_sharded_local(engines, batch)
        ws, wr = o.commit_batch(batch.tx_ref_start, batch.refs, batch.tx_ids, batch.callers)
        assert np.array_equal(st, ws)
        assert recs == wr
        assert rounds >= 2
    assert sum(t.size() for t in tables) == o.size()
    for t in tables:
        t.close()


def test_uniq_rebuild_with_duplicate_rows_after_a_commit(ctx, oracle):
    """A rebuild whose rows repeat StateRefs, run after a commit left its per-ref scratch behind: the
    first row of each key is kept (AppendOnlyPersistentMap, first value wins), whichever lane won the
    claim; size() and the conflict records of a batch that re-spends those states equal the oracle."""
    pre, b = G.uniq_workload(8000, 6000, seed=31, pre_hit=0.02, dbl=0.03, resubmit=0.01)
    refs, tx, idx, caller = pre
    n = len(idx)
    r36, t32 = refs.reshape(-1, 36), tx.reshape(-1, 32)
    rng = np.random.Generator(np.random.PCG64(32))
    head = np.arange(0, 1500)           # repeated BEFORE their originals: the repeat wins
    tail = np.arange(1500, 3000)        # repeated AFTER their originals: the original wins
    alt_tx = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    alt_idx = rng.integers(0, 50, size=n).astype(np.uint32)
    alt_call = rng.integers(0, 7, size=n).astype(np.uint32)
    rows_r = np.concatenate([r36[head], r36, r36[tail], r36[tail]])
    rows_t = np.concatenate([alt_tx[head], t32, alt_tx[tail], t32[tail]])
    rows_i = np.concatenate([alt_idx[head], idx, alt_idx[tail], idx[tail]])
    rows_c = np.concatenate([alt_call[head], caller, alt_call[tail], caller[tail]])
    dup_pre = (np.ascontiguousarray(rows_r).reshape(-1), np.ascontiguousarray(rows_t).reshape(-1),
               np.ascontiguousarray(rows_i), np.ascontiguousarray(rows_c))
    t = ctx.uniq_open(1 << 16)
    o = oracle.Uniq(1 << 16)
    # a first commit leaves own / sid / tslot scratch over more refs than the rebuild has
    _, warm = G.uniq_workload(20000, 0, seed=33, pre_hit=0.0, dbl=0.05)
    g0 = t.commit_batch(warm.tx_ref_start, warm.refs, warm.tx_ids, warm.callers)
    r0 = o.commit_batch(warm.tx_ref_start, warm.refs, warm.tx_ids, warm.callers)
    assert np.array_equal(g0[0], r0[0])
    t.rebuild(*dup_pre)
    o.preload(*dup_pre)
    assert t.size() == o.size()
    # re-spend every rebuilt state: each conflict record names the kept row's tx / index / caller
    _, again = G.uniq_workload(3000, 0, seed=34, pre_hit=0.0, dbl=0.0)
    again.refs[:36 * 3000] = np.ascontiguousarray(r36[:3000]).reshape(-1)
    g = t.commit_batch(again.tx_ref_start, again.refs, again.tx_ids, again.callers)
    r = o.commit_batch(again.tx_ref_start, again.refs, again.tx_ids, again.callers)
    assert np.array_equal(g[0], r[0])
    assert g[1] == r[1] and len(r[1]) >= 3000
    assert t.size() == o.size()
    t.close()


def test_commit_log_restart_on_gpu(ctx, tmp_path):
    """The notary commit log rebuilt into the GPU table at open answers like a provider that never
    restarted (tests/commit_log_case.py)."""
    from commit_log_case import run
    assert run(ctx, tmp_path) > 0


def test_commit_log_failure_is_fail_stop_on_gpu(ctx, tmp_path):
    """A failed append stops the GPU-backed provider; the reopened table (rebuilt from the log)
    serves the unacknowledged batch again (tests/commit_log_case.py)."""
    from commit_log_case import run_fail_stop
    assert run_fail_stop(ctx, tmp_path) > 0


def test_uniq_consumed_states_stay_findable(ctx, oracle):
    """After a commit into a half-full table (many probe collisions among the batch's new states), every state the
    batch consumed must be found by the next batch: each of its inputs re-spent by a transaction of its own
    conflicts exactly where the oracle's does.  (The read-only lookup's insert-time claims once put two colliding
    states into one slot when a claim word read by a plain load was re-read by the compiler after its test.)"""
    pre, b0 = G.uniq_workload(5000, 1000, seed=1, pre_hit=0.05, dbl=0.05)
    nref = len(b0.refs) // 36
    rng = np.random.Generator(np.random.PCG64(3))
    probe = G.uniq_batch_from_lists([(rng.bytes(32), [bytes(b0.refs[36 * i:36 * i + 36])], 7) for i in range(nref)])
    for _ in range(4):
        outs = run_both(ctx, oracle, pre, [b0, probe], cap=1024)
        for g, r in outs:
            assert np.array_equal(g[0], r[0])
            assert g[1] == r[1]
