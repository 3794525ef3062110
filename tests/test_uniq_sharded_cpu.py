"""CPU: the multi-GPU notary-uniqueness protocol (corda_amd.distributed: key-space routing,
ordered-commit rounds with an all-reduce MAX of per-tx votes, record merge) reproduces the
single-process oracle (PersistentUniquenessProvider.commit + commitInputStates in batch order) for
every partition of the key space.  The per-shard phases are the Python test double
tests/uniq_shard_ref.py; the GPU shard kernels are exercised by tests/test_gpu_uniq.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import cordagen as G
import golden_cases
from corda_amd import distributed as D
from uniq_shard_ref import RefShard


def _oracle_commit(oracle, pre, batches):
    o = oracle.Uniq(1 << 12)
    if pre is not None:
        o.preload(*pre)
    return [o.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers) for b in batches], o.size()


def _sharded(world, pre, batches):
    engines = [RefShard() for _ in range(world)]
    if pre is not None:
        refs, tx, idx, caller = pre
        for r, rows in enumerate(D.route_rows(refs, world)):
            engines[r].rebuild(refs.reshape(-1, 36)[rows].reshape(-1), tx.reshape(-1, 32)[rows].reshape(-1),
                               idx[rows], caller[rows])
    outs = []
    for b in batches:
        st, recs, _ = D.commit_sharded_local(engines, b)
        outs.append((st, recs))
    return outs, sum(e.size() for e in engines)


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_sharded_golden_scenarios(oracle, world):
    for case in golden_cases.uniq_cases():
        batches = [G.uniq_batch_from_lists([(bytes.fromhex(tx), [bytes.fromhex(s) for s in ins], c)
                                            for tx, ins, c in bt]) for bt in case["batches"]]
        got, gsize = _sharded(world, None, batches)
        want, osize = _oracle_commit(oracle, None, batches)
        assert gsize == osize, case["label"]
        for (gs, gr), (ws, wr), exp in zip(got, want, case["expected"]):
            assert gs.tolist() == exp, case["label"]
            assert gs.tolist() == ws.tolist(), case["label"]
            assert gr == wr, case["label"]


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_random_cfg5_shape(oracle, world):
    pre, b = G.uniq_workload(1500, 2000, seed=31, pre_hit=0.03, dbl=0.04, resubmit=0.02)
    got, gsize = _sharded(world, pre, [b])
    want, osize = _oracle_commit(oracle, pre, [b])
    assert gsize == osize
    assert np.array_equal(got[0][0], want[0][0])
    assert got[0][1] == want[0][1]
    assert (got[0][0] == 2).sum() > 0 and (got[0][0] == 1).sum() > 0


def test_state_owner_deterministic_and_balanced():
    refs = G.PRNG(3, b"own").np_bytes(36 * 20000)
    a = D.state_owner(refs, 8)
    assert np.array_equal(a, D.state_owner(refs.copy(), 8))
    counts = np.bincount(a, minlength=8)
    assert counts.min() > 0.8 * 20000 / 8 and counts.max() < 1.2 * 20000 / 8
    assert (D.state_owner(refs, 1) == 0).all()


def test_route_keeps_input_order_and_positions():
    _, b = G.uniq_workload(300, 0, seed=8, pre_hit=0.0, dbl=0.05)
    shards = D.route_uniq_batch(b.tx_ref_start, b.refs, 3)
    assert sum(s.nref for s in shards) == int(b.tx_ref_start[-1])
    refs = b.refs.reshape(-1, 36)
    for t in range(b.ntx):
        lo, hi = int(b.tx_ref_start[t]), int(b.tx_ref_start[t + 1])
        seen = []
        for s in shards:
            a, e = int(s.ref_start[t]), int(s.ref_start[t + 1])
            for j in range(a, e):
                p = int(s.ref_pos[j])
                assert s.refs.reshape(-1, 36)[j].tobytes() == refs[lo + p].tobytes()
                seen.append(p)
            assert list(s.ref_pos[a:e]) == sorted(s.ref_pos[a:e])
        assert sorted(seen) == list(range(hi - lo))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pre, b = G.uniq_workload(800, 1000, seed=19, pre_hit=0.03, dbl=0.04, resubmit=0.02)
    e = RefShard()
    refs, tx, idx, caller = pre
    rows = D.route_rows(refs, world)[rank]
    e.rebuild(refs.reshape(-1, 36)[rows].reshape(-1), tx.reshape(-1, 32)[rows].reshape(-1), idx[rows], caller[rows])
    st, recs, rounds = D.commit_sharded(e, b)
    _, b2 = G.uniq_workload(400, 0, seed=20, pre_hit=0.0, dbl=0.05)
    b2.refs[:36 * 200] = b.refs[:36 * 200]          # the second batch re-spends the first's inputs
    st2, recs2, _ = D.commit_sharded(e, b2)
    if rank == 0:
        q.put((st.tolist(), recs, st2.tolist(), recs2, rounds))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_commit_sharded_over_gloo_matches_oracle(oracle, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    st, recs, st2, recs2, rounds = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    pre, b = G.uniq_workload(800, 1000, seed=19, pre_hit=0.03, dbl=0.04, resubmit=0.02)
    _, b2 = G.uniq_workload(400, 0, seed=20, pre_hit=0.0, dbl=0.05)
    b2.refs[:36 * 200] = b.refs[:36 * 200]
    (w1, w2), _ = _oracle_commit(oracle, pre, [b, b2])
    assert st == w1[0].tolist() and recs == w1[1]
    assert st2 == w2[0].tolist() and recs2 == w2[1]
    assert rounds >= 1
