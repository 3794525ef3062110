"""GPU: the multi-GPU notary protocol (corda_amd.distributed.commit_sharded) across real processes,
each with its own libcordahip context and shard table on cuda:0, over a gloo process group (the
one-GPU rehearsal of the RCCL path; RCCL needs one GPU per rank).  Result == the oracle."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import cordagen as G

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import corda_amd
    from corda_amd import distributed as D, native
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    ctx = corda_amd.Context(0)
    pre, b = G.uniq_workload(20000, 30000, seed=41, pre_hit=0.02, dbl=0.03, resubmit=0.01)
    refs, tx, idx, caller = pre
    rows = D.route_rows(refs, world)[rank]
    t = ctx.uniq_open(1 << 16)
    t.rebuild(refs.reshape(-1, 36)[rows].reshape(-1).copy(), tx.reshape(-1, 32)[rows].reshape(-1).copy(),
              idx[rows].copy(), caller[rows].copy())
    eng = native.UniqShardEngine(t)
    st, recs, rounds = D.commit_sharded(eng, b)
    shard = D.route_uniq_batch(b.tx_ref_start, b.refs, world)[rank]
    sizes = [None] * world
    dist.all_gather_object(sizes, t.size())
    if rank == 0:
        q.put((st.tolist(), recs, rounds, sum(sizes)))
    dist.barrier()
    t.close()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_commit_sharded_processes_match_oracle(oracle, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    st, recs, rounds, size = q.get(timeout=200)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    pre, b = G.uniq_workload(20000, 30000, seed=41, pre_hit=0.02, dbl=0.03, resubmit=0.01)
    o = oracle.Uniq(1 << 16)
    o.preload(*pre)
    ws, wr = o.commit_batch(b.tx_ref_start, b.refs, b.tx_ids, b.callers)
    assert st == ws.tolist()
    assert recs == wr
    assert size == o.size()
    assert rounds >= 2
