"""CPU, world_size 2 over gloo: the multi-GPU sharding of the signature path (tx-boundary ranges,
status all-gather, bitmap layout) reproduces the single-process result.  The per-shard verify
here is the oracle (the GPU kernel is exercised by the -m gpu tests)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import cordagen as G
from corda_amd import distributed as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import oracle_bind as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = G.ed25519_batch(301, n_keys=8, corrupt=0.4, seed=44)

    def verify(sub):
        class B:
            pass
        x = B()
        for f in ("key_idx", "msg_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len",
                  "msg_data", "msg_off", "msg_len"):
            setattr(x, f, np.ascontiguousarray(getattr(sub, f)))
        x.n = len(x.key_idx)
        return torch.from_numpy(O.verify_batch(x))

    full = D.verify_sharded(verify, b)
    if rank == 0:
        q.put(full.numpy().tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_verify_matches_single_process(world):
    import oracle_bind as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    b = G.ed25519_batch(301, n_keys=8, corrupt=0.4, seed=44)
    assert got == O.verify_batch(b).tolist()


def test_tx_ranges_never_split_a_transaction():
    msg_idx = np.repeat(np.arange(1000), np.random.default_rng(1).integers(1, 5, size=1000)).astype(np.uint32)
    for world in (1, 2, 3, 8):
        rs = D.tx_ranges(msg_idx, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(msg_idx)
        for (a, b), (c, d) in zip(rs, rs[1:]):
            assert b == c
            if 0 < b < len(msg_idx):
                assert msg_idx[b - 1] != msg_idx[b]


def test_bitmap_layout():
    st = np.array([0, 1, 0, 0] + [1] * 60 + [0], dtype=np.uint8)
    bm = D.status_to_bitmap(st)
    assert bm.tolist() == [0b1101, 1]
