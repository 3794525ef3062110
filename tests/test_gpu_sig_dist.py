"""GPU: the multi-GPU signature path (corda_amd.distributed.verify_sharded) across real processes, each
with its own libcordahip context on cuda:0: the batch is device-resident, every rank verifies its
contiguous transaction range with chip_verify_batch_device, and the per-rank status bytes are
all-gathered (gloo here: the one-GPU rehearsal of the RCCL path).  Result == the oracle and the
generator labels, for an Ed25519 batch (comb + Straus keys) and a mixed ECDSA r1/k1 batch."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import cordagen as G

pytestmark = pytest.mark.gpu

FIELDS = ("key_idx", "msg_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len", "msg_data",
          "msg_off", "msg_len")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches():
    return [G.ed25519_batch(12000, n_keys=300, corrupt=0.1, seed=61),
            G.ecdsa_batch(6000, n_keys=64, corrupt=0.1, seed=62)]


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import corda_amd
    from corda_amd import distributed as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ctx = corda_amd.Context(0)

    class Dev:
        pass
    results = []
    for b in _batches():
        d = Dev()
        for f in FIELDS:
            a = np.ascontiguousarray(getattr(b, f))
            setattr(d, f, torch.from_numpy(a.view(np.int64 if a.dtype == np.uint64 else
                                                  (np.int32 if a.dtype == np.uint32 else np.uint8))).to(dev))

        def verify(sub):
            # the library's stream, ordered against torch's on both sides (torch's default stream is
            # handle 0, which the C-ABI reads as "the context's own stream")
            st = torch.empty(max(1, sub.key_idx.numel()), dtype=torch.uint8, device=dev)
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            ctx.verify_batch_device(sub, st, None, stream=s.cuda_stream)
            torch.cuda.current_stream(dev).wait_stream(s)
            return st[:sub.key_idx.numel()]
        full = D.verify_sharded(verify, d, msg_idx=b.msg_idx)
        results.append(full.cpu().numpy().tolist())
    if rank == 0:
        q.put(results)
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_verify_sharded_processes_match_oracle(oracle, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = q.get(timeout=200)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for b, got in zip(_batches(), results):
        got = np.array(got, dtype=np.uint8)
        assert len(got) == b.n
        assert np.array_equal(got, b.expected)
        assert np.array_equal(got, oracle.verify_batch(b, threads=8))
