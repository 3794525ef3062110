"""Multi-GPU sharding of the verification path (one process per GPU, torch.distributed).

Signatures shard by transaction: rank r verifies a contiguous range of
transactions — a transaction never splits, so "first failing signature of a tx" stays local —
and the per-rank accept bitmaps / status bytes are all-gathered (RCCL over xGMI on the GPU box;
gloo in the CPU tests).  There is no other data-path collective.
"""
from __future__ import annotations

import numpy as np


def tx_ranges(msg_idx: np.ndarray, world: int):
    """Split signatures into `world` contiguous ranges on transaction boundaries.

    A transaction is a run of equal msg_idx (its signers share the SignableData message).
    Returns [(lo, hi)] signature ranges, balanced by signature count."""
    n = len(msg_idx)
    if n == 0:
        return [(0, 0)] * world
    starts = np.concatenate([[0], np.nonzero(np.diff(msg_idx.astype(np.int64)) != 0)[0] + 1, [n]])
    bounds = [0]
    for r in range(1, world):
        target = n * r // world
        k = int(np.searchsorted(starts, target))
        b = int(starts[min(k, len(starts) - 1)])
        bounds.append(max(b, bounds[-1]))
    bounds.append(n)
    return [(bounds[i], bounds[i + 1]) for i in range(world)]


def sub_batch(b, lo: int, hi: int):
    """View of signatures [lo, hi) sharing the key / message pools (indices stay global)."""
    class _S:
        pass
    s = _S()
    s.key_idx, s.msg_idx = b.key_idx[lo:hi], b.msg_idx[lo:hi]
    s.sig_data, s.sig_off, s.sig_len = b.sig_data, b.sig_off[lo:hi], b.sig_len[lo:hi]
    s.key_data, s.key_off, s.key_len = b.key_data, b.key_off, b.key_len
    s.msg_data, s.msg_off, s.msg_len = b.msg_data, b.msg_off, b.msg_len
    return s


def gather_status(local_status, ranges, group=None):
    """All-gather per-rank status bytes (padded to the longest shard) into the full batch order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    width = max(1, max(hi - lo for lo, hi in ranges))
    buf = torch.full((width,), 0xFF, dtype=torch.uint8, device=local_status.device)
    buf[:local_status.numel()] = local_status
    out = torch.empty(world * width, dtype=torch.uint8, device=local_status.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    parts = [out[r * width:r * width + (hi - lo)] for r, (lo, hi) in enumerate(ranges)]
    return torch.cat(parts)


def status_to_bitmap(status):
    """bit i = (status[i] == VALID), 64 signatures per word (same layout as chip_verify_batch)."""
    st = np.asarray(status)
    n = len(st)
    bits = np.zeros(((n + 63) // 64) * 64, dtype=np.uint8)
    bits[:n] = (st == 0)
    b = bits.reshape(-1, 64).astype(np.uint64)
    return np.bitwise_or.reduce(b << np.arange(64, dtype=np.uint64), axis=1).astype(np.uint64)


def verify_sharded(verify_fn, batch, group=None, msg_idx=None):
    """Shard `batch` by transaction over the process group, verify the local shard with
    verify_fn(sub_batch) -> status (torch uint8 tensor), and all-gather the statuses.  `batch` may be
    device-resident (torch tensors: the shard is a view, verified by chip_verify_batch_device); the
    transaction boundaries then come from the host copy `msg_idx`."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    ranges = tx_ranges(np.asarray(batch.msg_idx if msg_idx is None else msg_idx), world)
    lo, hi = ranges[rank]
    local = verify_fn(sub_batch(batch, lo, hi))
    return gather_status(local, ranges, group)


# ---------------------------------------------------------------------------------------
# Notary uniqueness across GPUs.  The StateRef key space is partitioned: the
# owner of a state is a hash of its key, every rank holds its slice of the commit log in its own
# HBM (chip_uniq), the host routes each input to its owner (no all-to-all), and the ordered-commit
# rounds exchange one u8 vote per transaction per round with an all-reduce MAX (RCCL over xGMI).
_MIX1 = np.uint64(0xff51afd7ed558ccd)
_MIX2 = np.uint64(0xc4ceb9fe1a85ec53)
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def state_owner(refs36, world: int) -> np.ndarray:
    """Owner rank of each 36-byte StateRef key (32-byte txhash || LE u32 index): a 64-bit mix of
    the txhash prefix and the index.  Deterministic, so every rank computes the same map."""
    r = np.ascontiguousarray(np.asarray(refs36, dtype=np.uint8)).reshape(-1, 36)
    if world == 1 or len(r) == 0:
        return np.zeros(len(r), dtype=np.int64)
    h = np.ascontiguousarray(r[:, 0:8]).view("<u8").reshape(-1).copy()
    idx = np.ascontiguousarray(r[:, 32:36]).view("<u4").reshape(-1).astype(np.uint64)
    with np.errstate(over="ignore"):
        h ^= idx * _GOLD
        h ^= h >> np.uint64(33)
        h *= _MIX1
        h ^= h >> np.uint64(33)
        h *= _MIX2
        h ^= h >> np.uint64(33)
    return (h % np.uint64(world)).astype(np.int64)


class UniqShard:
    """The inputs of a batch one rank owns, grouped by transaction in input order:
    tx t's local inputs are refs[ref_start[t]:ref_start[t+1]], ref_pos their positions in t's
    full input list (chip_uniq_shard_batch layout)."""

    def __init__(self, ref_start, refs, ref_pos):
        self.ref_start = ref_start
        self.refs = refs
        self.ref_pos = ref_pos

    @property
    def nref(self):
        return int(self.ref_start[-1])


def route_uniq_batch(tx_ref_start, refs36, world: int):
    """Split a commit batch (tx_ref_start u64[ntx+1], refs 36-byte keys) into one UniqShard per rank."""
    start = np.asarray(tx_ref_start, dtype=np.uint64)
    ntx = len(start) - 1
    nref = int(start[-1]) if ntx >= 0 else 0
    refs = np.asarray(refs36, dtype=np.uint8)[:nref * 36].reshape(nref, 36)
    counts = np.diff(start.astype(np.int64))
    ref_tx = np.repeat(np.arange(ntx, dtype=np.int64), counts)
    pos = (np.arange(nref, dtype=np.int64) - start[:-1].astype(np.int64)[ref_tx]).astype(np.uint32)
    own = state_owner(refs, world)
    shards = []
    for r in range(world):
        sel = np.nonzero(own == r)[0]
        ls = np.zeros(ntx + 1, dtype=np.uint64)
        if ntx:
            ls[1:] = np.cumsum(np.bincount(ref_tx[sel], minlength=ntx)).astype(np.uint64)
        shards.append(UniqShard(ls, np.ascontiguousarray(refs[sel]).reshape(-1), pos[sel].copy()))
    return shards


def route_rows(refs36, world: int):
    """Committed rows (e.g. AppendOnlyPersistentMap.allPersisted) -> row indices each rank owns."""
    own = state_owner(refs36, world)
    return [np.nonzero(own == r)[0] for r in range(world)]


REC_BYTES = 56   # sizeof(chip_conflict)


def gather_records(local, group=None):
    """All-gather every rank's Conflict.stateHistory records as raw chip_conflict bytes (a u8 tensor
    of n * 56 bytes, on the GPU with RCCL) — one count all-gather and one padded record all-gather,
    no pickled host objects — and merge them in (tx, input_index) order."""
    import torch
    import torch.distributed as dist
    from .native import records_from_bytes
    world = dist.get_world_size(group)
    host = dist.get_backend(group) != "nccl"
    dev = torch.device("cpu") if host else local.device
    loc = local.to(dev)
    n = torch.tensor([loc.numel() // REC_BYTES], dtype=torch.int64, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(counts, n, group=group)
    width = max(1, int(counts.max().item())) * REC_BYTES
    buf = torch.zeros(width, dtype=torch.uint8, device=dev)
    buf[:loc.numel()] = loc
    out = torch.empty(world * width, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    raw = out.cpu().numpy()
    per = [records_from_bytes(raw[r * width:r * width + int(counts[r]) * REC_BYTES].tobytes()) for r in range(world)]
    return merge_records(per)


def merge_records(per_shard):
    """Union of the shards' Conflict.stateHistory records in (tx, input_index) order."""
    out = [rec for recs in per_shard for rec in recs]
    out.sort(key=lambda rec: (rec[0], rec[1]))
    return out


def commit_sharded_local(engines, batch):
    """All shards in one process (tests, one-GPU rehearsal of the protocol): the MAX all-reduce is an
    element-wise maximum over the shards' vote tensors.  `engines[r]` owns state_owner(...) == r."""
    import torch
    shards = route_uniq_batch(batch.tx_ref_start, batch.refs, len(engines))
    for e, s in zip(engines, shards):
        e.begin(s, batch.tx_ids, batch.callers)

    def reduce_max(votes):
        d = votes[0].clone()
        for v in votes[1:]:
            d = torch.maximum(d, v.to(d.device))
        return d
    rounds = 0
    while True:
        d = reduce_max([e.vote() for e in engines])
        und = [e.apply(d.to(e.vote_buf.device) if hasattr(e, "vote_buf") else d) for e in engines]
        rounds += 1
        assert len(set(und)) == 1, "shards disagree on the undecided count"
        if und[0] == 0:
            break
    d = reduce_max([e.classify() for e in engines])
    outs = [e.finish(d.to(e.vote_buf.device) if hasattr(e, "vote_buf") else d) for e in engines]
    return outs[0][0], merge_records([o[1] for o in outs]), rounds


def commit_sharded(engine, batch, group=None, shard=None):
    """This rank's part of a multi-GPU commit: route the batch, run the ordered-commit rounds with
    one all-reduce MAX of the per-tx vote bytes per round, classify the failed transactions with one
    more, and all-gather the conflict records.  Returns (status u8[ntx], records, rounds) on every
    rank.  `shard` may be this rank's pre-uploaded shard (engine.upload) to keep inputs resident."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if shard is None:
        shard = route_uniq_batch(batch.tx_ref_start, batch.refs, world)[rank]
        engine.begin(shard, batch.tx_ids, batch.callers)
    else:
        engine.begin(shard)
    # RCCL reduces device tensors in place; a CPU process group (gloo) gets host copies
    host = dist.get_backend(group) != "nccl"

    def reduce_max(v):
        if host and getattr(v, "is_cuda", False):
            c = v.cpu()
            dist.all_reduce(c, op=dist.ReduceOp.MAX, group=group)
            v.copy_(c)
        else:
            dist.all_reduce(v, op=dist.ReduceOp.MAX, group=group)
        return v
    rounds = 0
    while True:
        v = reduce_max(engine.vote())
        rounds += 1
        if engine.apply(v) == 0:
            break
    v = reduce_max(engine.classify())
    if hasattr(engine, "finish_device"):
        st, local = engine.finish_device(v)
        status = st.cpu().numpy()
    else:   # host-side shard engines (CPU tests): the same byte records, through the same collective
        import torch
        from .native import records_to_bytes
        status, recs = engine.finish(v)
        local = torch.frombuffer(bytearray(records_to_bytes(recs)) or bytearray(1), dtype=torch.uint8)
        local = local[:len(recs) * REC_BYTES]
    return status, gather_records(local, group), rounds
