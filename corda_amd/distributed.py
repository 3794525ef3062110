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


def verify_sharded(verify_fn, batch, group=None):
    """Shard `batch` by transaction over the process group, verify the local shard with
    verify_fn(sub_batch) -> status (torch uint8 tensor), and all-gather the statuses."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    ranges = tx_ranges(np.asarray(batch.msg_idx), world)
    lo, hi = ranges[rank]
    local = verify_fn(sub_batch(batch, lo, hi))
    return gather_status(local, ranges, group)
