"""Test double for the multi-GPU uniqueness protocol: a plain-Python restatement of one shard's
chip_uniq_shard_* phases (include/cordahip.h), so corda_amd.distributed.commit_sharded /
commit_sharded_local can be exercised on CPU (gloo) without a GPU.  TEST INFRASTRUCTURE ONLY.

Semantics per phase follow uniq.hip's header comment; the result must equal the single-process
oracle (oracle/uniq_ref.c: PersistentUniquenessProvider.commit + commitInputStates applied in batch
order) for any partition of the key space.
"""
import numpy as np
import torch

UND, COMMITTED, FAILED = 0, 1, 2


class RefShard:
    def __init__(self):
        self.table = {}   # 36-byte StateRef -> (consuming tx id, inputIndex, caller)

    def rebuild(self, refs36, tx32, idx, caller):
        refs36, tx32 = bytes(np.asarray(refs36, np.uint8)), bytes(np.asarray(tx32, np.uint8))
        for r in range(len(idx)):
            k = refs36[36 * r:36 * r + 36]
            if k not in self.table:
                self.table[k] = (tx32[32 * r:32 * r + 32], int(idx[r]), int(caller[r]))

    def size(self):
        return len(self.table)

    def begin(self, shard, tx_ids, callers):
        self.start = [int(x) for x in shard.ref_start]
        self.ntx = len(self.start) - 1
        raw = bytes(np.asarray(shard.refs, np.uint8))
        n = self.start[-1]
        self.keys = [raw[36 * r:36 * r + 36] for r in range(n)]
        self.pos = [int(p) for p in shard.ref_pos]
        ids = bytes(np.asarray(tx_ids, np.uint8))
        self.ids = [ids[32 * t:32 * t + 32] for t in range(self.ntx)]
        self.callers = [int(c) for c in callers]
        self.ref_tx = [t for t in range(self.ntx) for _ in range(self.start[t], self.start[t + 1])]
        self.pre = [k in self.table for k in self.keys]
        self.st = [UND] * self.ntx
        self.bcommit = {}

    def vote(self):
        bmin = {}
        for r, k in enumerate(self.keys):
            t = self.ref_tx[r]
            if self.st[t] != FAILED:
                bmin[k] = min(bmin.get(k, t), t)
        v = np.zeros(self.ntx, dtype=np.uint8)
        for t in range(self.ntx):
            if self.st[t] != UND:
                continue
            for r in range(self.start[t], self.start[t + 1]):
                if self.pre[r]:
                    v[t] = 2
                    break
                m = bmin[self.keys[r]]
                if m < t:
                    if self.st[m] == COMMITTED:
                        v[t] = 2
                        break
                    v[t] = 1
        return torch.from_numpy(v)

    def apply(self, d):
        d = d.cpu().numpy()
        und = 0
        for t in range(self.ntx):
            if self.st[t] != UND:
                continue
            if d[t] == 0:
                for r in range(self.start[t], self.start[t + 1]):
                    k = self.keys[r]
                    self.bcommit[k] = min(self.bcommit.get(k, (t, self.pos[r])), (t, self.pos[r]))
                self.st[t] = COMMITTED
            elif d[t] >= 2:
                self.st[t] = FAILED
            else:
                und += 1
        return und

    def _consumer(self, r, t):
        k = self.keys[r]
        if self.pre[r]:
            return self.table[k]
        c = self.bcommit.get(k)
        if c is None or c[0] >= t:
            return None
        return (self.ids[c[0]], c[1], self.callers[c[0]])

    def classify(self):
        v = np.zeros(self.ntx, dtype=np.uint8)
        for t in range(self.ntx):
            if self.st[t] != FAILED:
                continue
            for r in range(self.start[t], self.start[t + 1]):
                c = self._consumer(r, t)
                if c is None:
                    continue
                same = c == (self.ids[t], self.pos[r], self.callers[t])
                v[t] = max(v[t], 1) if same else 2
        return torch.from_numpy(v)

    def finish(self, d):
        d = d.cpu().numpy()
        recs = []
        for r, k in enumerate(self.keys):
            t = self.ref_tx[r]
            if self.st[t] != FAILED or k in self.keys[self.start[t]:r]:
                continue
            c = self._consumer(r, t)
            if c is not None:
                recs.append((t, self.pos[r], c[1], c[0], c[2]))
        for r, k in enumerate(self.keys):
            t = self.ref_tx[r]
            if self.st[t] == COMMITTED and k not in self.table:
                self.table[k] = (self.ids[t], self.pos[r], self.callers[t])
        status = np.array([0 if s == COMMITTED else (2 if d[t] >= 2 else 1) for t, s in enumerate(self.st)],
                          dtype=np.uint8)
        return status, recs
