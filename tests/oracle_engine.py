"""CPU stand-in for corda_amd.Context in host-logic tests: the oracle restatement behind the same
verify_batch / txid_batch / uniq_open methods.  TEST INFRASTRUCTURE ONLY (the product path never
falls back to it: corda_amd.crypto takes the engine from its caller)."""
import numpy as np

import oracle_bind as O


class _Table:
    def __init__(self, cap):
        self.u = O.Uniq(cap)

    def size(self):
        return self.u.size()

    def rebuild(self, refs36, tx32, idx, caller):
        self.u.preload(refs36, tx32, idx, caller)

    def commit_batch(self, tx_ref_start, refs36, tx_ids, callers, cap=None):
        return self.u.commit_batch(tx_ref_start, refs36, tx_ids, callers, cap)


class OracleEngine:
    def __init__(self, threads=8):
        self.threads = threads
        self.calls = 0

    def verify_batch(self, b, is_valid: bool = False):
        self.calls += 1
        st = O.verify_batch(b, threads=self.threads, is_valid=is_valid)
        bits = np.zeros(((len(st) + 63) // 64) * 64, dtype=np.uint64)
        bits[:len(st)] = (st == 0)
        bm = np.bitwise_or.reduce(bits.reshape(-1, 64) << np.arange(64, dtype=np.uint64), axis=1) if len(st) else bits
        return st, bm

    def txid_batch(self, tb):
        self.calls += 1
        return O.txid_batch(tb, threads=self.threads)

    def required_signers(self, q, b, status):
        self.calls += 1
        return O.required_signers(q, b, status)

    def uniq_open(self, cap):
        return _Table(cap)
