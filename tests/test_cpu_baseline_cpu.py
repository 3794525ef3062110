"""CPU: the OpenSSL baseline (tools/cordagen.c ossl_verify_many) scales with threads — each worker has its own
OSSL_LIB_CTX, so OpenSSL 3.0's global fetch / provider locks no longer serialise it (round 2's shared-context
harness ran slower at 16 threads than at one) — and agrees with the labels on canonical inputs."""
import os
import time

import numpy as np

import cordagen as G


def _rate(b, threads):
    best = 0.0
    for _ in range(2):
        t = time.perf_counter()
        ok = G.ossl_verify_batch(b, threads=threads)
        best = max(best, len(b.key_idx) / (time.perf_counter() - t))
    return best, ok


def test_openssl_baseline_scales_with_threads():
    n_cpu = len(os.sched_getaffinity(0))
    th = min(4, n_cpu)
    b = G.ed25519_batch(12000, n_keys=512, corrupt=0.10, seed=41)
    one, ok1 = _rate(b, 1)
    many, okn = _rate(b, th)
    assert np.array_equal(ok1, okn)
    # OpenSSL accepts exactly the canonical valid signatures of the batch (the i2p-only classes aside)
    assert int(ok1.sum()) <= int((b.expected == 0).sum())
    if th >= 4:
        assert many >= 2.0 * one, (one, many)
