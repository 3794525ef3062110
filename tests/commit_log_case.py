"""Shared scenario for the notary commit log (CPU oracle engine and GPU engine): commit batches with
a log, reopen a fresh provider from the log, and check that it answers exactly like the provider that
never restarted (PersistentUniquenessProvider.kt:50-113 semantics across a node restart)."""
import hashlib
import os

import numpy as np

from corda_amd import crypto as C


def _h(s):
    return hashlib.sha256(s.encode()).digest()


def batches(seed=7, n_batches=4, per=200):
    rng = np.random.Generator(np.random.PCG64(seed))
    issued = [C.StateRef(_h("issue%d" % k), int(k % 3)) for k in range(600)]
    out = []
    for b in range(n_batches):
        reqs = []
        for t in range(per):
            k = int(rng.integers(1, 4))
            states = [issued[int(j)] for j in rng.integers(0, len(issued), size=k)]
            if rng.random() < 0.05 and states:
                states.append(states[0])        # repeated input inside one tx (first index wins)
            reqs.append((states, _h("tx%d.%d" % (b, t)), int(rng.integers(0, 5))))
        if b and out:                            # a few re-notarisations of earlier transactions
            reqs += out[b - 1][:5]
        out.append(reqs)
    return out


def run(engine, tmpdir):
    path = os.path.join(str(tmpdir), "notary_commit_log.bin")
    bs = batches()
    live = C.PersistentUniquenessProvider(engine, 1 << 14)
    logged = C.PersistentUniquenessProvider(engine, 1 << 14, log_path=path)
    for reqs in bs[:2]:
        assert live.commit_batch(reqs) == logged.commit_batch(reqs)
    logged.close()
    size_before = logged.size()
    # simulate a crash mid-append: a torn partial row at the end is ignored at reopen
    with open(path, "ab") as f:
        f.write(b"\x01" * 17)
    restarted = C.PersistentUniquenessProvider(engine, 1 << 14, log_path=path)
    assert restarted.size() == size_before == live.size()
    for reqs in bs[2:]:
        assert live.commit_batch(reqs) == restarted.commit_batch(reqs)
    restarted.close()
    rows = np.fromfile(path, dtype=C.COMMIT_LOG_DTYPE)
    assert len(rows) == live.size()
    assert os.path.getsize(path) % C.COMMIT_LOG_DTYPE.itemsize == 0
    return len(rows)


def run_fail_stop(engine, tmpdir):
    """An append that fails leaves the device table ahead of the log: the provider must refuse that
    batch's results and every later commit (CommitLogFailure); a reopen rebuilds the table from the
    log, so the unacknowledged batch's states are free again and a retry commits them (status 0)."""
    import pytest
    path = os.path.join(str(tmpdir), "notary_commit_log_fs.bin")
    bs = batches(seed=11, n_batches=3)
    p = C.PersistentUniquenessProvider(engine, 1 << 14, log_path=path)
    first = p.commit_batch(bs[0])
    good_rows = os.path.getsize(path)

    def broken(rows):
        raise OSError(28, "No space left on device")

    p.log.append = broken
    with pytest.raises(C.CommitLogFailure):
        p.commit_batch(bs[1])
    with pytest.raises(C.CommitLogFailure):          # fail-stop: no later commit is served
        p.commit_batch(bs[2])
    p.close()
    assert os.path.getsize(path) == good_rows
    reopened = C.PersistentUniquenessProvider(engine, 1 << 14, log_path=path)
    ref = C.PersistentUniquenessProvider(engine, 1 << 14)
    assert ref.commit_batch(bs[0]) == first
    assert reopened.commit_batch(bs[1]) == ref.commit_batch(bs[1])
    reopened.close()
    return len(first)
