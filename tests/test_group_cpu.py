"""CPU: the range plans of the device group (chip_group_plan_sigs / chip_group_plan_tx, host-only functions of
libcordahip) and its key-space routing (chip_group_state_owner) — what decides which member GPU verifies which
transactions and which member's table slice holds which StateRef.  The group entries themselves run on the GPU
(tests/test_gpu_group.py)."""
import os

import numpy as np
import pytest

import corda_amd
from corda_amd import distributed as D
from corda_amd import native


def tx_runs(rng, ntx, max_sigs=4):
    """msg_idx of ntx transactions with 1..max_sigs signers each (a transaction = a run of equal msg_idx)."""
    sizes = rng.integers(1, max_sigs + 1, ntx)
    return np.repeat(np.arange(ntx, dtype=np.uint32), sizes), sizes


@pytest.mark.parametrize("k", [1, 2, 3, 8])
def test_plan_sigs_never_splits_a_transaction(k):
    rng = np.random.default_rng(k)
    msg, sizes = tx_runs(rng, 5000)
    n = len(msg)
    cut = native.plan_sigs(msg, k).astype(np.int64)
    assert len(cut) == k + 1 and cut[0] == 0 and cut[-1] == n
    assert np.all(np.diff(cut) >= 0)
    for c in cut[1:-1]:
        assert c == n or c == 0 or msg[c] != msg[c - 1]          # every cut on a transaction boundary
    share = np.diff(cut)
    assert share.max() - share.min() <= 2 * int(sizes.max())     # balanced to within a transaction or two


def test_plan_sigs_small_batches_and_empty_members():
    rng = np.random.default_rng(5)
    msg, _ = tx_runs(rng, 300)
    cut = native.plan_sigs(msg, 4, min_share=16384)               # below one member's share: one member
    assert list(cut) == [0] + [len(msg)] * 4
    cut = native.plan_sigs(msg, 4, min_share=len(msg) // 2)       # two shares: two members, two empty
    assert cut[1] not in (0, len(msg)) and list(cut[2:]) == [len(msg)] * 3
    assert list(native.plan_sigs(np.zeros(0, np.uint32), 3)) == [0, 0, 0, 0]
    one_tx = np.zeros(1000, np.uint32)                           # one transaction: never split
    assert list(native.plan_sigs(one_tx, 4)) == [0, 1000, 1000, 1000, 1000]
    more = np.arange(3, dtype=np.uint32)                         # fewer transactions than members
    cut = native.plan_sigs(more, 8)
    assert cut[0] == 0 and cut[-1] == 3 and np.all(np.diff(cut.astype(np.int64)) >= 0)
    assert sorted(set(np.diff(cut.astype(np.int64)))) == [0, 1]


def test_plan_tx_balances_by_the_prefix():
    rng = np.random.default_rng(9)
    sizes = rng.integers(1, 40, 2000)                            # signatures per transaction, skewed
    sizes[:50] = 400
    prefix = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    cut = native.plan_tx(2000, prefix, 4).astype(np.int64)
    assert cut[0] == 0 and cut[-1] == 2000 and np.all(np.diff(cut) > 0)
    work = np.diff(prefix[cut].astype(np.int64))
    assert work.max() - work.min() <= 2 * 400
    assert list(native.plan_tx(10, None, 5)) == [0, 2, 4, 6, 8, 10]
    assert list(native.plan_tx(100, None, 4, min_share=1000)) == [0, 100, 100, 100, 100]


def test_state_owner_is_the_distributed_routing():
    """chip_group_state_owner (one JVM driving n GPUs) and corda_amd.distributed.state_owner (one process per GPU)
    put every StateRef on the same member."""
    rng = np.random.default_rng(3)
    refs = rng.integers(0, 256, (4000, 36), dtype=np.uint8)
    refs[:, 32:36] = 0
    refs[:, 32] = rng.integers(0, 5, 4000)
    for k in (1, 2, 3, 8):
        want = D.state_owner(refs.reshape(-1), k)
        got = [native.state_owner(refs[i].tobytes(), k) for i in range(len(refs))]
        assert list(want) == got


def test_group_init_fails_loudly_without_gpu():
    lib = corda_amd.load()
    if lib.chip_device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(native.NativeUnavailable):
        native.Group([0, 0])


def test_forkjoin_serialises_concurrent_callers(tmp_path):
    """The group's member-thread pool under 6 concurrent callers: every call's f(i) runs once per member before
    run() returns, and the first non-zero result comes back (tests/cpp/forkjoin_check.cpp)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "fj")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-pthread", "-I", os.path.join(root, "corda_amd", "csrc"),
                           "-o", exe, os.path.join(root, "tests", "cpp", "forkjoin_check.cpp")])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.split() == ["0", "0"]
