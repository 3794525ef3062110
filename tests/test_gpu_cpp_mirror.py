"""GPU: the C++ reference-API mirror (include/corda/verify.hpp) end to end through libcordahip —
Crypto.doVerify / TransactionSignature.verify / SignedTransaction.verifySignaturesExcept /
WireTransaction.id / PersistentUniquenessProvider.commit / commitInputStates."""
import os
import subprocess

import pytest

from corda_amd import crypto as C

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_mirror_end_to_end(tmp_path):
    exe = os.path.join(ROOT, "tests", "cpp", "test_verify_mirror")
    if not os.path.exists(exe):
        exe = str(tmp_path / "mirror")
        subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"), "-o", exe,
                               os.path.join(ROOT, "tests", "cpp", "test_verify_mirror.cpp"),
                               "-L", os.path.join(ROOT, "corda_amd"), "-lcordahip", "-lcrypto",
                               "-Wl,-rpath," + os.path.join(ROOT, "corda_amd")])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


def test_cpp_commit_log_interop(ctx, tmp_path):
    """A commit log written by the Python provider reopens in the C++ provider (same rows, same
    rebuilt table); rows the C++ provider appends reopen in Python."""
    from commit_log_case import batches
    log = str(tmp_path / "commit_log.bin")
    p = C.PersistentUniquenessProvider(ctx, 1 << 14, log_path=log)
    reqs = batches()[0]
    outs = p.commit_batch(reqs)
    p.close()
    size0 = p.size()
    spent = next(st[0] for (st, _, _), (s, _) in zip(reqs, outs) if s == 0)
    exe = str(tmp_path / "commit_log_check")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"), "-o", exe,
                           os.path.join(ROOT, "tests", "cpp", "commit_log_check.cpp"),
                           "-L", os.path.join(ROOT, "corda_amd"), "-lcordahip",
                           "-Wl,-rpath," + os.path.join(ROOT, "corda_amd")])
    out = subprocess.run([exe, log, spent.txhash.hex(), str(spent.index)], check=True, capture_output=True,
                         text=True, timeout=120).stdout.split()
    assert int(out[0]) == size0
    assert out[1:3] == ["2", "0"] and int(out[3]) == size0 + 1
    q = C.PersistentUniquenessProvider(ctx, 1 << 14, log_path=log)
    assert q.size() == size0 + 1
    st, conflict = q.commit_batch([([C.StateRef(spent.txhash, 1000)], bytes(32), 3)])[0]
    assert st == 2 and conflict.state_history[0][1].id == bytes([0xA2]) + bytes(31)
    q.close()
