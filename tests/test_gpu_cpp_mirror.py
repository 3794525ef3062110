"""GPU: the C++ reference-API mirror (include/corda/verify.hpp) end to end through libcordahip —
Crypto.doVerify / TransactionSignature.verify / SignedTransaction.verifySignaturesExcept /
WireTransaction.id / PersistentUniquenessProvider.commit / commitInputStates."""
import os
import subprocess

import pytest

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
